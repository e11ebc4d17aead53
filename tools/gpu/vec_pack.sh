# Packed element areas: the GPU test suite, the vecrec bench line, and the
# vecrec decode's HBM writes/fetches (tools/tune/vec_write.py under
# rocprofv3 --pmc, one counter set per pass) plus its kernel stats.
#   gpurun -- 'TAG=r03p bash tools/gpu/vec_pack.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vpack}
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  && timeout -k 10 240 python3 -u bench.py --schema vecrec --no-cpu-baseline --steps 30 --warmup 5 > "$O/bench_vecrec.log" 2>&1 \
  && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$O/w" -o run --output-format csv -- python3 tools/tune/vec_write.py > "$O/w.log" 2>&1 \
  && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$O/f" -o run --output-format csv -- python3 tools/tune/vec_write.py > "$O/f.log" 2>&1 \
  && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/k" -o run --output-format csv -- python3 tools/tune/vec_write.py > "$O/k.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"
grep '^{' "$O/bench_vecrec.log" | tail -1
exit $rc
