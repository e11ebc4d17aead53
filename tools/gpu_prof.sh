# Parity tests, default bench, per-config benches, rocprofv3 stats + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
for sch in numerics recvar rpc; do
  timeout -k 10 300 python3 bench.py --schema $sch --steps 20 --warmup 3 > gpurun_out/bench_$sch.log 2>&1 || { tail gpurun_out/bench_$sch.log; exit 1; }
  tail -1 gpurun_out/bench_$sch.log
done
timeout -k 10 300 python3 bench.py --n 16777216 --steps 10 --warmup 3 --no-cpu-baseline --cold > gpurun_out/bench_16m.log 2>&1 || { tail gpurun_out/bench_16m.log; exit 1; }
tail -1 gpurun_out/bench_16m.log
B="python3 bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- $B > gpurun_out/prof_stats.log 2>&1 || { echo "stats failed"; tail gpurun_out/prof_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- $B --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 || { echo "fetch failed"; tail gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- $B --no-cpu-baseline > gpurun_out/prof_write.log 2>&1 || { echo "write failed"; tail gpurun_out/prof_write.log; exit 1; }
tail -1 gpurun_out/prof_stats.log
