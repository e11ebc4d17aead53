# Full round check: GPU parity tests, smoke, default bench, per-schema benches
# with the message leg, then rocprofv3 stats + FETCH/WRITE PMC passes per schema.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-full}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
for sch in numerics recvar rpc vecrec; do
  timeout -k 10 300 python bench.py --schema $sch --steps 20 --warmup 3 --msgs --no-cpu-baseline > $O/bench_$sch.log 2>&1 || { tail $O/bench_$sch.log; exit 1; }
  tail -1 $O/bench_$sch.log
done
[ -n "$NO_PROF" ] || PROF_TAG=${OUT_TAG:-full} bash tools/gpu/r01_prof.sh
