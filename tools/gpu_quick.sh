# GPU parity suite + smoke + var-schema benches (quick iteration loop).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -4 gpurun_out/smoke.log
for sch in ${SCHEMAS:-recvar rpc}; do
  timeout -k 10 300 python3 bench.py --schema $sch --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$sch.log 2>&1 || { tail gpurun_out/bench_$sch.log; exit 1; }
  tail -1 gpurun_out/bench_$sch.log
done
