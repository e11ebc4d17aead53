# Round-end measurement: GPU parity, smoke, headline bench (with CPU baseline,
# message and RPC legs), per-schema benches, cache-proof and host-inclusive
# runs, then rocprofv3 stats + FETCH/WRITE PMC passes for every schema.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r01z}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-160
timeout -k 10 300 python bench.py --no-cpu-baseline --rpc --msgs --cold --host-inclusive --steps 20 --warmup 3 > $O/bench_legs.log 2>&1 || { tail $O/bench_legs.log; exit 1; }
for sch in numerics recvar rpc vecrec; do
  timeout -k 10 300 python bench.py --schema $sch --steps 20 --warmup 3 --msgs > $O/bench_$sch.log 2>&1 || { tail $O/bench_$sch.log; exit 1; }
  tail -1 $O/bench_$sch.log | cut -c1-120
done
timeout -k 10 300 python bench.py --n 16777216 --steps 10 --warmup 3 --no-cpu-baseline --cold > $O/bench_16m.log 2>&1 || { tail $O/bench_16m.log; exit 1; }
tail -1 $O/bench_16m.log | cut -c1-120
[ -n "$NO_PROF" ] || PROF_TAG=$T bash tools/gpu/r01_prof.sh
