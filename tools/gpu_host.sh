# Host-inclusive (pinned H2D -> kernel -> D2H) and cold-cache rates.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for sch in rec128 numerics; do
  timeout -k 10 300 python3 bench.py --schema $sch --steps 20 --warmup 5 --no-cpu-baseline --host-inclusive --cold > gpurun_out/bench_host_$sch.log 2>&1 || { tail gpurun_out/bench_host_$sch.log; exit 1; }
  tail -1 gpurun_out/bench_host_$sch.log
done
