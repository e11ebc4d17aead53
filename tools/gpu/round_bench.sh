# Per-schema bench lines and rocprofv3 kernel stats for the DESIGN.md
# tables (one GPU box pass).  Every GPU step has its own time limit; the
# steps are chained so the first failure ends the pass.
#   gpurun -- 'TAG=r02n bash tools/gpu/round_bench.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-round}
mkdir -p "$O"
rc=0
for s in rec128 numerics recvar rpc vecrec; do
  extra=""
  [ "$s" = recvar ] && extra="--msgs"
  [ "$s" = rpc ] && extra="--msgs --rpc"
  timeout -k 10 300 python3 -u bench.py --schema "$s" --no-cpu-baseline --no-large $extra > "$O/bench_$s.log" 2>&1 || { rc=$?; break; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$s" -o k --output-format csv -- python3 bench.py --schema "$s" --no-cpu-baseline --no-large --steps 20 --warmup 5 > "$O/prof_$s.log" 2>&1 || { rc=$?; break; }
  tail -1 "$O/bench_$s.log" | cut -c1-400
done
exit $rc
