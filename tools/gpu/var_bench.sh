# Var-schema benches (recvar, rpc, vecrec) and their kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-var}
mkdir -p "$O"
for s in ${SCHEMAS:-recvar rpc vecrec}; do
  timeout -k 10 300 python3 -u bench.py --schema $s --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_$s.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$s" -o run --output-format csv -- python3 bench.py --schema $s --no-cpu-baseline --steps 20 > "$O/prof_$s.log" 2>&1 || exit 1
done
python3 tools/gpu/kstats.py "$O" > "$O/summary.txt" 2>&1
cat "$O/summary.txt"
