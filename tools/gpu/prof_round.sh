# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes (separate runs,
# no tracing domains) of bench.py per schema, in the layout
# tools/prof_summary.py reads: stats_<s>/, fetch_<s>/, write_<s>/.
#   gpurun -- 'TAG=r02o bash tools/gpu/prof_round.sh'
#   python tools/prof_summary.py r02o gpurun_out/r02o
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof}
mkdir -p "$O"
B="bench.py --no-cpu-baseline --no-large --no-cold --no-host-inclusive --steps 10 --warmup 3"
for s in ${SCHEMAS:-rec128 numerics recvar rpc vecrec}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/stats_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/stats_$s.log" 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/fetch_$s.log" 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$s" -o k --output-format csv -- python3 $B --schema "$s" > "$O/write_$s.log" 2>&1 || exit $?
  echo "$s done"
done
