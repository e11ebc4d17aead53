# rocprofv3 kernel stats + FETCH/WRITE PMC passes of bench.py for every schema.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_${PROF_TAG:-r01b}
mkdir -p $O
for sch in ${SCHEMAS:-rec128 numerics recvar rpc vecrec}; do
  B="python3 bench.py --schema $sch --steps 20 --warmup 3 --no-cpu-baseline"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats_$sch -o run --output-format csv -- $B > $O/stats_$sch.log 2>&1 || { echo "stats $sch failed"; tail $O/stats_$sch.log; exit 1; }
  tail -1 $O/stats_$sch.log
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$sch -o run --output-format csv -- $B > $O/fetch_$sch.log 2>&1 || { echo "fetch $sch failed"; tail $O/fetch_$sch.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_$sch -o run --output-format csv -- $B > $O/write_$sch.log 2>&1 || { echo "write $sch failed"; tail $O/write_$sch.log; exit 1; }
done
