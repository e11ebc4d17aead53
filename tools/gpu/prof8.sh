set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-prof8}
mkdir -p $O
for sch in recvar rpc vecrec; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$sch -o run --output-format csv -- python bench.py --schema $sch --steps 20 --warmup 3 --no-cpu-baseline --msgs > $O/stats_$sch.log 2>&1 || { echo "stats failed"; tail $O/stats_$sch.log; exit 1; }
echo "== $sch"
python - <<PY
import csv
for r in csv.DictReader(open("$O/stats_$sch/run_kernel_stats.csv")):
    if "k_" in r["Name"]:
        print(f'{r["Name"][:60]:60s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1000:8.2f}us')
PY
done
