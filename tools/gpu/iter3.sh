# GPU parity (all), numerics bench (group path) + rocprof stats, headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-iter3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --schema numerics --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_numerics.log 2>&1 || { tail $O/bench_numerics.log; exit 1; }
tail -1 $O/bench_numerics.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --schema numerics --steps 20 --warmup 3 --no-cpu-baseline > $O/stats.log 2>&1 || { echo "stats failed"; tail $O/stats.log; exit 1; }
python - <<PY
import csv
for r in csv.DictReader(open("$O/stats/run_kernel_stats.csv")):
    if "k_" in r["Name"]:
        print(f'{r["Name"][:70]:70s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1000:8.2f}us')
PY
