# All GPU parity tests, smoke, default bench, recvar/rpc benches with the
# message and RPC legs, rocprof kernel stats of the recvar + RPC benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-iter2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 python bench.py --schema recvar --steps 20 --warmup 3 --no-cpu-baseline --rpc > $O/bench_recvar.log 2>&1 || { tail $O/bench_recvar.log; exit 1; }
tail -1 $O/bench_recvar.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --schema recvar --steps 20 --warmup 3 --no-cpu-baseline --rpc > $O/stats.log 2>&1 || { echo "stats failed"; tail $O/stats.log; exit 1; }
python - <<PY
import csv
for r in csv.DictReader(open("$O/stats/run_kernel_stats.csv")):
    print(f'{r["Name"][:70]:70s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1000:8.2f}us')
PY
