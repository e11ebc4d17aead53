# RPC header batches: GPU parity tests, smoke, bench --rpc, rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-rpc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rpc.py -x -v --timeout 120 --timeout-method thread > $O/pytest_rpc.log 2>&1 || { tail -40 $O/pytest_rpc.log; exit 1; }
tail -2 $O/pytest_rpc.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --rpc --no-cpu-baseline > $O/bench_rpc.log 2>&1 || { tail $O/bench_rpc.log; exit 1; }
tail -1 $O/bench_rpc.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --rpc --no-cpu-baseline > $O/stats.log 2>&1 || { echo "stats failed"; tail $O/stats.log; exit 1; }
grep -h "k_rpc\|k_scan" $O/stats/run_kernel_stats.csv | cut -c1-200
