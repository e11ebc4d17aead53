set -o pipefail
mkdir -p gpurun_out/r01b
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01b/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01b/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/r01b/bench_default.log 2>&1 &&
for s in recvar rpc vecrec numerics; do timeout -k 10 120 python bench.py --schema $s --no-cpu-baseline > gpurun_out/r01b/bench_$s.log 2>&1 || exit 1; done
