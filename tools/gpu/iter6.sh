set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu/scanprobe.sh > $O/scanprobe.log 2>&1 || { tail $O/scanprobe.log; exit 1; }
for sch in recvar rpc vecrec numerics; do
  timeout -k 10 300 python bench.py --schema $sch --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$sch.log 2>&1 || { tail $O/bench_$sch.log; exit 1; }
  tail -1 $O/bench_$sch.log | cut -c1-120
  python -c "import json;d=json.loads(open('$O/bench_$sch.log').read().strip().split('\n')[-1]);print(d['encode_ms'],d['decode_ms'],d['roofline'])"
done
