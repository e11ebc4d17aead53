set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-iter8}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for sch in recvar rpc vecrec; do
  timeout -k 10 300 python bench.py --schema $sch --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$sch.log 2>&1 || { tail $O/bench_$sch.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$sch.log').read().strip().split('\n')[-1]);print('$sch', d['value'], d['encode_ms'],d['decode_ms'],d['roofline']['frac'])"
done
OUT=${PROF_OUT:-prof9} bash tools/gpu/prof8.sh 2>&1 | grep -v "^\[" | grep "==\|k_var\|k_scan"
