# Var-path check + timing after a kernel change: GPU parity tests of the var
# schemas, then bench lines (no CPU baseline) for recvar / rpc / vecrec.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-varq}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_codegen.py tests/test_gpu_parity.py tests/test_gpu_messages.py tests/test_containers.py tests/test_record_index.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for s in ${SCH:-recvar rpc vecrec}; do
  timeout -k 10 180 python -u bench.py --schema $s --no-cpu-baseline --no-large --steps 30 --warmup 5 > $O/bench_$s.log 2>&1 || { tail -5 $O/bench_$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_$s.log') if l.startswith('{')][-1]); print('$s', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'frac', d['roofline']['frac'])"
done
