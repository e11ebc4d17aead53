set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-ab3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_messages.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VARIANTS="3,2,-1,4096,8,0 3,2,-1,4096,8,1 3,2,-1,8192,8,0 3,2,-1,4096,4,0 3,2,-1,4096,16,0" timeout -k 10 300 python tools/tune/ab_var.py recvar rpc vecrec > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
