set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu/scanprobe.sh || exit 1
VARIANTS="3,2,4096,4096,16 3,2,4096,4096,8 3,2,4096,4096,4 3,2,0,4096,8 3,2,0,4096,4 3,2,8192,8192,8 3,2,2048,4096,4" timeout -k 10 300 python tools/tune/ab_var.py recvar rpc vecrec > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
