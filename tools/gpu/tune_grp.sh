set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tune_grp
mkdir -p $O
timeout -k 10 300 python tools/tune/tune_grp.py > $O/grp.log 2>&1 || { tail -20 $O/grp.log; exit 1; }
grep -v amdgpu.ids $O/grp.log | head -12
VENC=3 VDEC=2 timeout -k 10 200 python tools/tune/stamps_var.py recvar rpc > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
