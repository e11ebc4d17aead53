set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pcsamp
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d $O/rpc -o run --output-format csv -- python tools/tune/run_enc.py rpc 100 > $O/rpc.log 2>&1; rc=$?
tail -5 $O/rpc.log
ls -R $O | head -20
exit $rc
