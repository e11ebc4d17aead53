# GPU: message-framing parity tests, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-msgs}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_messages.py -x -v --timeout 120 --timeout-method thread > $O/pytest_msgs.log 2>&1 || { tail -40 $O/pytest_msgs.log; exit 1; }
tail -3 $O/pytest_msgs.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
