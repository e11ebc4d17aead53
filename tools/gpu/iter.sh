# Iteration: GPU parity (messages + core), then per-kernel stats, stamps, A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-iter}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
OUT_TAG=${OUT_TAG:-iter}/prof bash tools/gpu/prof_msgs.sh
