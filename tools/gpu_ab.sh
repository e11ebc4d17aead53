# A/B of var kernels (bit-exact cross-check inside) + phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tune/ab_var.py recvar rpc && \
timeout -k 10 200 python3 tools/tune/stamps_var.py recvar rpc
