# Decode timing of three schemas (tools/tune/dec_ab.py, default options)
# after a decode kernel change: vecrec, recvar, rpc.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-decq}; mkdir -p $O
for s in vecrec recvar rpc; do
  VALS="- -" timeout -k 10 120 python3 -u tools/tune/dec_ab.py $s > $O/ab_$s.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/ab_$s.log | tail -2
done
