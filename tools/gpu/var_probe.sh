# Var-kernel phase stamps + image/window size A/B + message-path bench legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-varprobe}
mkdir -p $O
VENC=3 VDEC=2 WIN=4096 timeout -k 10 200 python3 tools/tune/stamps_var.py recvar rpc > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
VARIANTS="3,2,4096,4096 3,2,8192,8192 3,2,16384,16384 3,2,32768,16384 1,1,4096,4096" timeout -k 10 300 python3 tools/tune/ab_var.py recvar rpc > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
for sch in recvar rpc rec128; do
  timeout -k 10 200 python3 bench.py --schema $sch --msgs --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_msgs_$sch.log 2>&1 || { tail -20 $O/bench_msgs_$sch.log; exit 1; }
  tail -1 $O/bench_msgs_$sch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sch', d['value'], d.get('messages'))"
done
