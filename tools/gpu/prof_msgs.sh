# Per-kernel stats of the message path + encode A/B after the copy-loop change.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-profmsgs}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 tools/tune/run_msgs.py recvar rpc > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/${OUT_TAG:-profmsgs}/stats/run_kernel_stats.csv".replace("${OUT_TAG:-profmsgs}", __import__("os").environ.get("OUT_TAG", "profmsgs")))[0]
for r in csv.DictReader(open(f)):
    print(f'{r["Name"][:60]:60s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1000:8.2f}us')
PY
VENC=3 VDEC=2 WIN=4096 timeout -k 10 200 python3 tools/tune/stamps_var.py recvar rpc > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
VARIANTS="3,2,4096,4096 3,2,8192,8192" timeout -k 10 300 python3 tools/tune/ab_var.py recvar rpc > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
