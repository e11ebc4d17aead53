set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab2
mkdir -p $O
VARIANTS="3,2,4096,4096 3,2,0,4096 3,2,2048,4096 3,2,8192,8192 3,2,16384,2048 2,2,4096,16384" timeout -k 10 300 python tools/tune/ab_var.py recvar rpc vecrec > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/scan -o run --output-format csv -- python tools/tune/scan_probe.py > $O/scan.log 2>&1 || { tail -20 $O/scan.log; exit 1; }
python - <<PY
import csv
rows = list(csv.DictReader(open("$O/scan/run_kernel_trace.csv")))
import collections
d = collections.defaultdict(list)
for r in rows:
    if "k_scan" in r["Kernel_Name"] or "k_rpc" in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:40], r.get("Grid_Size_X") or r.get("Grid_Size"))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort(); print(k, len(v), "median ns", v[len(v)//2])
PY
