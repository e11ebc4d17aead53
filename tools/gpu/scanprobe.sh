set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/scanprobe
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/scan -o run --output-format csv -- python tools/tune/scan_probe.py > $O/scan.log 2>&1 || { tail -20 $O/scan.log; exit 1; }
python - <<PY
import csv, collections, glob
f = glob.glob("$O/scan/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print(list(rows[0].keys()))
d = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"]
    if "k_scan" in k or "k_rpc" in k:
        d[(k[:40], r.get("Grid_Size_X", r.get("Grid_Size", "?")))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort(); print(k, len(v), "median ns", v[len(v)//2])
PY
