set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 tools/tune/ab_var.py recvar rpc 2>&1 | grep -v amdgpu.ids
B="python3 bench.py --schema recvar --steps 5 --warmup 1 --no-cpu-baseline"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmcv_$i -o run --output-format csv -- $B > gpurun_out/pmcv_$i.log 2>&1 || echo "set $i failed: $set"
done
python3 - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmcv_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_var_\w+|k_scan\w*)", r["Kernel_Name"])
        if m: agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:18s} {c:24s} {sum(v)/len(v):16.1f}")
PY
