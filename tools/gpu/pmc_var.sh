set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --schema ${SCH:-recvar} --steps 5 --warmup 1 --no-cpu-baseline"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/pmc_${SCH:-recvar}_$i -o run --output-format csv -- $B > gpurun_out/pmc_${SCH:-recvar}_$i.log 2>&1 || echo "set $i failed: $set"
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_recvar_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_var" in k or "k_scan" in k or "k_ix" in k:
            agg[(k.split("(")[0].split("::")[-1], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:18s} {c:24s} {sum(v)/len(v):16.1f}")
PY
