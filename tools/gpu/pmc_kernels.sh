# PMC counter passes (one rocprofv3 run per pass) over a command; per-kernel
# means per launch.   CMD="python3 tools/tune/run_msgs.py recvar" bash tools/gpu/pmc_kernels.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-pmck}
mkdir -p $O
CMD=${CMD:-python3 tools/tune/run_msgs.py recvar}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- $CMD > $O/p$i.log 2>&1 || echo "set $i failed: $set"
done
python3 tools/gpu/pmc_sum.py "$O"; exit 0
python3 - "$O" <<'PY'
import csv, glob, collections, re, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+|xdrg_spec_\w+)", r["Kernel_Name"])
        if m:
            agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:18s} {c:26s} {sum(v)/len(v):16.1f}")
PY
