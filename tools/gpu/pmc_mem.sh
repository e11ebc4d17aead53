# Memory-pipeline counters (TA/TD/TCP/TCC, one rocprofv3 pass per set) of the
# kernels of tools/tune/run_enc.py <schema>:  SCH="recvar rpc" bash tools/gpu/pmc_mem.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-pmc_mem}
mkdir -p $O
for s in ${SCH:-recvar}; do
  i=0
  for set in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $O/$s/p$i -o run --output-format csv -- python3 tools/tune/run_enc.py $s 10 > $O/$s.p$i.log 2>&1 || { echo "pass $i failed: $set"; tail -3 $O/$s.p$i.log; exit 1; }
  done
  python3 - "$O/$s" <<'PY'
import collections, csv, glob, re, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+|xdrg_spec_\w+)", r["Kernel_Name"])
        if m:
            agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{sys.argv[1].split('/')[-1]:8s} {k:24s} {c:30s} {sum(v) / len(v):16.0f}")
PY
done
