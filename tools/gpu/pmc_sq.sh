# SQ instruction mix / wait counters of the var encode + decode kernels (rpc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_sq
mkdir -p $O
S=${SCH:-rpc}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "k_var" -d $O/p1 -o run --output-format csv -- python tools/tune/run_enc.py $S 20 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM --kernel-include-regex "k_var" -d $O/p2 -o run --output-format csv -- python tools/tune/run_enc.py $S 20 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python - <<PY
import csv, glob, collections
for pd in ("p1", "p2"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % pd, recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        import re; m = re.search(r"(k_\w+)<[^>]*>", r["Kernel_Name"]); agg[(m.group(0) if m else r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(pd, k[0], k[1], round(sum(v) / len(v)))
PY
