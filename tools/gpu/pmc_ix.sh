# SQ counters of the speculative record index walk (xdrg_spec_rxs_walk).
#   gpurun -- 'SCH=recvar bash tools/gpu/pmc_ix.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_ix_${SCH:-recvar}
mkdir -p $O
S=${SCH:-recvar}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_BUSY_CYCLES --kernel-include-regex "rxs_walk" -d $O/p1 -o run --output-format csv -- python3 tools/gpu/ix_bench.py $S > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "rxs_walk" -d $O/p2 -o run --output-format csv -- python3 tools/gpu/ix_bench.py $S > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 - <<PY
import csv, glob, collections
for pd in ("p1", "p2"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % pd, recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(pd, k, round(sum(v) / len(v)))
PY
