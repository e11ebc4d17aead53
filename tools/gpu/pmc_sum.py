"""Per-kernel, per-wave summary of a pmc_kernels.sh output directory."""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+|xdrg_spec_\w+)", r["Kernel_Name"])
        if m:
            agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted(set(k for k, _ in agg)):
    def g(c):
        v = agg.get((k, c), [])
        return sum(v) / len(v) if v else 0.0
    w = g("SQ_WAVES")
    if not w:
        continue
    wc = max(1.0, g("SQ_WAVE_CYCLES"))
    print(f"{k:16s} waves={w:8.0f} valu/w={g('SQ_INSTS_VALU')/w:7.0f} salu/w={g('SQ_INSTS_SALU')/w:6.0f} "
          f"lds/w={g('SQ_INSTS_LDS')/w:5.0f} smem/w={g('SQ_INSTS_SMEM')/w:4.0f} vmr/w={g('SQ_INSTS_VMEM_RD')/w:5.0f} "
          f"vmw/w={g('SQ_INSTS_VMEM_WR')/w:5.0f} wavecyc/w={wc/w:7.0f} wait={g('SQ_WAIT_ANY')/wc:.2f} "
          f"waitinst={g('SQ_WAIT_INST_ANY')/wc:.2f} busy={g('SQ_BUSY_CYCLES'):9.0f} "
          f"ldsconf={g('SQ_LDS_BANK_CONFLICT'):8.0f} fetchKiB={g('FETCH_SIZE'):9.0f} writeKiB={g('WRITE_SIZE'):9.0f}")
