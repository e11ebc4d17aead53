"""Per-schema kernel times of tools/gpu/ix_bench.py under rocprofv3
--kernel-trace (the trace's kernels between one encode and the next)."""
import collections, csv, glob, re, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
seg, cur = [], None
for r in rows:
    n = r['Kernel_Name']
    if 'spec_encode' in n or 'k_var_encode' in n:
        cur = collections.defaultdict(list)
        seg.append(cur)
    if cur is None:
        continue
    m = re.search(r'(k_\w+|xdrg_\w+|rocclr_\w+)', n)
    cur[m.group(1) if m else n[:24]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for name, c in zip(sys.argv[2].split(','), seg):
    print(name, {k: (len(v), round(sum(v) / len(v), 1)) for k, v in c.items()
                 if any(t in k for t in ('rxs', 'ix', 'rx_', 'scan', 'decode'))})
