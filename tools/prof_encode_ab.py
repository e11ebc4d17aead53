"""Per-schema kernel times and HBM bytes of the encode A/B under rocprofv3
(tools/gpu/r04z.sh: tools/tune/stream_ab.py recvar rpc, VARIANTS="two_pass
walk_first", one process).  The schemas run one after the other, so a
kernel's launches split at the first launch of the second schema's size
pass (recvar: k_size_linear, rpc: xdrg_spec_size).  HBM bytes per launch =
2 * FETCH_SIZE + WRITE_SIZE (KiB; MI355X_MICROARCH.md gfx950 correction).

    python tools/prof_encode_ab.py gpurun_out/r04z > profiles/r04z/encode_ab.json
"""
import collections
import csv
import json
import re
import sys


def short(k):
    m = re.search(r"(k_\w+|xdrg_spec_\w+)", k)
    return m.group(1) if m else k[:40]


def schema_of(rows, key):
    """recvar until the first rpc size pass (xdrg_spec_size), then rpc."""
    out, cur = [], "recvar"
    for r in sorted(rows, key=lambda r: int(r[key])):
        if short(r["Kernel_Name"]) == "xdrg_spec_size":
            cur = "rpc"
        out.append((cur, r))
    return out


d = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(dict))
tr = list(csv.DictReader(open(f"{d}/stats/k_kernel_trace.csv")))
acc = collections.defaultdict(list)
for s, r in schema_of(tr, "Start_Timestamp"):
    acc[(s, short(r["Kernel_Name"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (s, k), v in acc.items():
    if k.startswith(("k_size", "k_scan", "xdrg_spec_size", "xdrg_spec_encode")):
        res[s][k]["launches"] = len(v)
        res[s][k]["mean_us"] = round(sum(v) / len(v), 2)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [r for r in csv.DictReader(open(f"{d}/{c.split('_')[0].lower()}/k_counter_collection.csv"))]
    a = collections.defaultdict(list)
    for s, r in schema_of(rows, "Start_Timestamp"):
        a[(s, short(r["Kernel_Name"]))].append(float(r["Counter_Value"]))
    for (s, k), v in a.items():
        if k in res[s]:
            res[s][k][c + "_KiB"] = round(sum(v) / len(v), 1)
for s in res:
    for k, e in res[s].items():
        if "FETCH_SIZE_KiB" in e and "WRITE_SIZE_KiB" in e:
            e["hbm_MB"] = round(1024 * (2 * e["FETCH_SIZE_KiB"] + e["WRITE_SIZE_KiB"]) / 1e6, 1)
json.dump(res, sys.stdout, indent=1, sort_keys=True)
print()
