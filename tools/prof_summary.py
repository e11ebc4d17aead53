"""Summarise rocprofv3 outputs of bench.py into profiles/ (committed).

    python tools/prof_summary.py <round tag> <prof dir> [schemas...]

<prof dir> is what tools/gpu/prof_round.sh leaves: stats_<schema>/,
fetch_<schema>/, write_<schema>/ per schema.  Writes, per schema,
profiles/<tag>_<schema>_kernel_stats.csv (the rocprofv3 --stats table as
produced) and one profiles/<tag>_pmc.json with per-kernel FETCH_SIZE /
WRITE_SIZE per launch and HBM bytes with the gfx950 correction
(MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half the bytes of a wide
coalesced stream, so hbm = 2*FETCH_SIZE + WRITE_SIZE; both in KiB), plus
profiles/pmc_traffic.json, the per-(schema, kernel) traffic table bench.py
reads for roofline.traffic.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d):
    """{(kernel, counter): [value per launch]} over the launches of each
    kernel at its largest grid: a frame walk's main pass, not the deep
    passes launched after it on a few workgroups (their counts would pull
    the mean per launch down by the launches per step)."""
    f = [os.path.join(r, x) for r, _, fs in os.walk(d) for x in fs if x.endswith("counter_collection.csv")][0]
    rows = list(csv.DictReader(open(f)))
    grid = collections.defaultdict(int)
    for r in rows:
        grid[r["Kernel_Name"]] = max(grid[r["Kernel_Name"]], int(r["Grid_Size"]))
    agg = collections.defaultdict(list)
    for r in rows:
        if int(r["Grid_Size"]) == grid[r["Kernel_Name"]]:
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def short(kname):
    m = re.search(r"(k_\w+|xdrg_spec_\w+)", kname)
    return m.group(1) if m else kname.split("(")[0][:60]


def main():
    tag, pd = sys.argv[1:3]
    schemas = sys.argv[3:] or ["rec128", "numerics", "recvar", "rpc", "vecrec"]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    allpmc, traffic = {}, {}
    for sch in schemas:
        sd = os.path.join(pd, f"stats_{sch}")
        stats = [os.path.join(r, x) for r, _, fs in os.walk(sd) for x in fs if x.endswith("kernel_stats.csv")][0]
        shutil.copy(stats, os.path.join(prof, f"{tag}_{sch}_kernel_stats.csv"))
        f, w = counters(os.path.join(pd, f"fetch_{sch}")), counters(os.path.join(pd, f"write_{sch}"))
        out = {}
        for (k, c), v in list(f.items()) + list(w.items()):
            if not short(k).startswith(("k_", "xdrg_spec_")):
                continue  # torch / runtime kernels of the bench's own checks
            e = out.setdefault(short(k), {"launches": len(v)})
            e[c + "_KiB_per_launch"] = round(sum(v) / len(v), 1)
        for k, e in out.items():
            if "FETCH_SIZE_KiB_per_launch" in e and "WRITE_SIZE_KiB_per_launch" in e:
                e["hbm_bytes_per_launch"] = int(1024 * (2 * e["FETCH_SIZE_KiB_per_launch"]
                                                        + e["WRITE_SIZE_KiB_per_launch"]))
                traffic[f"{sch}:{k}"] = e["hbm_bytes_per_launch"]
        allpmc[sch] = out
    json.dump(allpmc, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
    # merged into the table: the schemas not profiled here keep their rows
    tp = os.path.join(prof, "pmc_traffic.json")
    old = json.load(open(tp)) if os.path.exists(tp) else {}
    rows = {k: v for k, v in old.get("hbm_bytes_per_launch", {}).items() if k.split(":")[0] not in schemas}
    rows.update(traffic)
    srcs = {k: v for k, v in old.get("sources", {}).items() if k not in schemas}
    srcs.update({s: f"profiles/{tag}_pmc.json" for s in schemas})
    json.dump({"records": 1 << 20,
               "hbm_bytes_per_launch": dict(sorted(rows.items())),
               "sources": dict(sorted(srcs.items())),
               "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --schema <s> "
                         "(per schema: sources); 2*FETCH_SIZE+WRITE_SIZE, gfx950 correction"},
              open(tp, "w"), indent=1)
    print(json.dumps(allpmc, indent=1)[:4000])


if __name__ == "__main__":
    main()
