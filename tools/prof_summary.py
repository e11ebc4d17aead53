"""Summarise rocprofv3 outputs of bench.py into profiles/ (committed).

    python tools/prof_summary.py <round tag> <stats dir> <fetch dir> <write dir> [records]

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats table as
produced), profiles/<tag>_pmc.json (per-kernel FETCH_SIZE / WRITE_SIZE per
launch and HBM bytes with the gfx950 correction: FETCH_SIZE reads half the
bytes of a wide coalesced stream, so hbm = 2*FETCH_SIZE + WRITE_SIZE, KiB),
and profiles/pmc_traffic.json for bench.py's roofline.traffic.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d):
    f = [os.path.join(d, x) for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main():
    tag, sd, fd, wd = sys.argv[1:5]
    records = int(sys.argv[5]) if len(sys.argv) > 5 else 1 << 20
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = [os.path.join(sd, x) for x in os.listdir(sd) if x.endswith("kernel_stats.csv")][0]
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    f, w = counters(fd), counters(wd)
    out = {}
    for (k, c), v in list(f.items()) + list(w.items()):
        e = out.setdefault(k, {"launches": len(v)})
        e[c + "_KiB_per_launch"] = sum(v) / len(v)
    for k, e in out.items():
        if "FETCH_SIZE_KiB_per_launch" in e and "WRITE_SIZE_KiB_per_launch" in e:
            e["hbm_bytes_per_launch"] = int(1024 * (2 * e["FETCH_SIZE_KiB_per_launch"]
                                                    + e["WRITE_SIZE_KiB_per_launch"]))
    json.dump(out, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
    for k, e in out.items():
        if "k_fixed_reg" in k and "hbm_bytes_per_launch" in e:
            json.dump({"kernel": "k_fixed_reg", "schema": "rec128", "records": records,
                       "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                       "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                 "passes of bench.py; 2*FETCH_SIZE+WRITE_SIZE, gfx950 correction)"},
                      open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
