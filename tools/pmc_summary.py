"""Summarise tools/pmc.sh output into profiles/: per-kernel kernel-trace stats and
per-launch HBM traffic from FETCH_SIZE / WRITE_SIZE (KB counters).

gfx950 caveat (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly 1/2 of the
bytes of a WIDE (16 B/lane) coalesced streaming read; other access widths are
uncalibrated.  The chain's kernels read 2-8 B per lane, so the raw counters are
reported as they are (`fetch_raw`, `write`) and `bytes_per_launch` = raw FETCH +
WRITE; `bytes_per_launch_fetch_x2` is the upper estimate with the 16-B/lane
correction applied to the read side.

Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def label(name):
    n = name.replace("void ", "").split("(")[0].split("<")[0]
    n = n.replace("mm::", "")
    return n[: -len("_kernel")] if n.endswith("_kernel") else n


def main():
    d, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as f, open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as g:
            g.write(f.read())
    acc = defaultdict(lambda: defaultdict(list))
    for sub in ("fetch", "write"):
        for p in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(p)):
                acc[label(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"note": __doc__.split("Usage")[0].strip(), "kernels": {}}
    for k, cs in acc.items():
        f = cs.get("FETCH_SIZE", [])
        w = cs.get("WRITE_SIZE", [])
        fb = 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out["kernels"][k] = {"launches_profiled": max(len(f), len(w)), "fetch_raw": fb, "write": wb,
                             "bytes_per_launch": (fb or 0) + (wb or 0),
                             "bytes_per_launch_fetch_x2": 2 * (fb or 0) + (wb or 0)}
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as g:
        json.dump(out, g, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main()
