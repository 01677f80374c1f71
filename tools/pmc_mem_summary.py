"""Per-launch memory-pipeline counters (TA / TCP / TD passes of tools/pmc_mem.sh).
Usage: python tools/pmc_mem_summary.py gpurun_out/prof_<tag> > profiles/<round>_<w>_mem_counters.json"""
import collections
import csv
import json
import os
import sys


def main(d):
    out = collections.defaultdict(dict)
    for pas in sorted(os.listdir(d)):
        path = os.path.join(d, pas, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mm::", "").split("<")[0]
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r["Dispatch_Id"])
        for name, counters in agg.items():
            n = len(disp[name])
            out[name]["launches_profiled"] = n
            for c, v in counters.items():
                out[name][c + "_per_launch"] = v / n
    json.dump({"note": "rocprofv3 --pmc passes of tools/pmc_mem.sh, values summed over the device "
                       "and divided by the kernel's profiled dispatches", "kernels": out}, sys.stdout, indent=1,
              sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
