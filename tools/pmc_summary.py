"""Summarise tools/pmc.sh output into profiles/<tag>_pmc_summary.json (+ the
kernel-trace stats CSV) for bench.py's `traffic` / `limiter` fields.

Per kernel: launches per step, average duration (kernel trace), FETCH_SIZE /
WRITE_SIZE bytes per launch, SQ issue/wait shares and the limiter they point at, and `valu_frac`:
SQ_INSTS_VALU per launch over the duration against the chip's f64-VALU issue
ceiling (1024 SIMDs x one wave64 instruction per 4 cycles at 2.4 GHz).
Per step ("chain"): bytes = sum over kernels of bytes per launch x launches per
step.  `source_sha` (bench.source_sha) ties the file to the kernel sources it
measured: bench.py ignores a profile of other sources.

gfx950 caveats (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly 1/2 of the
bytes of a WIDE (16 B/lane) coalesced streaming read; other widths are
uncalibrated.  The chain's kernels read 2-8 B per lane, so `fetch_raw` is the
counter as it stands; `bytes_per_step` = raw FETCH + WRITE, and
`bytes_per_step_fetch_x2` applies the 16-B/lane correction to the read side (an
upper estimate).  Infinity-Cache hits are counted as fabric traffic.  SQ cycle
counters are in quad-cycles.

Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <out-tag> [steps-per-run]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK = 8.0e12
VALU_PEAK = 256 * 4 * 2.4e9 / 4  # wave64 VALU instr/s: 1024 SIMDs, one f64 FMA per 4 cycles at 2.4 GHz


# kernels whose launch name (the bench's per-kernel stats) differs from the function's
ALIAS = {"comp_rms_t": "comp_rms"}


def label(name):
    n = name.replace("void ", "").split("(")[0].split("<")[0]
    n = n.replace("mm::", "")
    n = n[: -len("_kernel")] if n.endswith("_kernel") else n
    return ALIAS.get(n, n)


def counters(d, sub):
    acc = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            acc[label(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def limiter(sq, hbm_util):
    wc = sq.get("SQ_WAVE_CYCLES") or 0.0
    if not wc:
        return None, {}
    sh = {"valu_issue": sq.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, "any_issue": sq.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
          "wait_mem_barrier": sq.get("SQ_WAIT_ANY", 0.0) / wc, "wait_dependency": sq.get("SQ_WAIT_INST_ANY", 0.0) / wc}
    if hbm_util is not None and hbm_util >= 0.5:
        return "hbm", sh
    if sh["valu_issue"] >= 0.5:
        return "valu-issue", sh
    if sh["wait_mem_barrier"] >= sh["wait_dependency"]:
        return "memory-latency (s_waitcnt / barrier)", sh
    return "dependent-issue-latency", sh


def main():
    d, tag = sys.argv[1], sys.argv[2]
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 9.0  # bench: 2 warm-up + 5 timed + 2 profiled
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    import bench
    sha = bench.source_sha()
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    dur = {}
    if stats:
        with open(stats[0]) as f, open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as g:
            g.write(f.read())
        for row in csv.DictReader(open(stats[0])):
            k = label(row["Name"])
            dur[k] = (float(row["AverageNs"]), int(row["Calls"]))
    fw = counters(d, "fetch")
    for k, v in counters(d, "write").items():
        fw[k].update(v)
    sq = counters(d, "sq")
    for k, v in counters(d, "sq2").items():
        sq[k].update(v)
    out = {"note": __doc__.split("Usage")[0].strip(), "source_sha": sha, "steps_per_run": steps, "kernels": {}}
    chain_b = chain_b2 = chain_ns = 0.0
    by_limit = defaultdict(float)
    for k in sorted(set(fw) | set(dur)):
        cs = fw.get(k, {})
        f, w = cs.get("FETCH_SIZE", []), cs.get("WRITE_SIZE", [])
        fb = 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        launches = max(len(f), len(w)) / steps if (f or w) else (dur[k][1] / steps if k in dur else 0.0)
        bpl = (fb or 0) + (wb or 0)
        avg_ns, calls = dur.get(k, (None, None))
        util = bpl / (avg_ns * 1e-9) / HBM_PEAK if avg_ns else None
        q = {c: sum(v) / len(v) for c, v in sq.get(k, {}).items() if v}
        lim, shares = limiter(q, util)
        vi = q.get("SQ_INSTS_VALU")
        valu_frac = vi / (avg_ns * 1e-9) / VALU_PEAK if vi and avg_ns else None
        out["kernels"][k] = {"launches_per_step": launches, "avg_ns": avg_ns, "fetch_raw": fb, "write": wb,
                             "bytes_per_launch": bpl, "bytes_per_launch_fetch_x2": 2 * (fb or 0) + (wb or 0),
                             "hbm_util": util, "valu_frac": valu_frac, "limiter": lim, "sq_shares": shares, "sq": q}
        chain_b += bpl * launches
        chain_b2 += (2 * (fb or 0) + (wb or 0)) * launches
        if avg_ns and lim:
            by_limit[lim] += avg_ns * launches
            chain_ns += avg_ns * launches
    dom = max(by_limit, key=by_limit.get) if by_limit else None
    out["chain"] = {"bytes_per_step": chain_b, "bytes_per_step_fetch_x2": chain_b2, "kernel_ns_per_step": chain_ns,
                    "limiter": dom, "time_share_by_limiter": {k: v / chain_ns for k, v in by_limit.items()} if chain_ns
                    else {}}
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as g:
        json.dump(out, g, indent=1)
    print(json.dumps({k: {"ns": v["avg_ns"], "MB": round(v["bytes_per_launch"] / 1e6, 1), "lim": v["limiter"],
                          "valu_issue": round(v["sq_shares"].get("valu_issue", 0), 3),
                          "valu_frac": v["valu_frac"] and round(v["valu_frac"], 3)} for k, v in out["kernels"].items()},
                     indent=0))
    print(json.dumps(out["chain"]))


if __name__ == "__main__":
    main()
