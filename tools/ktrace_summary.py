"""Per-launch kernel durations from a rocprofv3 kernel trace (tools/ktrace.sh):
the last chain's launches in order, with gaps."""
import csv
import glob
import sys

d = sys.argv[1]
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# the last chain: from the last 'eq' / 'pre_pointwise' launch to the end
starts = [i for i, n in enumerate(names) if "eq_kernel" in n or "pre_pointwise" in n]
i0 = starts[-1] if starts else 0
prev_end = None
tot = 0
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    prev_end = e
    tot += e - s
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mm::", "")[:40]
    print(f"{n:42s} {(e - s) / 1e3:9.1f} us  gap {gap:7.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', ''))}")
print(f"kernels {tot / 1e3:.1f} us, wall {(prev_end - int(rows[i0]['Start_Timestamp'])) / 1e3:.1f} us")
