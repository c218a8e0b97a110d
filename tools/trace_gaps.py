"""Per-kernel-name durations and the GPU idle gaps between consecutive kernels, over the last
launches of a rocprofv3 kernel trace (the timed epochs of a bench run)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
rows = rows[-last:]
dur = defaultdict(list)
gap_after = defaultdict(list)
prev_end = None
prev_name = None
total_gap = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"][:60]
    dur[name].append((e - s) / 1e3)
    if prev_end is not None:
        g = max(0, s - prev_end) / 1e3
        gap_after[prev_name].append(g)
        total_gap += g
    prev_end, prev_name = max(e, prev_end or 0), name
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} kernels over {span:.1f} us, idle {total_gap:.1f} us")
print(f"{'kernel':60s} {'n':>5s} {'avg_us':>9s} {'gap_after_avg':>13s}")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    ga = gap_after.get(k, [0])
    print(f"{k:60s} {len(dur[k]):5d} {sum(dur[k])/len(dur[k]):9.2f} {sum(ga)/len(ga):13.2f}")
