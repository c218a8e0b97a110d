"""The kernels around each launch whose name matches a pattern, from a rocprofv3 kernel trace (csv):
queue, start relative to the match, duration -- to see where a library's work (e.g. RCCL's
collective kernel) lands relative to the timed launches beside it.

    python3 tools/trace_around.py run_kernel_trace.csv 'nccl|rccl|AllReduce' [before] [after] [max_matches]
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pat = re.compile(sys.argv[2], re.I)
before = int(sys.argv[3]) if len(sys.argv) > 3 else 4
after = int(sys.argv[4]) if len(sys.argv) > 4 else 8
maxm = int(sys.argv[5]) if len(sys.argv) > 5 else 3
hits = [i for i, r in enumerate(rows) if pat.search(r["Kernel_Name"])]
print(f"{len(hits)} matches of {sys.argv[2]!r} in {len(rows)} kernels")
qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
for h in hits[:maxm]:
    t0 = int(rows[h]["Start_Timestamp"])
    print(f"--- match at kernel {h}")
    for r in rows[max(0, h - before):h + after + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get(qkey, "?") if qkey else "?"
        print(f"  q{q:>3} {(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us  {r['Kernel_Name'][:90]}")
