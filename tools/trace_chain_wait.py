"""Per chain kernel type, its duration with and without the bulk queue running beside it, in a rocprofv3
--kernel-trace CSV of tools/probes/probe_chol (the second factor of the first size by default: diagonal
kernels 64 .. 127 at m = 8192).  usage: trace_chain_wait.py <kernel_trace.csv> [first_diag last_diag]"""
import collections
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
a, b = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (64, 127)
di = [i for i, x in enumerate(r) if 'chol_diag' in x['Kernel_Name']]
st, j = di[a], di[b]
seg = r[st:j + 1]
cq = seg[0]['Queue_Id']
bulk = [(int(x['Start_Timestamp']), int(x['End_Timestamp'])) for x in seg if x['Queue_Id'] != cq]
span = (max(int(x['End_Timestamp']) for x in seg) - int(seg[0]['Start_Timestamp'])) / 1000
stats = collections.defaultdict(list)
for x in seg:
    if x['Queue_Id'] != cq:
        continue
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    ov = sum(max(0, min(e, be) - max(s, bs)) for bs, be in bulk) / max(1, e - s)
    n = x['Kernel_Name'].split('(')[0].replace('void scs::', '').replace('scs::', '')[:30]
    stats[n].append(((e - s) / 1000, ov))
print(f"span of diagonal kernels {a}..{b}: {span:.1f} us")
for n, v in stats.items():
    lo = [d for d, o in v if o < 0.2]
    hi = [d for d, o in v if o >= 0.8]
    print(f"{n:32s} n={len(v):4d} total {sum(d for d, _ in v):8.1f} us avg {sum(d for d, _ in v) / len(v):6.1f} | "
          f"bulk-free n={len(lo)} avg {sum(lo) / max(1, len(lo)):6.1f} | bulk-on n={len(hi)} avg {sum(hi) / max(1, len(hi)):6.1f}")
