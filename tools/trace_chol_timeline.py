"""Timeline of one Cholesky factor in a rocprofv3 --kernel-trace CSV of tools/probes/probe_chol (the
second m = 8192 factor by default): per window the busy fraction of the chain and bulk queues, and
the chain queue's idle gaps (what it waited behind) -- where the factor's span exceeds its busiest
queue.  usage: trace_chol_timeline.py <kernel_trace.csv> [factor index 0..3] [window us]"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
fi = int(sys.argv[2]) if len(sys.argv) > 2 else 1
win = float(sys.argv[3]) if len(sys.argv) > 3 else 250.0
di = [i for i, x in enumerate(r) if 'chol_diag' in x['Kernel_Name']]
spans = [(64, 128), (128, 192), (256, 384), (384, 512)]
a, b = spans[fi]
st, j = di[a], di[b - 1]
while j + 1 < len(r) and 'persist' not in r[j + 1]['Kernel_Name'] and 'rowsum' not in r[j + 1]['Kernel_Name']:
    j += 1
seg = r[st:j + 1]
t0 = int(seg[0]['Start_Timestamp'])
t1 = max(int(x['End_Timestamp']) for x in seg)
chain_q = seg[0]['Queue_Id']
qs = sorted(set(x['Queue_Id'] for x in seg))
bulk_q = [q for q in qs if q != chain_q and sum(1 for x in seg if x['Queue_Id'] == q) > 5]
bulk_q = bulk_q[0] if bulk_q else None


def name(x):
    return x['Kernel_Name'].split('(')[0].replace('void scs::', '').replace('scs::', '')[:40]


def iv(q):
    return [(int(x['Start_Timestamp']) - t0, int(x['End_Timestamp']) - t0, name(x)) for x in seg if x['Queue_Id'] == q]


C, B = iv(chain_q), iv(bulk_q) if bulk_q else []
span = (t1 - t0) / 1e3
print(f"factor {fi}: span {span:.2f} ms; chain q{chain_q} {len(C)} kernels, bulk q{bulk_q} {len(B)} kernels")


def busy(ivs, lo, hi):
    return sum(max(0, min(e, hi) - max(s, lo)) for s, e, _ in ivs)


w = win * 1e3
n = int((t1 - t0) // w) + 1
print("window(us)  chain%  bulk%   diag kernels started")
for k in range(n):
    lo, hi = k * w, (k + 1) * w
    nd = sum(1 for s, e, nm in C if lo <= s < hi and 'chol_diag' in nm)
    print(f"{lo / 1e3:8.0f}   {100 * busy(C, lo, hi) / w:5.0f}  {100 * busy(B, lo, hi) / w:5.0f}   {nd}")
gaps = []
for (s0, e0, n0), (s1, e1, n1) in zip(C, C[1:]):
    if s1 - e0 > 8000:   # > 8 us
        gaps.append((s1 - e0, e0, n0, n1))
tot = sum(g[0] for g in gaps)
print(f"chain idle gaps > 8 us: {len(gaps)}, {tot / 1e6:.2f} ms; all chain idle {(t1 - t0 - busy(C, 0, t1 - t0)) / 1e6:.2f} ms")
for g in sorted(gaps, reverse=True)[:12]:
    print(f"   {g[0] / 1e3:7.1f} us at {g[1] / 1e3:8.1f} us: {g[2]} -> {g[3]}")
bg = [(s1 - e0) for (s0, e0, n0), (s1, e1, n1) in zip(B, B[1:]) if s1 - e0 > 8000]
print(f"bulk idle gaps > 8 us: {len(bg)}, {sum(bg) / 1e6:.2f} ms; bulk busy {busy(B, 0, t1 - t0) / 1e6:.2f} ms")
