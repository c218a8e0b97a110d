"""Summarise the Cholesky factors in a rocprofv3 --kernel-trace CSV of tools/probes/probe_chol (two factors
at m = 8192, then two at m = 16384, each after its sizes' 64 stand-alone diagonal launches): per kernel and
queue the launches, total and mean duration, each queue's busy time and the factor's span.
usage: trace_chol_factor.py <kernel_trace.csv>"""
import collections
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
di = [i for i, x in enumerate(r) if 'chol_diag' in x['Kernel_Name']]
# probe order: 64 alone (8192), 2 x 64 in factors, 64 alone (16384), 2 x 128 in factors
for (a, b), n in zip([(64, 128), (128, 192), (256, 384), (384, 512)], [8192, 8192, 16384, 16384]):
    if b > len(di):
        break
    st, j = di[a], di[b - 1]
    while j + 1 < len(r) and 'persist' not in r[j + 1]['Kernel_Name'] and 'rowsum' not in r[j + 1]['Kernel_Name']:
        j += 1
    seg = r[st:j + 1]
    t0 = int(seg[0]['Start_Timestamp'])
    t1 = max(int(x['End_Timestamp']) for x in seg)
    print(f"m = {n}: factor span {(t1 - t0) / 1e6:.2f} ms, {len(seg)} kernels")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for x in seg:
        k = x['Kernel_Name'].split('(')[0].replace('void scs::', '').replace('scs::', '')[:48] + ' q' + x['Queue_Id']
        agg[k][0] += 1
        agg[k][1] += (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:9]:
        print(f"   {k:54s} {v[0]:5d} {v[1] / 1e3:8.2f} ms {v[1] / v[0]:7.1f} us")
    for q in sorted(set(x['Queue_Id'] for x in seg)):
        iv = sorted((int(x['Start_Timestamp']), int(x['End_Timestamp'])) for x in seg if x['Queue_Id'] == q)
        busy, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"   queue {q} busy {busy / 1e6:.2f} ms")
