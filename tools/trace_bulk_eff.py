"""Per-launch efficiency of the Cholesky's bulk trailing updates (C12b) in a rocprofv3 --kernel-trace
CSV of tools/probes/probe_chol run at ONE size (PROBE_SIZES=m): the first factor after the 64
stand-alone diagonal launches; its gram_sia_kernel<1, 2, true, ...> launches on the bulk queue, in
order, are C12b of outer steps t = 0, 1, ... (outer block OB): tiles = nc(nc+1)/2 - OB(2OB+1) with
nc = nblk - OB(t+1), 2 * 128 * 128 * (OB * 128) flop each.
usage: trace_bulk_eff.py <kernel_trace.csv> <m> [OB]"""
import collections
import csv
import sys

PEAK = 78.6e12
r = list(csv.DictReader(open(sys.argv[1])))
m = int(sys.argv[2])
ob = int(sys.argv[3]) if len(sys.argv) > 3 else 8
nblk = m // 128
r.sort(key=lambda x: int(x['Start_Timestamp']))
di = [i for i, x in enumerate(r) if 'chol_diag' in x['Kernel_Name']]
st, j = di[64], di[64 + nblk - 1]
while j + 1 < len(r) and 'persist' not in r[j + 1]['Kernel_Name'] and 'rowsum' not in r[j + 1]['Kernel_Name']:
    j += 1
seg = r[st:j + 1]
t0 = int(seg[0]['Start_Timestamp'])
t1 = max(int(x['End_Timestamp']) for x in seg)
span = (t1 - t0) / 1e9
print(f"m = {m}: factor span {span * 1e3:.2f} ms ({m ** 3 / 3 / span / 1e12:.1f} TF/s on m^3/3), {len(seg)} kernels")
agg = collections.defaultdict(lambda: [0, 0.0])
for x in seg:
    k = x['Kernel_Name'].split('(')[0].replace('void scs::', '').replace('scs::', '')[:48] + ' q' + x['Queue_Id']
    agg[k][0] += 1
    agg[k][1] += (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:10]:
    print(f"   {k:54s} {v[0]:5d} {v[1] / 1e3:9.2f} ms {v[1] / v[0]:8.1f} us")
bulk = [x for x in seg if 'gram_sia_kernel<1, 2, true' in x['Kernel_Name'].replace('void scs::', '').replace('scs::', '')]
qs = collections.Counter(x['Queue_Id'] for x in bulk)
q = qs.most_common(1)[0][0]
bulk = [x for x in bulk if x['Queue_Id'] == q]
tot_f, tot_t = 0.0, 0.0
print(f"C12b launches on queue {q}: {len(bulk)}")
for t, x in enumerate(bulk):
    nc = nblk - ob * (t + 1)
    tiles = nc * (nc + 1) // 2 - ob * (2 * ob + 1)
    if tiles <= 0:
        break
    f = tiles * 2.0 * 128 * 128 * ob * 128
    d = (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e9
    tot_f += f
    tot_t += d
    if t < 4 or t % 8 == 0:
        print(f"   t = {t:3d}: {tiles:7d} tiles {d * 1e3:8.3f} ms {f / d / 1e12:6.1f} TF/s ({f / d / PEAK:.3f})")
print(f"C12b total: {tot_f:.3e} flop in {tot_t * 1e3:.1f} ms = {tot_f / tot_t / 1e12:.1f} TF/s ({tot_f / tot_t / PEAK:.3f}); "
      f"{tot_f / (m ** 3 / 3):.3f} of m^3/3")
