"""Summarise one Cholesky factor from a rocprofv3 --kernel-trace CSV: per-kernel/queue totals, queue busy time,
outer-block start times.  usage: trace_chol_factor.py <kernel_trace.csv> [n_diag_launches] [outer_stride]"""
import csv, collections, sys
r=list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x:int(x['Start_Timestamp']))
idx=[i for i,x in enumerate(r) if 'chol_diag' in x['Kernel_Name']]
nd=int(sys.argv[2]) if len(sys.argv)>2 else 256
last=idx[-1]; st=idx[-nd]
t0=int(r[st]['Start_Timestamp'])
seg=r[st:last+1]
agg=collections.defaultdict(lambda:[0,0.0])
for x in seg:
    n=x['Kernel_Name'].split('(')[0][:60]+' q'+x['Queue_Id']; d=(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3
    agg[n][0]+=1; agg[n][1]+=d
print('span', (int(r[last]['End_Timestamp'])-t0)/1e6)
for k,v in sorted(agg.items(), key=lambda kv:-kv[1][1])[:8]: print(f"{k:66s} {v[0]:6d} {v[1]:10.1f} {v[1]/v[0]:8.1f}")
for q in sorted(set(x['Queue_Id'] for x in seg)):
    iv=sorted((int(x['Start_Timestamp']),int(x['End_Timestamp'])) for x in seg if x['Queue_Id']==q)
    busy=0; cs,ce=iv[0]
    for s,e in iv[1:]:
        if s>ce: busy+=ce-cs; cs,ce=s,e
        else: ce=max(ce,e)
    busy+=ce-cs
    print('queue',q,'busy ms',round(busy/1e6,2))
# per outer block (8 diag) chain timing
di=[i for i,x in enumerate(seg) if 'chol_diag' in x['Kernel_Name']]
for b in range(0, len(di), 8*int(sys.argv[3]) if len(sys.argv)>3 else 8):
    i=di[b]; s=int(seg[i]['Start_Timestamp'])
    print(f"outer {b//8:3d} start {(s-t0)/1e6:8.2f} ms")
