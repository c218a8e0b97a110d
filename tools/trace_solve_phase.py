"""Summarise the solve phase after the last big Gram launch from a rocprofv3 --kernel-trace CSV.
usage: trace_solve_phase.py <kernel_trace.csv> [n_lines_of_timeline]"""
import csv, collections, sys
r=list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x:int(x['Start_Timestamp']))
big=[i for i,x in enumerate(r) if int(x['End_Timestamp'])-int(x['Start_Timestamp'])>50e6]
i0=big[-1]; t0=int(r[i0]['End_Timestamp'])
seg=r[i0+1:]
end=[i for i,x in enumerate(seg) if 'score_tail' in x['Kernel_Name'] or 'chol_fwd' in x['Kernel_Name']][0]
seg=seg[:end]
tend=max(int(x['End_Timestamp']) for x in seg)
print('factor span ms', (tend-t0)/1e6, 'kernels', len(seg), collections.Counter(x['Queue_Id'] for x in seg))
agg=collections.defaultdict(lambda:[0,0.0])
for x in seg:
    n=x['Kernel_Name'].split('(')[0][:60]+' q'+x['Queue_Id']; d=(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3
    agg[n][0]+=1; agg[n][1]+=d
for k,v in sorted(agg.items(), key=lambda kv:-kv[1][1])[:25]: print(f"{k:66s} {v[0]:6d} {v[1]:10.1f} {v[1]/v[0]:8.1f}")
if len(sys.argv)>2:
    n=int(sys.argv[2])
    for x in seg[:n]:
        s,e=int(x['Start_Timestamp']),int(x['End_Timestamp'])
        print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} q{x['Queue_Id']} {x['Kernel_Name'].split('(')[0][:50]} grid={x['Grid_Size_X']}")
