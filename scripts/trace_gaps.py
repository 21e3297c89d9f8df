"""Kernel time and inter-kernel gaps over the second half of a rocprofv3 kernel trace (the steady
solves of a bench run).  usage: python scripts/trace_gaps.py <trace_kernel_trace.csv>"""
import csv, sys, collections
f=sys.argv[1]
v=[]
for r in csv.DictReader(open(f)):
    v.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][-60:], r.get('Stream_Id', '')))
v.sort()
# steady region: last solve = kernels after the last-but-one k_spmv_stream burst... take last 40% of spmv kernels
sp=[i for i,x in enumerate(v) if 'spmv_stream' in x[2]]
lo=sp[len(sp)//2]; hi=sp[-1]
seg=v[lo:hi+1]
span=(seg[-1][1]-seg[0][0])/1e3
busy=sum((x[1]-x[0]) for x in seg)/1e3
print('span us',span,'busy us',busy,'frac',busy/span, 'spmv', len([x for x in seg if 'spmv_stream' in x[2]]))
gaps=collections.defaultdict(float); cnt=collections.Counter()
for a,b in zip(seg,seg[1:]):
    g=(b[0]-a[1])/1e3
    if g>0: gaps[(a[2],b[2])]+=g; cnt[(a[2],b[2])]+=1
for k,g in sorted(gaps.items(), key=lambda t:-t[1])[:12]: print(round(g,1), cnt[k], k)
tot=collections.defaultdict(float)
for x in seg: tot[x[2]]+=(x[1]-x[0])/1e3
for k,t in sorted(tot.items(), key=lambda t:-t[1])[:14]: print(round(t,1), k)
