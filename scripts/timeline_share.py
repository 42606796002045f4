"""Each kernel's share of the GPU timeline in a window of a rocprofv3 kernel trace
(time split evenly among the kernels running at once), per batch.
Usage: timeline_share.py <trace dir> <from ms> <to ms, relative to the last kernel end> <batches>"""
import csv,sys,collections
d=sys.argv[1]; a_ms=float(sys.argv[2]); b_ms=float(sys.argv[3]); nb=float(sys.argv[4])
K=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
ks=[(int(k['Start_Timestamp']),int(k['End_Timestamp']),k['Kernel_Name']) for k in K]
t_end=max(e for s,e,n in ks)
A=t_end+a_ms*1e6;B=t_end+b_ms*1e6
ev=[]
import re
def short(n):
    n=re.sub(r'otm::\(anonymous namespace\)::','',n); n=n.split('(')[0]
    if 'copyBuffer' in n: n='copyBuffer'
    if 'rocprim' in n: n='rocprim'
    return n[:40]
for s,e,n in ks:
    if e<=A or s>=B: continue
    ev.append((max(s,A),1,short(n))); ev.append((min(e,B),-1,short(n)))
ev.sort()
run=collections.Counter(); share=collections.Counter(); last=A; idle=0
for t,dlt,n in ev:
    dt=t-last
    if run:
        tot=sum(run.values())
        for k,c in run.items(): share[k]+=dt*c/tot
    else: idle+=dt
    last=t
    run[n]+=dlt
    if run[n]==0: del run[n]
W=B-A
print(f"window {W/1e6:.2f} ms, idle {idle/1e6:.2f} ms, per batch ({nb}):")
for k,v in share.most_common(30): print(f"  {k:42s} {v/1e3/nb:8.1f} us/batch")
print(f"  total {sum(share.values())/1e3/nb:.1f} us/batch")
