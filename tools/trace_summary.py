"""Steady-state summary of a pipelined config-3/4 kernel trace (the compact CSV `tools/trace_steps.py ... dump` writes):
over the longest cluster of fused-kernel launches, the medians / min / max of the fused, lean and slot durations, the
time from each batch's lean pass ending to its fused kernel starting (the feature chain's slack) and from the previous
fused launch ending (negative: the launches overlap).

usage: python tools/trace_summary.py steps.csv"""
import csv, sys
rows=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name']) for r in csv.DictReader(open(sys.argv[1]))]
rows.sort()
ens=[r for r in rows if r[2]=='ens']
# longest cluster
cl=[];cur=[ens[0]]
for a,b in zip(ens,ens[1:]):
    if b[0]-a[1]>2_000_000: cl.append(cur); cur=[]
    cur.append(b)
cl.append(cur)
c=max(cl,key=len)
lo,hi=c[0][0]-300_000,c[-1][1]
R=[r for r in rows if lo<=r[0]<=hi]
slots=[r for r in R if r[2]=='slot']; leans=[r for r in R if r[2]=='lean']; E=[r for r in R if r[2]=='ens']
print(len(slots),len(leans),len(E))
# align: assume the k-th lean precedes k-th ens
import statistics as st
n=min(len(leans),len(E))
off=0
# find offset such that lean[k].end <= ens[k+off].start mostly
wait_feat=[];overlap=[];dur=[];ldur=[];sdur=[]
for k in range(n):
    l=leans[k]; e=E[k]
    wait_feat.append((e[0]-l[1])/1e3)
    dur.append((e[1]-e[0])/1e3); ldur.append((l[1]-l[0])/1e3)
for k in range(1,len(E)):
    overlap.append((E[k][0]-E[k-1][1])/1e3)
sd=[(s[1]-s[0])/1e3 for s in slots]
q=lambda x:(round(st.median(x),2), round(min(x),2), round(max(x),2))
print('ens dur', q(dur)); print('lean dur', q(ldur)); print('slot dur', q(sd))
print('ens start - lean end', q(wait_feat)); print('ens start - prev ens end', q(overlap))
print('step (ens start to start)', q([(E[k][0]-E[k-1][0])/1e3 for k in range(1,len(E))]))
# how many ens started within 3us of its lean's end (feature-bound) vs within 3 us of previous ens end
fb=sum(1 for w in wait_feat if w<3); print('ens starting <3us after its lean ends:', fb, 'of', n)
