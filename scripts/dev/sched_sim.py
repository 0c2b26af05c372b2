"""Makespan of the MLP work lists over 8 XCDs x 64 workgroup slots: equal-count contiguous XCD
shares (round 3) vs the cost-balanced assignment of metaopt_amd/ops/population.py _xcd_schedule
(simulated in units of one 64x64 backward chunk)."""
import numpy as np, heapq
rng = np.random.RandomState(0)
P=256
w = np.array([int(np.exp(rng.uniform(np.log(64), np.log(1024)))) for _ in range(P)])
wp = (w+63)//64*64
def lpt(cost, n_xcd=8):
    n=len(cost); q,r=divmod(n,n_xcd); pos=np.arange(n)
    share=np.where(pos < r*(q+1), pos//(q+1), r+(pos-r*(q+1))//max(q,1))
    return np.lexsort((-cost, share)), share
def sim(K, N, slots_per_xcd=64, per_chunk=1.0, overhead=0.0):
    nk = K//64
    cost = np.repeat(N//64, nk).astype(float)*per_chunk + overhead
    order, share = lpt(cost)
    cost = cost[order]
    # xcd x processes contiguous positions share==x in order (xcd_remap)
    ends=[]
    for x in range(8):
        c = cost[share==x]
        heap=[0.0]*slots_per_xcd
        for t in c:
            s=heapq.heappop(heap); heapq.heappush(heap, s+t)
        ends.append(max(heap))
    ideal = cost.sum()/(8*slots_per_xcd)
    return max(ends), ideal, ends
for name,K,N in [("bwd0", np.full(P,832), wp), ("bwd1", wp, wp), ("bwd3", wp, np.full(P,64))]:
    m, ideal, ends = sim(K,N)
    print(name, "makespan", round(m,1), "ideal", round(ideal,1), "eff", round(ideal/m,3), "xcd ends", [round(e,1) for e in ends])

def sim2(K, N, slots_per_xcd=64):
    nk = K//64; cost_t = nk*(N//64)  # per trial
    load=np.zeros(8); xcd_of=np.zeros(P,int)
    for t in np.argsort(-cost_t, kind="stable"):
        x=int(np.argmin(load)); xcd_of[t]=x; load[x]+=cost_t[t]
    ends=[]
    for x in range(8):
        items=[]
        for t in np.flatnonzero(xcd_of==x):
            items += [N[t]//64]*nk[t]
        items=sorted(items, reverse=True)
        heap=[0.0]*slots_per_xcd
        for c in items:
            s=heapq.heappop(heap); heapq.heappush(heap, s+c)
        ends.append(max(heap))
    ideal=cost_t.sum()/(8*slots_per_xcd)
    return max(ends), ideal, ends
for name,K,N in [("bwd0", np.full(P,832), wp), ("bwd1", wp, wp), ("bwd3", wp, np.full(P,64))]:
    m, ideal, ends = sim2(K,N)
    print("balanced", name, "makespan", round(m,1), "ideal", round(ideal,1), "eff", round(ideal/m,3), [round(e,1) for e in ends])
