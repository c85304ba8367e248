"""List-scheduling simulation of a cast launch from per-block stamps (bench.py --stats with SVO_STAMPS=path):
blocks dealt round robin to 8 XCDs of 1024 wave slots, greedy in dispatch order.  usage: python tools/sim_dispatch.py stamps.npy"""
import numpy as np, heapq, sys
st = np.load(sys.argv[1]).astype(np.float64) / 100.0
dur = st[:, 1] - st[:, 0]
start = st[:, 0] - st[:, 0].min()
n = len(dur)
print("blocks", n, "mean", dur.mean(), "max", dur.max(), "sum/8192", dur.sum() / 8192)
def sim(order, slots_per_xcd=1024, xcds=8):
    # block i of the dispatch goes to XCD i % 8 (round robin), greedy in order within an XCD
    ends = []
    for x in range(xcds):
        q = order[x::xcds]
        h = [0.0] * slots_per_xcd
        heapq.heapify(h)
        m = 0
        for b in q:
            t = heapq.heappop(h)
            e = t + dur[b]
            m = max(m, e)
            heapq.heappush(h, e)
        ends.append(m)
    return max(ends), ends
base = np.arange(n)
print("actual makespan", (st[:,1].max() - st[:,0].min()))
print("sim in-order", sim(base)[0])
print("sim LPT (block)", sim(np.argsort(-dur, kind="stable"))[0])
# per tile row (blocks are 240 per tile row for 1080p: tiles_x = 120 footprint columns x 2 subrows)
for per in (240, 960):
    if n % per == 0:
        rows = dur.reshape(-1, per)
        ordr = np.argsort(-rows.sum(1), kind="stable")
        order = (ordr[:, None] * per + np.arange(per)[None, :]).reshape(-1)
        print("sim LPT by group of %d blocks" % per, sim(order)[0])
# blocks of 8 per XCD chunk
print("sim reversed", sim(base[::-1])[0])
rows = dur.reshape(-1, 240)
print("row sums (top first) ", np.round(rows.sum(1)[:40]/240,1))
print("row max", np.round(rows.max(1)[:40],0))
mx = rows.max(1)
ordr = np.argsort(-mx, kind="stable")
order = (ordr[:, None] * 240 + np.arange(240)[None, :]).reshape(-1)
print("sim LPT by row max", sim(order)[0])
ordr = np.argsort(-rows.sum(1), kind="stable")
print(ordr[:20])
for g in (2, 4, 8, 16, 30, 60, 120):
    if n % g: continue
    gr = dur.reshape(-1, g)
    for nm, key in (("max", gr.max(1)), ("sum", gr.sum(1))):
        ordr = np.argsort(-key, kind="stable")
        order = (ordr[:, None] * g + np.arange(g)[None, :]).reshape(-1)
        print("sim LPT groups of %d by %s: %.1f" % (g, nm, sim(order)[0]))
# hybrid: the heaviest fraction of waves first (longest first), the rest in the shipped order
for frac in (0.01, 0.02, 0.05, 0.1, 0.2):
    k = int(n * frac)
    heavy = np.argsort(-dur, kind="stable")[:k]
    mask = np.ones(n, bool); mask[heavy] = False
    order = np.concatenate([heavy, np.arange(n)[mask]])
    print("sim heaviest %4.1f%% first: %.1f" % (100 * frac, sim(order)[0]))
