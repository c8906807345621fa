"""Ring simulator: one wave of k_stream's schedule on the real cosh^4 tree (diagnostic tool, no GPU).

Models what the persistent kernel's wave does with its LDS ring of sibling pairs -- rounds of <= 64
pairs popped from the top, each pair's refining tasks pushed back as child pairs, the bottom SPILL
pairs moved to the HBM cellar above the spill line, cellar prefetches issued and landed at ring-size
thresholds, bursts cut at the give / poll round -- over the bench's jobs (shares of the tree at seed
depth D). The tree comes from Python's math.cosh (a dynamics model: a 1-ulp difference from glibc
moves nothing that matters here). Against the GPU's DIAG counters (profiles/r03_ab/diag_pipe0.json)
the LIFO schedule gives 61.9 lanes per round (GPU 62.1) and 0.034 spilled pairs per task (0.036).

  python tools/ring_sim.py [--eps 1e-10] [--mode lifo|pipe] [--issue 160] [--land 64] [--hi 192]
"""
import argparse
import collections
import math
import sys


def build_tree(eps, a=0.0, b=5.0):
    """pairs[i] = [left child pair, right child pair, depth]: pair i is the children of refining task
    i (-1: that child accepts)."""
    F = lambda x: math.cosh(x) ** 4
    pairs = []
    st = [(a, b, F(a), F(b), 0, -1, 0)]
    while st:
        l, r, fl, fr, d, par, side = st.pop()
        lr = (fl + fr) * (r - l) / 2
        m = (l + r) / 2
        fm = F(m)
        la = (fl + fm) * (m - l) / 2
        ra = (fm + fr) * (r - m) / 2
        if abs(la + ra - lr) > eps:
            pid = len(pairs)
            pairs.append([-1, -1, d])
            if par >= 0:
                pairs[par][side] = pid
            st.append((l, m, fl, fm, d + 1, pid, 0))
            st.append((m, r, fm, fr, d + 1, pid, 1))
    return pairs


def nodes_at(pairs, D):
    out, st = [], [(0, 0)]
    while st:
        pid, d = st.pop()
        if d == D:
            out.append(pid)
            continue
        c0, c1, _ = pairs[pid]
        if c1 >= 0:
            st.append((c1, d + 1))
        if c0 >= 0:
            st.append((c0, d + 1))
    return out


def run(pairs, mode="lifo", D=7, shares=37, HI=192, SPILL=64, ISSUE=160, LAND=64, GIVE=32):
    nodes = nodes_at(pairs, D)
    jobs = [nodes[i::shares] for i in range(shares)]
    ev = collections.Counter()
    rounds = lanes = tasks = poll = 0
    for job in jobs:
        ring, cellar, pend = list(job), [], None
        while ring or cellar or pend is not None:
            ev["outer"] += 1
            if pend is not None and len(ring) <= LAND:
                ring = pend + ring
                pend = None
                ev["land"] += 1
            if not ring:
                if cellar:
                    k = min(len(cellar), 192)
                    ring = cellar[-k:]
                    del cellar[-k:]
                    ev["sync_refill"] += 1
                continue
            if len(ring) > HI:
                if pend is not None:
                    cellar.extend(pend)
                    pend = None
                    ev["cancel"] += 1
                cellar.extend(ring[:SPILL])
                ring = ring[SPILL:]
                ev["spill"] += 1
                continue
            poll += 1
            if cellar and pend is None and len(ring) <= ISSUE:
                k = min(len(cellar), 64)
                pend = cellar[-k:]
                del cellar[-k:]
                ev["issue"] += 1
            lo = LAND if pend is not None else (ISSUE if cellar else 0)
            bmax = GIVE - poll % GIVE
            r = 0
            nxt = None
            while True:
                if mode == "pipe" and nxt is not None:
                    cur = nxt
                else:
                    n = min(len(ring), 64)
                    cur = ring[len(ring) - n:]
                    del ring[len(ring) - n:]
                if mode == "pipe":   # the next round's pairs are read before this round's pushes
                    n2 = min(len(ring), 64)
                    nxt = ring[len(ring) - n2:]
                    del ring[len(ring) - n2:]
                ring.extend([pairs[p][0] for p in cur if pairs[p][0] >= 0] + [pairs[p][1] for p in cur if pairs[p][1] >= 0])
                r += 1
                rounds += 1
                lanes += len(cur)
                tasks += 2 * len(cur)
                sz = len(ring) + (len(nxt) if nxt else 0)
                if not (lo < sz <= HI) or r == bmax:
                    break
            if nxt:
                ring.extend(nxt)
            poll += r - 1
            ev["burst"] += 1
    out = {"mode": mode, "rounds": rounds, "lanes_per_round": round(lanes / rounds, 2),
           "spilled_pairs_per_task": round(ev["spill"] * SPILL / tasks, 4),
           "mean_burst_rounds": round(rounds / max(ev["burst"], 1), 2)}
    out.update({k + "_per_round": round(v / rounds, 4) for k, v in sorted(ev.items())})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--mode", default="lifo", choices=("lifo", "pipe"))
    ap.add_argument("--issue", type=int, default=160)
    ap.add_argument("--land", type=int, default=64)
    ap.add_argument("--hi", type=int, default=192)
    ap.add_argument("--shares", type=int, default=37)
    a = ap.parse_args()
    sys.setrecursionlimit(10000)
    pairs = build_tree(a.eps)
    D = int(math.floor(math.log2(a.shares))) + 2
    print(run(pairs, a.mode, D=D, shares=a.shares, HI=a.hi, ISSUE=a.issue, LAND=a.land))


if __name__ == "__main__":
    main()
