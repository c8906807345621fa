"""The contiguous-block seeding partition of lone launches (k_stream with AQ_LONE_BLOCK, aq_abi.inc
launch_stream): share sh of S = 2^Dp shares evaluates the path of its block root (depths 0..Dp-1)
and its block's subtree (depths Dp..D, D = Dp + s), counts a path node when its block starts at the
node's leftmost position and every subtree node, and pushes the children of the refining depth-D
nodes. Restated here over a tree built with the reference's refine test (aquadPartA.c:185-191;
Python's cosh: the partition is about the tree's shape, not its last bits) and checked to count every
node at depth <= D exactly once and to seed exactly the tree's refining depth-D nodes."""
import math

import pytest


def _tree_checks(eps, W=3072, s=4, a=0.0, b=5.0):
    F = lambda x: math.cosh(x) ** 4
    sp = 1
    while sp * 2 <= W:
        sp *= 2
    Dp = sp.bit_length() - 1
    D = Dp + s
    memo = {}

    def interval(d, g):
        lo, hi = a, b
        for i in range(d):
            mm = (lo + hi) / 2                                   # :187
            if (g >> (d - 1 - i)) & 1:
                lo = mm
            else:
                hi = mm
        return lo, hi

    def refines(d, g):
        if (d, g) not in memo:
            lo, hi = interval(d, g)
            m = (lo + hi) / 2
            fl, fr, fm = F(lo), F(hi), F(m)
            lr = (fl + fr) * (hi - lo) / 2                       # :185
            la = (fl + fm) * (m - lo) / 2                        # :189
            ra = (fm + fr) * (hi - m) / 2                        # :190
            memo[(d, g)] = abs((la + ra) - lr) > eps             # :191
        return memo[(d, g)]

    truth, seeds_truth, stack = set(), set(), [(0, 0)]
    while stack:
        d, g = stack.pop()
        truth.add((d, g))
        if refines(d, g):
            if d < D:
                stack += [(d + 1, 2 * g), (d + 1, 2 * g + 1)]
            else:
                seeds_truth.add((d, g))
    counted, seeds = [], set()
    for sh in range(sp):
        nodes = [(d, sh >> (Dp - d)) for d in range(Dp)] + \
                [(Dp + e, (sh << e) + t) for e in range(s + 1) for t in range(1 << e)]
        assert Dp + len(nodes) - Dp + 2 <= 64   # one lane per node, plus F(A) and F(B)
        leaf = {n for n in nodes if not refines(*n)}
        for d, g in nodes:
            reach = not ({(i, g >> (d - i)) for i in range(d)} & leaf)
            owned = d >= Dp or (sh & ((1 << (Dp - d)) - 1)) == 0
            if reach and owned:
                counted.append((d, g))
            if reach and refines(d, g) and d == D:
                seeds.add((d, g))
    return truth, counted, seeds_truth, seeds


@pytest.mark.parametrize("eps", [1e-3, 1e-6])
def test_block_partition_counts_each_node_once(eps):
    truth, counted, seeds_truth, seeds = _tree_checks(eps)
    assert len(counted) == len(set(counted)) and set(counted) == truth
    assert seeds == seeds_truth
