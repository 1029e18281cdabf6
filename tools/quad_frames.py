"""Search the lane frames of quad-mode BLAKE2b.

In quad mode lane i of a quad holds one element of each row a, b, c, d of
the working vector.  The column step pairs a_j, b_j, c_j, d_j; the diagonal
step a_j, b_{j+1}, c_{j+2}, d_{j+3}.  An operation on two rows held for
different G indices reads one of them across lanes by DPP:
  * xor (VOP2) takes a DPP source for free;
  * a 64-bit add is v_lshl_add_u64 (VOP3, no DPP on gfx9): with a DPP source
    it becomes a VOP2 carry pair, one instruction more ("costly add");
  * a DPP source written fewer than 2 instructions earlier needs filler
    instructions in between (the gfx9 DPP hazard): 2 after a one-instruction
    64-bit write, 1 after a two-instruction one read in the same order; the
    two message adds of a step (a + x, a + y) fill one slot each for free.
For every 2-step periodic assignment this prints the Pareto set of
(costly adds, fillers) per 2 steps.  Result: (4, 0) -- what the loop does --
or (3, 7) / (2, 9), against ~3.75 independent instructions per 2 steps that
could fill (the 45 loads / reads / writes of a compression over its 12 step
pairs): the missing fillers would be s_nops, so (4, 0) is the cheapest.

    python tools/quad_frames.py
"""
import itertools

DELTA = {0: (0, 0, 0, 0), 1: (0, 1, 2, 3)}  # column, diagonal
# one G step: (kind, destination row, other row); rows a=0 b=1 c=2 d=3
OPS = [("add", 0, 1), ("xor", 3, 0), ("add", 2, 3), ("xor", 1, 2),
       ("add", 0, 1), ("xor", 3, 0), ("add", 2, 3), ("xor", 1, 2)]
NEWEST = {0: 1, 1: 0, 2: 3, 3: 2, 4: 1, 5: 0, 6: 3, 7: 2}  # operand written by the previous op


def step(G):
    """All (frames after, costly adds, fillers, choices) of one step from frames G."""
    res = []

    def dfs(k, g, cost, fill, single_prev, ch):
        if k == 8:
            res.append((g, cost, fill, tuple(ch)))
            return
        kind, x, y = OPS[k]
        free = 1 if k in (1, 5) else 0  # (a + y) after op 1, (a + x) after op 5
        opts = []
        if g[x] == g[y]:
            opts.append((g, 0, 0, "L"))
        else:
            for dpp, r in ((y, g[x]), (x, g[y])):
                h = list(g)
                h[x] = r
                need = 0
                if dpp == NEWEST[k]:
                    need = 1 if k == 0 else (2 if single_prev else 1)
                    need = max(0, need - free)
                opts.append((tuple(h), 1 if kind == "add" else 0, need, "D" + "abcd"[dpp]))
        for h, c, f, tag in opts:
            dfs(k + 1, h, cost + c, fill + f, kind == "add" and tag == "L", ch + [tag])
    dfs(0, tuple(G), 0, 0, False, [])
    return res


def trans(G, cur, nxt):
    return tuple((G[k] + DELTA[cur][k] - DELTA[nxt][k]) % 4 for k in range(4))


def main():
    best = {}
    for G0 in itertools.product(range(4), repeat=4):
        for G1, c1, f1, ch1 in step(G0):
            for G2, c2, f2, ch2 in step(trans(G1, 0, 1)):
                if trans(G2, 1, 0) == G0:
                    best.setdefault((c1 + c2, f1 + f2), (G0, ch1, ch2))
    pareto, bf = [], None
    for key in sorted(best):
        if bf is None or key[1] < bf:
            pareto.append(key)
            bf = key[1]
    print("per 2 steps (costly adds, fillers), Pareto set:")
    for key in pareto:
        G0, ch1, ch2 = best[key]
        print("  %s  frames %s  column %s  diagonal %s" % (key, G0, " ".join(ch1), " ".join(ch2)))


if __name__ == "__main__":
    main()
