"""Can the quad loop's 40 per-lane message reads be paired into ds_read2_b64?
A pair of read slots shares one per-lane address when the 4 lanes' word
positions differ by the same offset.  Tries every layout of the line's eight
16-B chunks in LDS and prints the largest matching (diagnostics; see
DESIGN.md 4.2).  Result: at most 5 pairs.

--words: word-level layouts instead, as two ds_write2_b64 per lane would
write them (lane L's words 4L, 4L+1 at a per-lane base and base + alpha,
words 4L+2, 4L+3 at a second base and base + beta; alpha, beta uniform),
searched by hill climbing (20000 steps per seed, positions < 48 words).
Result over seven seeds: at most 4 pairs -- the chunk layouts stay best."""
import itertools, random, sys
import networkx as nx
S=[[0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15],
[14,10,4,8,9,15,13,6,1,12,0,2,11,7,5,3],
[11,8,12,0,5,2,15,13,10,14,3,6,7,1,9,4],
[7,9,3,1,13,12,11,14,2,6,5,10,4,0,15,8],
[9,0,5,7,2,4,10,15,14,1,11,12,6,8,3,13],
[2,12,6,10,0,11,8,3,4,13,7,5,15,14,1,9],
[12,5,1,15,14,13,4,10,0,7,6,3,9,2,8,11],
[13,11,7,14,12,1,3,9,5,0,15,4,8,6,2,10],
[6,15,14,9,11,3,0,8,12,2,13,7,1,4,10,5],
[10,2,8,4,7,6,1,5,15,11,9,14,3,12,13,0]]
slots=[]
for r in range(10):
    s=S[r]
    slots.append(tuple(s[2*i] for i in range(4)))
    slots.append(tuple(s[2*i+1] for i in range(4)))
    slots.append(tuple(s[8+2*i] for i in range(4)))
    slots.append(tuple(s[9+2*i] for i in range(4)))


def max_pairs(pos):
    G = nx.Graph()
    P = [tuple(pos[w] for w in sl) for sl in slots]
    for a, b in itertools.combinations(range(40), 2):
        d = [P[b][i] - P[a][i] for i in range(4)]
        if d[0] != 0 and abs(d[0]) < 256 and len(set(d)) == 1:
            G.add_edge(a, b)
    return len(nx.max_weight_matching(G, maxcardinality=True))


def chunk_layouts():
    best = (0, None)
    hist = {}
    for perm in itertools.permutations(range(8)):
        pos = [0] * 16
        for c in range(8):
            pos[2 * c] = 2 * perm[c]
            pos[2 * c + 1] = 2 * perm[c] + 1
        m = max_pairs(pos)
        hist[m] = hist.get(m, 0) + 1
        if m > best[0]:
            best = (m, perm)
            print(best, flush=True)
    print(hist)


def word_layouts(seed, steps=20000, span=48):
    rng = random.Random(seed)

    def layout(base, al, be):
        pos = [0] * 16
        for L in range(4):
            pos[4 * L], pos[4 * L + 1] = base[L][0], base[L][0] + al
            pos[4 * L + 2], pos[4 * L + 3] = base[L][1], base[L][1] + be
        return pos if len(set(pos)) == 16 else None

    def draw():
        while True:
            c = ([[rng.randrange(span), rng.randrange(span)] for _ in range(4)],
                 rng.randrange(1, span), rng.randrange(1, span))
            if layout(*c):
                return c

    cur = draw()
    cm = best = max_pairs(layout(*cur))
    for it in range(steps):
        base, al, be = [list(x) for x in cur[0]], cur[1], cur[2]
        k = rng.randrange(10)
        if k < 8:
            base[k // 2][k % 2] = rng.randrange(span)
        elif k == 8:
            al = rng.randrange(1, span)
        else:
            be = rng.randrange(1, span)
        pos = layout(base, al, be)
        if not pos:
            continue
        m = max_pairs(pos)
        if m >= cm:
            cur, cm = (base, al, be), m
            if m > best:
                best = m
                print(seed, it, best, pos, flush=True)
        if it % 2000 == 0 and rng.random() < 0.3:
            cur = draw()
            cm = max_pairs(layout(*cur))
    print("seed", seed, "best", best)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--words":
        for seed in range(1, 8):
            word_layouts(seed)
    else:
        chunk_layouts()
