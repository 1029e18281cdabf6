"""Can the quad loop's 40 per-lane message reads be paired into ds_read2_b64?
A pair of read slots shares one per-lane address when the 4 lanes' word
positions differ by the same offset.  Tries every layout of the line's eight
16-B chunks in LDS and prints the largest matching (diagnostics; see
DESIGN.md 4.2).  Result: at most 5 pairs."""
import itertools, networkx as nx
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
best=(0,None)
hist={}
for perm in itertools.permutations(range(8)):
    pos=[0]*16
    for c in range(8):
        pos[2*c]=2*perm[c]; pos[2*c+1]=2*perm[c]+1
    G=nx.Graph()
    P=[tuple(pos[w] for w in sl) for sl in slots]
    for a,b in itertools.combinations(range(40),2):
        d=[P[b][i]-P[a][i] for i in range(4)]
        if d[0]!=0 and len(set(d))==1: G.add_edge(a,b)
    m=len(nx.max_weight_matching(G,maxcardinality=True))
    hist[m]=hist.get(m,0)+1
    if m>best[0]: best=(m,perm); print(best,flush=True)
print(hist)
