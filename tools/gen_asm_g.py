# Generates tools/asm_g_bodies.h for tools/asm_g_ubench.hip (python3 tools/gen_asm_g.py > tools/asm_g_bodies.h)
# Generate inline-asm bodies for one half-round (4 independent G) in three orders.
def regs():
    R = {}
    base = 10
    for name in "abcd":
        for k in range(4):
            R[f"{name}{k}"] = base; base += 2
    for k in range(4):
        R[f"t{k}"] = base; base += 2   # d' (xor+rot32 result)
        R[f"u{k}"] = base; base += 2   # xor scratch
    R["x"] = base; base += 2
    R["y"] = base; base += 2
    return R, base

def p(r):  # pair
    return f"v[{r}:{r+1}]"
def lo(r): return f"v{r}"
def hi(r): return f"v{r+1}"

def g_steps(R, k):
    a, b, c, d, t, u, x, y = (R[f"a{k}"], R[f"b{k}"], R[f"c{k}"], R[f"d{k}"], R[f"t{k}"], R[f"u{k}"], R["x"], R["y"])
    S = []
    S.append(("S1a", f"v_lshl_add_u64 {p(a)}, {p(a)}, 0, {p(x)}"))
    S.append(("S1b", f"v_lshl_add_u64 {p(a)}, {p(a)}, 0, {p(b)}"))
    S.append(("S2", f"v_xor_b32 {lo(t)}, {hi(d)}, {hi(a)}"))
    S.append(("S2", f"v_xor_b32 {hi(t)}, {lo(d)}, {lo(a)}"))
    S.append(("S3", f"v_lshl_add_u64 {p(c)}, {p(c)}, 0, {p(t)}"))
    S.append(("S4a", f"v_xor_b32 {lo(u)}, {lo(b)}, {lo(c)}"))
    S.append(("S4a", f"v_xor_b32 {hi(u)}, {hi(b)}, {hi(c)}"))
    S.append(("S4b", f"v_alignbit_b32 {lo(b)}, {hi(u)}, {lo(u)}, 24"))
    S.append(("S4b", f"v_alignbit_b32 {hi(b)}, {lo(u)}, {hi(u)}, 24"))
    S.append(("S5a", f"v_lshl_add_u64 {p(a)}, {p(a)}, 0, {p(y)}"))
    S.append(("S5b", f"v_lshl_add_u64 {p(a)}, {p(a)}, 0, {p(b)}"))
    S.append(("S6a", f"v_xor_b32 {lo(u)}, {lo(t)}, {lo(a)}"))
    S.append(("S6a", f"v_xor_b32 {hi(u)}, {hi(t)}, {hi(a)}"))
    S.append(("S6b", f"v_alignbit_b32 {lo(d)}, {hi(u)}, {lo(u)}, 16"))
    S.append(("S6b", f"v_alignbit_b32 {hi(d)}, {lo(u)}, {hi(u)}, 16"))
    S.append(("S7", f"v_lshl_add_u64 {p(c)}, {p(c)}, 0, {p(d)}"))
    S.append(("S8a", f"v_xor_b32 {lo(u)}, {lo(b)}, {lo(c)}"))
    S.append(("S8a", f"v_xor_b32 {hi(u)}, {hi(b)}, {hi(c)}"))
    S.append(("S8b", f"v_alignbit_b32 {lo(b)}, {lo(u)}, {hi(u)}, 31"))
    S.append(("S8b", f"v_alignbit_b32 {hi(b)}, {hi(u)}, {lo(u)}, 31"))
    return S

def order(kind):
    R, top = regs()
    Gs = [g_steps(R, k) for k in range(4)]
    out = []
    if kind == "gmajor":
        for G in Gs: out += [s for _, s in G]
    elif kind == "rr":  # round-robin instruction by instruction
        for i in range(20):
            for G in Gs: out.append(G[i][1])
    elif kind == "step":
        steps = ["S1a","S1b","S2","S3","S4a","S4b","S5a","S5b","S6a","S6b","S7","S8a","S8b"]
        for st in steps:
            for G in Gs:
                out += [s for tag, s in G if tag == st]
    return out, top

for kind in ("gmajor", "rr", "step"):
    ins, top = order(kind)
    body = "\\n".join(ins)
    print(f'#define ASM_HALF_{kind.upper()} "{body}\\n"')
print(f"#define ASM_TOP_REG {top}")


def variant(kind, sgpr_msg=False, align_as_xor=False, add_as_xor=False):
    ins, top = order(kind)
    out = []
    for s in ins:
        if sgpr_msg:
            s = s.replace("v[58:59]", "s[40:41]").replace("v[60:61]", "s[42:43]")
        if align_as_xor and s.startswith("v_alignbit_b32"):
            parts = s.split(", ")
            s = "v_xor_b32 " + parts[0].split()[1] + ", " + parts[1] + ", " + parts[2]
        out.append(s)
    return "\\n".join(out)

def variant_addxor():
    ins, top = order("step")
    out = []
    for s in ins:
        if s.startswith("v_lshl_add_u64"):
            # v_lshl_add_u64 v[a:a+1], v[a:a+1], 0, v[b:b+1] -> v_xor_b32 va, va, vb
            parts = s.replace("v_lshl_add_u64 ", "").split(", ")
            d = int(parts[0][2:].split(":")[0]); b = int(parts[3][2:].split(":")[0])
            s = "v_xor_b32 v%d, v%d, v%d" % (d, d, b)
        out.append(s)
    return "\\n".join(out)

def independent_mix():
    # same class mix as one half-round (24 lshl_add, 24 alignbit, 32 xor) in
    # step order, but no instruction depends on the previous 16
    out = []
    pattern = (["A"] * 8 + ["X"] * 8 + ["A"] * 4 + ["X"] * 8 + ["L"] * 8 + ["A"] * 8 + ["X"] * 8 +
               ["L"] * 8 + ["A"] * 4 + ["X"] * 8 + ["L"] * 8)
    ia = il = ix = 0
    for c in pattern:
        if c == "A":
            r = 10 + 2 * (ia % 8); out.append("v_lshl_add_u64 v[%d:%d], v[%d:%d], 0, v[58:59]" % (r, r + 1, r, r + 1)); ia += 1
        elif c == "L":
            r = 26 + (il % 16); out.append("v_alignbit_b32 v%d, v%d, v59, 7" % (r, r)); il += 1
        else:
            r = 42 + (ix % 16); out.append("v_xor_b32 v%d, v%d, v60" % (r, r)); ix += 1
    return "\\n".join(out)

print('#define ASM_HALF_STEP_ADDXOR "%s\\n"' % variant_addxor())
print('#define ASM_HALF_INDEP_MIX "%s\\n"' % independent_mix())
print('#define ASM_HALF_STEP_SMSG "%s\\n"' % variant("step", sgpr_msg=True))
print('#define ASM_HALF_STEP_ALIGNXOR "%s\\n"' % variant("step", align_as_xor=True))
