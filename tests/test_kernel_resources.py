"""Register budgets of the shipped kernels, from the built code object (CPU).

Occupancy is part of each kernel's design: the hot
lane-mode kernel must fit 4 waves per SIMD with nothing spilled, the quad
kernels hold their whole chain state and two message sets in registers, and
an exclusive quad wave owns its SIMD's whole register file.  A compiler or
source change that spills or loses occupancy fails here instead of showing up
as a slower bench on the GPU."""
import pytest

import codeobj

pytestmark = pytest.mark.skipif(not codeobj.available(),
                                reason="needs the built library and ROCm's llvm-readelf")


@pytest.fixture(scope="module")
def res(tmp_path_factory):
    return codeobj.resources(str(tmp_path_factory.mktemp("co")))


def one(res, short):
    hits = codeobj.find(res, short)
    assert hits, short
    return hits


def test_hot_kernel_fits_four_waves_unspilled(res):
    (k,) = one(res, "k_chunks").values()
    assert k["vgpr_count"] <= 128 and k["agpr_count"] == 0
    assert k["vgpr_spill_count"] == 0 and k["sgpr_spill_count"] == 0


@pytest.mark.parametrize("short", ["k_quad_long", "k_quad_chunks", "k_quad_relay",
                                   "k_desc_relay", "k_chain_step", "k_single",
                                   "k_compress_only", "k_general", "k_verify",
                                   "k_chain_keys", "k_order_place"])
def test_no_spills(res, short):
    for name, k in one(res, short).items():
        assert k["vgpr_spill_count"] == 0 and k["sgpr_spill_count"] == 0, (name, k)


def test_exclusive_quad_wave_owns_its_simd(res):
    """k_quad_long<true> touches a255, so a wave allocates all 512 registers
    (VGPR + AGPR) of its SIMD and no lane wave shares it."""
    hits = one(res, "k_quad_long")
    excl = [k for n, k in hits.items() if "ILb1E" in n]
    assert len(excl) == 1
    k = excl[0]
    assert k["vgpr_count"] + k.get("agpr_count", 0) >= 504 or k["vgpr_count"] >= 504, k


def test_known_spills_stay_bounded(res):
    """The two kernels that spill today, bounded so they cannot grow
    unnoticed: k_lane_rest (~10 VGPRs around the chain loop, none inside it,
    DESIGN.md 4.2) and k_sha_desc (2 SGPRs)."""
    (lr,) = one(res, "k_lane_rest").values()
    assert lr["vgpr_count"] <= 128 and lr["vgpr_spill_count"] <= 12
    (sha,) = one(res, "k_sha_desc").values()
    assert sha["vgpr_count"] <= 102 and sha["vgpr_spill_count"] == 0
    assert sha["sgpr_spill_count"] <= 2


@pytest.mark.parametrize("short", ["k_quad_long", "k_quad_chunks", "k_quad_relay",
                                   "k_desc_relay", "k_chain_step", "k_single"])
def test_quad_dpp_instructions_are_8_byte_aligned(tmp_path, short):
    """A VOP2 DPP instruction (8 bytes) that straddles an 8-byte boundary
    issues ~10 % slower for a wave alone (tools/align_ubench.hip), and the
    quad kernels moved 7-10 % with nothing but their code offset
    (profiles/r02/quad_fast/ab_fastpad.log): every quad asm block starts
    with .p2align 3 and keeps its 4-byte instructions in pairs
    (blake2b_dev.hpp CIR_QALIGN).  Checked on the built code object."""
    table = codeobj.disassembly(str(tmp_path), with_addr=True)
    hits = codeobj.find(table, short)
    assert hits, short
    for name, body in hits.items():
        # the DPP carry pairs come only from the asm G steps; the compiler's
        # own DPP xors (the general path's finalisation) are not aligned by it
        dpp = [(a, ins) for a, ins in body if ins.split()[0] in ("v_add_co_u32_dpp",
                                                                  "v_addc_co_u32_dpp")]
        assert dpp, name
        bad = [(hex(a), ins) for a, ins in dpp if a is None or a % 8]
        assert not bad, (name, len(bad), len(dpp), bad[:3])


def test_hot_loop_reads_overlap_round_zero(tmp_path):
    """k_chunks' line loop issues the next line's LDS-DMA only after round
    0's column step (blake2b_dev.hpp compress_sm hook, uniform.hpp): between
    the last of the line's eight ds_read_b128 and the first following
    global_load_lds there is a whole G step of VALU work (about 80
    instructions), and no lgkmcnt(0) wait right after the reads.  The overlap
    is worth 1.2-1.4 % of config 2 (profiles/r03_s2/ab_overlap.log)."""
    table = codeobj.disassembly(str(tmp_path))
    (body,) = codeobj.find(table, "k_chunks").values()
    reads = [i for i, ins in enumerate(body) if ins.startswith("ds_read_b128")]
    assert len(reads) >= 16  # the full-wave and the partial-wave loops
    checked = 0
    i = 0
    while i < len(reads):
        group = [reads[i]]
        while i + 1 < len(reads) and reads[i + 1] - group[-1] < 12:
            i += 1
            group.append(reads[i])
        i += 1
        if len(group) != 8:
            continue
        last = group[-1]
        nxt = next((j for j in range(last, len(body)) if body[j].startswith("global_load_lds")),
                   None)
        if nxt is None:
            continue
        between = body[last + 1:nxt]
        valu = [ins for ins in between if ins.startswith("v_")]
        assert len(valu) >= 60, (last, nxt, len(valu))
        assert "s_waitcnt lgkmcnt(0)" not in body[last + 1:last + 4], body[last + 1:last + 4]
        checked += 1
    assert checked >= 2


def test_hot_loop_instruction_budget(tmp_path):
    """k_chunks' line loop is one compression per iteration at the G-step
    floor: 96 G steps x (6 v_lshl_add_u64 + 8
    v_xor_b32 + 6 v_alignbit_b32) = 1920 VALU, rot32 free, plus under 50 of
    glue (the feed-forward as 16 v_bitop3_b32 three-way xors, the LDS read
    addresses) -- 1958 today; the PMC count per compression
    adds the per-chain set-up and exit work.  A compiler or source change that adds moves, spills or
    64-bit add pairs to the loop fails here."""
    table = codeobj.disassembly(str(tmp_path), with_addr=True)
    (body,) = codeobj.find(table, "k_chunks").values()
    at = {a: i for i, (a, _) in enumerate(body)}
    loops = []
    for i, (a, ins) in enumerate(body):
        op = ins.split()
        if not op[0].startswith("s_cbranch"):
            continue
        off = int(op[-1])
        off = off - 65536 if off > 32767 else off
        j = at.get(a + 4 + 4 * off)
        if j is not None and j < i:
            ops = [x.split()[0] for _, x in body[j:i + 1]]
            if ops.count("ds_read_b128") == 8:
                loops.append(ops)
    assert len(loops) >= 2, len(loops)  # the full-wave and the partial-wave loops
    for ops in loops:
        valu = [o for o in ops if o.startswith("v_")]
        assert ops.count("v_alignbit_b32") == 576
        assert 576 <= ops.count("v_lshl_add_u64") <= 584
        assert 768 <= ops.count("v_xor_b32_e32") + ops.count("v_xor_b32_e64") <= 776
        assert 1920 <= len(valu) <= 1970, len(valu)
        assert not any(o.startswith(("scratch_", "buffer_store", "v_readlane", "v_writelane"))
                       for o in ops)
