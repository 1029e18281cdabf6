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
