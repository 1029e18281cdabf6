"""The relay hand-off's ISA assumptions, checked on the built library (CPU).

The relays (kernels.hip relay_segment: k_quad_relay, k_desc_relay and their
finishers) hand a chain value from one workgroup to the next without
acquire/release fences (those write back / invalidate the whole L2).  That
is correct only because of how the code generator emits three things, so
this test disassembles the gfx950 code object inside libciruela_amd.so and
pins them; a compiler change that breaks one fails here, not as a silently
wrong digest on the GPU:
  * the chain values are stored and loaded with sc1 (agent-scope relaxed
    atomics: written through to, and read from, the level every XCD sees);
  * the producer's `s_waitcnt vmcnt(0)` follows the two state stores and
    precedes the flag store with no memory instruction in between;
  * the consumer polls the flag with an sc1 load, waits for it
    (vmcnt(0)), reads it into a scalar and branches, and loads the chain
    values only after that loop.
"""
import re

import pytest

import codeobj


def kernels(tmp_path):
    """The relay kernels' instructions, by short name."""
    table = codeobj.disassembly(str(tmp_path))
    want = {}
    for k in ("k_quad_relay", "k_desc_relay", "k_quad_relay_finish", "k_desc_relay_finish"):
        hits = codeobj.find(table, k)
        want[k] = next(iter(hits.values())) if len(hits) == 1 else None
    return want


def idx(body, pred):
    return [i for i, ins in enumerate(body) if pred(ins)]


def is_sc1(op):
    return lambda ins: ins.split()[0] == op and re.search(r"\bsc1\b", ins) is not None


def is_vmem(ins):
    return ins.split()[0].startswith(("global_", "buffer_", "flat_"))


needs_llvm = pytest.mark.skipif(not codeobj.available(),
                                reason="needs the built library and ROCm's llvm-objdump")


@needs_llvm
@pytest.mark.parametrize("kernel", ["k_quad_relay", "k_desc_relay"])
def test_relay_publish_and_poll(tmp_path, kernel):
    body = kernels(tmp_path)[kernel]
    assert body, "kernel %s not found in the code object" % kernel
    # consumer: one sc1 flag load, polled; then the two sc1 chain-value loads
    flag_loads = idx(body, is_sc1("global_load_dword"))
    state_loads = idx(body, is_sc1("global_load_dwordx2"))
    assert len(flag_loads) == 1 and len(state_loads) == 2, (flag_loads, state_loads)
    f = flag_loads[0]
    assert all(s > f for s in state_loads)
    between = body[f + 1:min(state_loads)]
    w = idx(between, lambda ins: ins.startswith("s_waitcnt") and "vmcnt(0)" in ins)
    r = idx(between, lambda ins: ins.startswith("v_readfirstlane_b32"))
    b = idx(between, lambda ins: ins.startswith("s_cbranch"))
    assert w and r and b and w[0] < r[0] < b[0], between[:12]
    # the loop branches back to (or before) the flag load
    assert any(ins.startswith(("s_cbranch", "s_branch")) for ins in between)
    # producer: two sc1 state stores, vmcnt(0), then the sc1 flag store
    state_stores = idx(body, is_sc1("global_store_dwordx2"))
    flag_stores = idx(body, is_sc1("global_store_dword"))
    assert len(state_stores) == 2 and len(flag_stores) == 1, (state_stores, flag_stores)
    fs = flag_stores[0]
    assert all(s < fs for s in state_stores)
    tail = body[max(state_stores) + 1:fs]
    waits = idx(tail, lambda ins: ins.startswith("s_waitcnt") and "vmcnt(0)" in ins)
    assert waits, "no s_waitcnt vmcnt(0) between the state stores and the flag store"
    assert not any(is_vmem(ins) for ins in tail[waits[-1] + 1:]), tail[waits[-1]:]


@needs_llvm
@pytest.mark.parametrize("kernel", ["k_quad_relay_finish", "k_desc_relay_finish"])
def test_relay_finisher_reads_state_sc1(tmp_path, kernel):
    body = kernels(tmp_path)[kernel]
    assert body, "kernel %s not found in the code object" % kernel
    assert len(idx(body, is_sc1("global_load_dwordx2"))) == 2
