"""CPU: plan-specialized kernels -- the walker source
codegen.cpp emits for a plan, and its compile for gfx950 with hiprtc (no
device needed).  The GPU parity of the compiled kernels is in
tests/test_gpu_parity.py / test_gpu_messages.py ("specialized")."""
import ctypes as C
import os

import pytest

from xdrpp_amd import _abi as A
from xdrpp_amd import marshal as M
from xdrpp_amd import schemas as S


def source(plan) -> str:
    L = A.lib()
    n = C.c_size_t(0)
    rc = L.xdrg_plan_kernel_source(plan.handle, None, 0, C.byref(n))
    if rc:
        return rc
    buf = C.create_string_buffer(n.value + 1)
    assert L.xdrg_plan_kernel_source(plan.handle, buf, n.value + 1, C.byref(n)) == A.OK
    return buf.value.decode()


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
def test_source_is_straight_line(name):
    p = M.Plan(S.ALL[name])
    src = source(p)
    assert "struct plan_walk" in src and "xdrg_spec_encode" in src
    assert "load_op" not in src and "ops[" not in src  # no op table, no dispatch
    # the record-start parse of the plain-stream index (index_kernels.h)
    assert "struct plan_rx" in src and "xdrg_spec_ix_seg" in src
    if name == "rpc":
        # nested unions become switch statements with the reference's case values
        # (size, encode, decode, record parse)
        assert src.count("switch (") >= 3 * 4
        assert "XDRG_ERR_BAD_DISCRIMINANT" in src
        # every payload takes a slot, no container: the encode walks once into
        # a word list (xid, mtype, 4 call words, 2 x flavor + length)
        assert "kWords = 10u" in src
        assert "return (v == 0u || v == 1u);" in src  # first checked word: mtype
    if name == "recvar":
        assert "kWords = 7u" in src
    if name == "vecrec":
        assert "kWords = 0u" in src  # containers: the walk runs per window
        assert "for (; i < cnt; ++i)" in src
        # int vals<16>: four elements per 16-byte load (encode), two per
        # 8-byte store (decode)
        assert "i + 4u <= cnt" in src and "i + 2u <= cnt" in src


def test_index_candidate_filters():
    """The speculative record index's candidate tests (index_kernels.h
    rxs_walk_body): containertest opens with uvec<u_4_12> (unbounded), so
    its first word alone passes almost anything; the first element's
    discriminant (the next word) must be 4 or 12 when the count is nonzero."""
    src = source(M.Plan(S.ALL["containertest"]))
    assert "return (v == 0u || (w == 4u || w == 12u));" in src
    # a record whose first field is not such a container has no second test
    rpc = source(M.Plan(S.ALL["rpc"]))
    assert "bool second_ok(uint32_t v, uint32_t w) const { return true; }" in rpc
    # the staged parse keeps its first failure instead of returning early
    j = rpc.index("uint32_t rlen_st(")
    st = rpc[j:rpc.index("};", j)]
    assert "return past" not in st and "r = (r == 0u && (lim - p < 24u)) ? past : r;" in st


def test_fixed_plans_have_no_specialized_source():
    assert source(M.Plan(S.rec128)) == -3  # XDRG_EUNSUPPORTED


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
def test_source_compiles_for_gfx950(name):
    """hiprtc (or the kernel cache) yields a code object; the plan reports
    it.  Runs on the CPU: compiling touches no device."""
    p = M.Plan(S.ALL[name])
    L = A.lib()
    rc = L.xdrg_plan_build_kernels(p.handle)
    assert rc == A.OK, L.xdrg_last_hip_error().decode()
    info = A.XdrgPlanInfo()
    A.check(L.xdrg_plan_get_info(p.handle, C.byref(info)), "xdrg_plan_get_info")
    assert info.specialized == 1


# ------------------------------------------------- ahead-of-time code objects
AOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "xdrpp_amd", "aot")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
def test_aot_code_object_runs(dev, name):
    """The emitted source compiled ahead of time by hipcc --genco
    (xdrpp_amd/build.py aot_kernels), attached with xdrg_plan_load_kernels:
    its encode reproduces the reference's bytes, its decode reads them back."""
    import numpy as np
    import torch
    from conftest import golden
    co = os.path.join(AOT, f"{name}.co")
    if not os.path.exists(co):
        pytest.skip("aot code objects not built")
    code = open(co, "rb").read()
    p = M.Plan(S.ALL[name])
    L = A.lib()
    assert L.xdrg_plan_load_kernels(p.handle, code, len(code)) == A.OK
    info = A.XdrgPlanInfo()
    A.check(L.xdrg_plan_get_info(p.handle, C.byref(info)), "xdrg_plan_get_info")
    n = 1024
    nat, heap = golden(name, n, "native"), golden(name, n, "heap")
    want = golden(name, n, "xdr")
    mar = M.Marshaler(p, dev)
    r = mar.encode(torch.from_numpy(nat.copy()).to(dev), n, torch.from_numpy(heap.copy()).to(dev))
    assert np.array_equal(r.xdr.cpu().numpy(), want)
    nat2, heap2 = mar.decode(r.xdr, n, r.offsets)
    r2 = mar.encode(nat2, n, heap2)
    assert np.array_equal(r2.xdr.cpu().numpy(), want)
    A.check(L.xdrg_plan_get_info(p.handle, C.byref(info)), "xdrg_plan_get_info")
    assert info.specialized == 1


@pytest.mark.gpu
def test_foreign_code_object_refused(dev):
    """A code object compiled from another plan's source (here rpc's, given
    to recvar) is refused at load: the plan runs on the interpreter and its
    bytes stay the reference's (spec.cpp checks xdrg_spec_src_hash)."""
    import numpy as np
    import torch
    from conftest import golden
    co = os.path.join(AOT, "rpc.co")
    if not os.path.exists(co):
        pytest.skip("aot code objects not built")
    code = open(co, "rb").read()
    p = M.Plan(S.ALL["recvar"])
    L = A.lib()
    assert L.xdrg_plan_load_kernels(p.handle, code, len(code)) == A.OK
    n = 1024
    mar = M.Marshaler(p, dev)
    r = mar.encode(torch.from_numpy(golden("recvar", n, "native").copy()).to(dev), n,
                   torch.from_numpy(golden("recvar", n, "heap").copy()).to(dev))
    assert np.array_equal(r.xdr.cpu().numpy(), golden("recvar", n, "xdr"))
    info = A.XdrgPlanInfo()
    A.check(L.xdrg_plan_get_info(p.handle, C.byref(info)), "xdrg_plan_get_info")
    assert info.specialized == 0


# ------------------------------------------------- recursive plans: frame walks
@pytest.mark.parametrize("name", ["rp_list", "test_recursive"])
def test_recursive_plans_get_frame_walks(name):
    """A recursive plan (rp__list, test_recursive) gets the frame walks of
    sub_kernels.h with its ops as constants: a pc switch whose scalar fields
    fall through (one dispatch per struct), and the four frame-walk kernels
    only; hiprtc compiles it and the plan reports it specialized."""
    t = S.ALL.get(name) or S.CONTAINERS[name]
    p = M.Plan(t)
    src = source(p)
    assert "struct plan_ops" in src and "[[fallthrough]]" in src
    for k in ("xdrg_spec_sub_size", "xdrg_spec_sub_depth", "xdrg_spec_sub_encode", "xdrg_spec_sub_decode"):
        assert k in src
    assert "struct plan_walk" not in src
    L = A.lib()
    assert L.xdrg_plan_build_kernels(p.handle) == A.OK, L.xdrg_last_hip_error().decode()
    info = A.XdrgPlanInfo()
    A.check(L.xdrg_plan_get_info(p.handle, C.byref(info)), "xdrg_plan_get_info")
    assert info.specialized == 1
