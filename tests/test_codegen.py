"""CPU: plan-specialized kernels -- the walker source
codegen.cpp emits for a plan, and its compile for gfx950 with hiprtc (no
device needed).  The GPU parity of the compiled kernels is in
tests/test_gpu_parity.py / test_gpu_messages.py ("specialized")."""
import ctypes as C

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
    if name == "rpc":
        # nested unions become switch statements with the reference's case values
        assert src.count("switch (") >= 2 * 4
        assert "XDRG_ERR_BAD_DISCRIMINANT" in src
    if name == "vecrec":
        assert "for (uint32_t i = 0; i < cnt; ++i)" in src


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
