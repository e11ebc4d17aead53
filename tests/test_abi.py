"""CPU: the C-ABI library loads and exports every symbol include/xdrgpu.h
declares; struct layouts agree between the header, ctypes and numpy; no
compute call is made (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from xdrpp_amd import _abi as A
from xdrpp_amd.xdr_types import OP_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "xdrgpu.h")


def header_functions() -> set[str]:
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(xdrg_[a-z0-9_]+)\s*\(", src))


def test_header_declares_exactly_the_exported_tuple():
    assert header_functions() == set(A.EXPORTED)


def test_library_exports_every_header_symbol():
    L = A.lib()
    for name in header_functions():
        assert hasattr(L, name), f"libxdrgpu.so does not export {name}"
    # and as dynamic symbols with C linkage (no mangling)
    out = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = header_functions() - syms
    assert not missing, missing


def test_abi_version():
    assert A.lib().xdrg_abi_version() == A.ABI_VERSION
    assert re.search(rf"#define XDRG_ABI_VERSION {A.ABI_VERSION}\b", open(HEADER).read())


LAYOUT_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "xdrgpu.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
#define Z(T) printf(#T " %zu\n", sizeof(T))
int main(void) {
  Z(xdrg_op); F(xdrg_op, kind); F(xdrg_op, flags); F(xdrg_op, depth); F(xdrg_op, noff);
  F(xdrg_op, arg0); F(xdrg_op, arg1); F(xdrg_op, arg2); F(xdrg_op, arg3); F(xdrg_op, arg4);
  F(xdrg_op, name);
  Z(xdrg_bytes_ref); F(xdrg_bytes_ref, off); F(xdrg_bytes_ref, len); F(xdrg_bytes_ref, rsv);
  Z(xdrg_plan_info); F(xdrg_plan_info, path); F(xdrg_plan_info, native_stride);
  F(xdrg_plan_info, fixed_size); F(xdrg_plan_info, max_depth); F(xdrg_plan_info, nops);
  F(xdrg_plan_info, has_checks); F(xdrg_plan_info, max_record_bytes);
  F(xdrg_plan_info, group_records); F(xdrg_plan_info, specialized);
  Z(xdrg_status); F(xdrg_status, first_error); F(xdrg_status, total_bytes);
  Z(xdrg_error); F(xdrg_error, code); F(xdrg_error, exc); F(xdrg_error, record);
  F(xdrg_error, op); F(xdrg_error, rsv); F(xdrg_error, total_bytes);
  return 0;
}
"""


def test_struct_layouts(tmp_path):
    """Header layouts (compiled with gcc) == ctypes mirrors == numpy op dtype."""
    src = tmp_path / "probe.c"
    src.write_text(LAYOUT_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in
               subprocess.run([str(exe)], capture_output=True, text=True, check=True)
               .stdout.splitlines())
    got = {k: int(v) for k, v in got.items()}
    mirrors = {"xdrg_op": A.XdrgOp, "xdrg_plan_info": A.XdrgPlanInfo,
               "xdrg_status": A.XdrgStatus, "xdrg_error": A.XdrgError}
    for cname, ct in mirrors.items():
        assert got[cname] == C.sizeof(ct), cname
        for f, _ in ct._fields_:
            assert got[f"{cname}.{f}"] == getattr(ct, f).offset, (cname, f)
    assert got["xdrg_op"] == OP_DTYPE.itemsize
    for f in OP_DTYPE.names:
        assert got[f"xdrg_op.{f}"] == OP_DTYPE.fields[f][1], f
    # staged var-length field: what the schemas lay out in native records
    assert (got["xdrg_bytes_ref"], got["xdrg_bytes_ref.off"], got["xdrg_bytes_ref.len"],
            got["xdrg_bytes_ref.rsv"]) == (16, 0, 8, 12)


def test_host_only_entry_points_need_no_device():
    L = A.lib()
    assert L.xdrg_error_message(0).decode() == ""
    assert L.xdrg_error_message(999).decode() != ""


def test_product_fails_loudly_without_the_library(tmp_path, monkeypatch):
    """No CPU fallback: a missing .so is an ImportError, not a silent path."""
    monkeypatch.setattr(A, "_lib", None)
    monkeypatch.setattr(A, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(ImportError):
        A.lib()


def test_no_oracle_in_product_package():
    """The product package never imports the oracle or the reference."""
    pkg = os.path.join(ROOT, "xdrpp_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle_bridge" not in txt and "liboracle" not in txt, f
                assert "/root/reference" not in txt, f


def _create(ops: np.ndarray, stride: int):
    L = A.lib()
    h = C.c_void_p()
    rc = L.xdrg_plan_create(ops.ctypes.data_as(C.POINTER(A.XdrgOp)), len(ops), None, 0, stride,
                            C.byref(h))
    return rc, h


def test_plan_op_count_limit():
    """Status keys carry a 16-bit op index (0xffff = record level): a plan of
    65535 or more ops is refused, one just below the limit is accepted."""
    L = A.lib()
    for nops, want in ((0xFFFE, A.OK), (0xFFFF, -3), (0x10000, -3)):
        ops = np.zeros(nops, dtype=OP_DTYPE)
        ops["kind"] = A.OP_U32
        ops["noff"] = 0
        ops["depth"] = 1
        ops[-1]["kind"] = A.OP_END
        rc, h = _create(ops, 4)
        assert rc == want, (nops, rc)
        if rc == A.OK:
            L.xdrg_plan_destroy(h)


def test_plan_options_are_per_plan_and_validated():
    """Launch options live on the plan (no process-global knobs): unknown
    options and out-of-range values are refused."""
    from xdrpp_amd import marshal as M
    from xdrpp_amd import schemas as S
    L = A.lib()
    p = M.Plan(S.recvar, {"var_encode_kernel": 1, "image_bytes": 2048})
    assert L.xdrg_plan_set_option(p.handle, 999, 0) == -1
    assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["var_encode_kernel"], 2) == -1
    assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["enc_unroll"], 5) == -1
    assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["enc_unroll"], 16) == A.OK
    for v in (0, 1, 2, 3):  # record index: list ranking / host-gated walk / asynchronous walk / walk only
        assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["index_fast"], v) == A.OK
    assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["index_fast"], 4) == -1
    for v in (-1, 0, 8192, 32768):  # LDS stage of a group's element arrays
        assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["stage_bytes"], v) == A.OK
    assert L.xdrg_plan_set_option(p.handle, A.PLAN_OPTIONS["stage_bytes"], 32769) == -1
    with pytest.raises(A.AbiError):
        M.Plan(S.recvar, {"var_decode_kernel": 7})


def test_no_tuning_hooks_exported():
    """Nothing but the header's entry points is exported with the xdrg_
    prefix (no process-global tuning knobs)."""
    out = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert {s for s in syms if s.startswith("xdrg")} == set(A.EXPORTED)
