"""The C++ drop-in layer (include/xdrpp_gpu.hh) over the reference's own
xdr_traits<T>, run through oracle/_ref/dropin_test (built by oracle/Makefile
against the reference headers; skipped where it was not built).

CPU: plans recorded from xdr_traits<T> equal the plans xdrpp_amd compiles
from its Python schema mirror, op for op; host staging equals the
reference-side staged layout; the record index walk equals the
reference's offsets.
GPU: to_opaque_batch / from_opaque_batch against the reference's xdr_put /
xdr_get in the same process, and the reference's exceptions on bad input.
"""
import os
import subprocess

import numpy as np
import pytest

from xdrpp_amd import _abi as A
from xdrpp_amd import schemas as S
from xdrpp_amd.xdr_types import OP_DTYPE, compile_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "dropin_test")

pytestmark = pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/dropin_test not built")


def run(*args, timeout=300):
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)


def read_plan(path):
    raw = open(path, "rb").read()
    nops, ntab, stride, identity = np.frombuffer(raw[:16], dtype="<u4")
    ops = np.frombuffer(raw[16:16 + 32 * nops], dtype=OP_DTYPE).copy()
    tab = np.frombuffer(raw[16 + 32 * nops:16 + 32 * nops + 4 * ntab], dtype="<u4").copy()
    return ops, tab, int(stride), bool(identity)


def normalized(ops):
    """Compare wire semantics: an unvalidated enum is a 32-bit word whether
    the C++ schema declares it as an enum or as int32_t; names are ids."""
    o = ops.copy()
    o["name"] = 0
    unval = (o["kind"] == A.OP_ENUM) & ((o["flags"] & A.F_VALIDATE) == 0)
    o["kind"][unval] = A.OP_U32
    return o


def test_cpp_staging_matches_reference_layout():
    r = run("stage")
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("name", ["numerics", "numerics_validated", "rec128", "recvar", "rpc",
                                  "vecrec"])
def test_recorded_plan_equals_compiled_plan(tmp_path, name):
    r = run("plans", str(tmp_path))
    assert r.returncode == 0, r.stderr
    ops, tab, stride, identity = read_plan(tmp_path / f"{name}.plan")
    t = S.numerics_validated if name == "numerics_validated" else S.ALL[name]
    cp = compile_plan(t)
    assert stride == cp.stride
    assert np.array_equal(normalized(ops), normalized(cp.ops))
    assert np.array_equal(tab, cp.table)
    assert identity == (name in ("numerics", "numerics_validated", "rec128"))


@pytest.mark.gpu
def test_cpp_dropin_on_gpu():
    r = run("gpu", os.path.join(ROOT, "tests", "golden"), timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


# ------------------------------------- genuine xdrc output: containers_test
CBIN = os.path.join(ROOT, "oracle", "_ref", "containers_test")
needs_cbin = pytest.mark.skipif(not os.path.exists(CBIN), reason="oracle/_ref/containers_test not built")


def crun(*args, timeout=300):
    return subprocess.run([CBIN, *args], capture_output=True, text=True, timeout=timeout)


@needs_cbin
@pytest.mark.parametrize("name", list(S.CONTAINERS))
def test_containers_recorded_plan_equals_compiled_plan(tmp_path, name):
    """Element subroutines recorded from the generated xdr_traits equal the
    Python mirror's, op for op (bodies after the record's END, breadth
    first; test_recursive's elements enter the record's own ops)."""
    r = crun("plans", str(tmp_path))
    assert r.returncode == 0, r.stderr
    ops, tab, stride, identity = read_plan(tmp_path / f"{name}.plan")
    cp = compile_plan(S.CONTAINERS[name])
    assert stride == cp.stride and not identity
    assert np.array_equal(normalized(ops), normalized(cp.ops))
    assert np.array_equal(tab, cp.table)


@needs_cbin
def test_containers_staging_round_trip():
    r = crun("stage")
    assert r.returncode == 0, r.stdout + r.stderr


@needs_cbin
@pytest.mark.gpu
def test_containers_dropin_on_gpu():
    r = crun("gpu", timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
