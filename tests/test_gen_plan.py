"""Device plans emitted at generation time by the product's xdrc back end
(xdrpp_amd/gen/gen_plan.cc, `xdrc -plan`), run inside the
reference's xdrc driver over its AST (oracle/xdrc_driver.cc, built with
XDRC_PLAN by oracle/Makefile `plans`).

CPU: for every struct and union of tests/xdrtest.x (28 types), xdrpp/rpc_msg.x,
xdrpp/rpcb_prot.x and the oracle's bench/validated files, the emitted op
table, case/enum table, stride, fixed size and bad-discriminant messages
equal the plan the Python compiler builds from the same .x file; the C part
of a header compiles as C11 and creates its plans through libxdrgpu.so;
and the C++ part (xdr::gpu::emitted_plan<T>) equals the plan recorded from
the reference's xdr_traits<T>, with plan_for<T>() recording nothing
(oracle/_ref/emitted_test plans).
GPU: to_opaque_batch / from_opaque_batch through emitted plans and their
ahead-of-time kernels against the reference's xdr_put / xdr_get
(oracle/_ref/emitted_test gpu)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

from xdrpp_amd import _abi as A
from xdrpp_amd import marshal as M
from xdrpp_amd.xdr_types import OP_DTYPE
import xdrc_front as xdrc  # noqa: E402  (oracle/, test infrastructure)

REF = "/root/reference"
PLAN = os.path.join(ROOT, "oracle", "_ref", "gen", "plan")
BIN = os.path.join(ROOT, "oracle", "_ref", "emitted_test")
FILES = {  # plan header -> (.x file, enums that opt in to validation)
    "xdrtest_plan.hh": (f"{REF}/tests/xdrtest.x", ()),
    "rpc_msg_plan.hh": (f"{REF}/xdrpp/rpc_msg.x", ()),
    "rpcb_prot_plan.hh": (f"{REF}/xdrpp/rpcb_prot.x", ()),
    "bench_plan.hh": (os.path.join(ROOT, "oracle", "x", "bench.x"), ()),
    "validated_plan.hh": (os.path.join(ROOT, "oracle", "x", "validated.x"), ("other_color",)),
}

needs_plans = pytest.mark.skipif(not os.path.exists(os.path.join(PLAN, "xdrtest_plan.hh")),
                                 reason="oracle/_ref/gen/plan not built (make -C oracle plans)")

_BLOCK = re.compile(
    r"/\* (\S+): (\d+) ops, stride (\d+), (?:fixed (\d+) wire bytes|variable length) \*/\n"
    r"static const xdrg_op xdrg_plan_(\w+)_ops\[\d+\] = \{\n(.*?)\};\n"
    r"static const uint32_t xdrg_plan_\w+_table\[\d+\] = \{\n(.*?)\};\n"
    r"#define XDRG_PLAN_\w+_NOPS \d+u\n#define XDRG_PLAN_\w+_NTABLE (\d+)u\n"
    r"#define XDRG_PLAN_\w+_STRIDE \d+u\n#define XDRG_PLAN_\w+_FIXED_SIZE \d+u\n"
    r"(?:static const struct \{ uint32_t op; const char \*what; \} xdrg_plan_\w+_union_msgs\[\d+\] = \{\n(.*?)\};\n)?",
    re.S)


def emitted(header):
    """{type name: (ops, table, stride, fixed_size, messages, C name)} of a plan header."""
    text = open(os.path.join(PLAN, header)).read()
    out = {}
    for m in _BLOCK.finditer(text):
        name, nops, stride, fixed, c, ops_s, tab_s, ntab, msgs_s = m.groups()
        rows = [[int(v.rstrip("u")) for v in r.strip(" {},").split(", ")] for r in ops_s.strip().split("\n")]
        ops = np.array([tuple(r) for r in rows], dtype=OP_DTYPE)
        assert len(ops) == int(nops)
        tab = np.array([int(v.rstrip("u")) for v in tab_s.replace(",", " ").split()], dtype=np.uint32)[:int(ntab)]
        msgs = dict((int(a), b) for a, b in re.findall(r'\{(\d+)u, "([^"]*)"\}', msgs_s or ""))
        out[name] = (ops, tab, int(stride), int(fixed) if fixed else None, msgs, c)
    return out


@needs_plans
@pytest.mark.parametrize("header", list(FILES))
def test_emitted_plans_equal_compiled(header):
    x, validate = FILES[header]
    if not os.path.exists(x):
        pytest.skip(f"{x} absent")
    sp = xdrc.load_file(x, validate_enums=validate)
    em = emitted(header)
    want = [n for n, t in sp.types.items() if type(t).__name__ in ("Struct", "Union")]
    assert sorted(em) == sorted(want)
    if header == "xdrtest_plan.hh":
        assert len(want) >= 20  # every struct and union of the reference's 28 types
    for n in want:
        cp = sp.plan(n)
        ops, tab, stride, fixed, msgs, _ = em[n]
        assert np.array_equal(ops, cp.ops), n
        assert np.array_equal(tab, cp.table), n
        assert stride == cp.stride and fixed == cp.fixed_size, n
        assert msgs == cp.messages, n


@needs_plans
def test_emitted_header_is_c_and_creates_plans(tmp_path):
    """The C part of a plan header: compiles as C11 (no C++ section without
    __cplusplus) and every create function builds its plan in libxdrgpu.so
    (host-only) with the info of the same type's runtime-compiled plan."""
    em = emitted("xdrtest_plan.hh")
    sp = xdrc.load_file(FILES["xdrtest_plan.hh"][0])
    body = "\n".join(
        f'  {{ xdrg_plan *p = 0; xdrg_plan_info i; if (xdrg_plan_create_{c}(&p)) return 1;'
        f' xdrg_plan_get_info(p, &i);'
        f' printf("{n} %u %u %u %u %u\\n", i.path, i.native_stride, i.fixed_size, i.max_depth, i.nops);'
        f' xdrg_plan_destroy(p); }}' for n, (*_, c) in em.items())
    prog = tmp_path / "main.c"
    prog.write_text('#include <stdio.h>\n#include "xdrtest_plan.hh"\nint main(void) {\n' + body + "\n  return 0;\n}\n")
    exe = tmp_path / "main"
    libdir = os.path.join(ROOT, "xdrpp_amd")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-Wno-unused-const-variable", "-x", "c",
                           "-I", os.path.join(ROOT, "include"), "-I", PLAN, "-o", str(exe), str(prog),
                           "-L", libdir, "-lxdrgpu", f"-Wl,-rpath,{libdir}"])
    lines = subprocess.check_output([str(exe)], text=True).strip().split("\n")
    assert len(lines) == len(em)
    for line in lines:
        n = line.split()[0]
        p = M.Plan(sp.plan(n))
        i = A.XdrgPlanInfo()
        A.check(A.lib().xdrg_plan_get_info(p.handle, A.C.byref(i)), "info")
        assert line == f"{n} {i.path} {i.native_stride} {i.fixed_size} {i.max_depth} {i.nops}"


@needs_plans
def test_emitted_kernel_sources_are_the_plans():
    """The kernel sources xdrc -plan -kernels wrote are what the library
    generates for the same plan (xdrg_plan_kernel_source)."""
    import ctypes as C
    for header, typ in (("bench_plan.hh", "recvar"), ("rpc_msg_plan.hh", "rpc_msg"),
                        ("xdrtest_plan.hh", "containertest"), ("xdrtest_plan.hh", "hasbytes")):
        x, validate = FILES[header]
        if not os.path.exists(x):
            continue
        c = emitted(header)[typ][5]
        src = open(os.path.join(PLAN, "kernels", f"{c}.hip")).read()
        p = M.Plan(xdrc.load_file(x, validate_enums=validate).plan(typ))
        n = C.c_size_t(0)
        A.check(A.lib().xdrg_plan_kernel_source(p.handle, None, 0, C.byref(n)), "size")
        buf = C.create_string_buffer(n.value + 1)
        A.check(A.lib().xdrg_plan_kernel_source(p.handle, buf, n.value + 1, C.byref(n)), "source")
        assert buf.value.decode() == src, typ
        assert os.path.exists(os.path.join(PLAN, "kernels", f"{c}.co")), c


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/emitted_test not built")
def test_cpp_emitted_plans_equal_recorded():
    r = subprocess.run([BIN, "plans"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "emitted plans equal the recorded ones" in r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/emitted_test not built")
def test_cpp_emitted_plans_on_gpu():
    env = dict(os.environ, XDRG_PLAN_KERNEL_DIR=os.path.join(PLAN, "kernels"))
    r = subprocess.run([BIN, "gpu"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("bit-exact through the emitted plan") == 9, r.stdout
