"""The XDR-language front end (oracle/xdrc_front.py, test infrastructure)
and the plans it yields.  CPU only: parsing, plan equality with the hand-written descriptors,
the reference's own .x files when the reference tree is present, and the
emitted C header compiled and run against libxdrgpu.so's host-only plan
creation (no GPU call)."""
import os
import subprocess
import textwrap

import numpy as np
import pytest

from conftest import ROOT

from xdrpp_amd import _abi as A
from xdrpp_amd import marshal as M
from xdrpp_amd import rpc as R
from xdrpp_amd import schemas as S
import xdrc_front as xdrc  # noqa: E402  (oracle/, test infrastructure)
from xdrpp_amd.xdr_types import compile_plan

REF = "/root/reference"
BENCH_X = os.path.join(ROOT, "oracle", "x", "bench.x")


def same_plan(a, b):
    return (np.array_equal(a.ops, b.ops) and np.array_equal(a.table, b.table)
            and a.stride == b.stride and a.fixed_size == b.fixed_size and a.messages == b.messages)


@pytest.mark.parametrize("name", ["rec128", "recvar", "vecrec"])
def test_bench_x_equals_descriptors(name):
    sp = xdrc.load_file(BENCH_X)
    assert same_plan(sp.plan(name), compile_plan(S.ALL[name]))


@pytest.mark.skipif(not os.path.exists(f"{REF}/xdrpp/rpc_msg.x"), reason="reference tree absent")
def test_reference_rpc_msg_x():
    sp = xdrc.load_file(f"{REF}/xdrpp/rpc_msg.x")
    assert same_plan(sp.plan("rpc_msg"), compile_plan(S.rpc_msg))
    assert sp.consts["AUTH_SYS"] == 1 and sp.consts["MSG_DENIED"] == 1


@pytest.mark.skipif(not os.path.exists(f"{REF}/tests/xdrtest.x"), reason="reference tree absent")
def test_reference_xdrtest_x():
    sp = xdrc.load_file(f"{REF}/tests/xdrtest.x")
    assert same_plan(sp.plan("numerics"), compile_plan(S.numerics))
    # all 28 types plan: containers of variable-size elements and the
    # recursive test_recursive through element subroutines (XDRG_F_SUB)
    assert len(sp.types) == 28
    for n in sp.types:
        M.Plan(sp.plan(n)).close()
    tr = sp.plan("test_recursive")
    sub = [o for o in tr.ops if o["kind"] == A.OP_VECTOR]
    assert len(sub) == 2 and all(o["flags"] & A.F_SUB and o["arg4"] == 0 for o in sub)
    t = sp.proc_table()
    assert t[:, :3].tolist() == [[0x20000000, 1, 1], [0x20000000, 1, 2], [0x20000000, 2, 1],
                                 [0x20000000, 2, 2], [0x20000000, 2, 3], [0x20000000, 2, 4],
                                 [0x20000001, 1, 1], [0x20000001, 1, 2]]
    assert any("operator" in lit for lit in sp.literals)


GRAMMAR = textwrap.dedent("""
    %#include <something.h>
    /* comment */ const N = 0x10;   // trailing comment
    const M = -3;
    enum color { RED = 0, GREEN = 2, BLUE, };
    typedef opaque blob<N>;
    typedef string name<>;
    typedef int quad[4];
    namespace outer {
    struct point { hyper x; hyper y; };
    }
    union tagged switch (color c) {
      case RED:
      case GREEN:
        point p;
      case BLUE:
        void;
      default:
        unsigned hyper raw;
    };
    union flag switch (bool b) { case TRUE: int v; case FALSE: void; };
    struct rec {
      quad q;
      blob data;
      name who;
      union switch (int k) { case M: int neg; case 1: double pos; } body;
      enum { A = 1, B = 2 } e;
      struct { int u; int v; } inner;
      outer::point *maybe;
      tagged t;
      flag f;
      bool bits[3];
      string plain;
    };
    program P { version V1 { void NULLPROC(void) = 0; rec GET(int, hyper) = 7; } = 1;
                version V2 { int X(rec) = 3; } = 2; } = 400000;
""")


def test_grammar_features():
    sp = xdrc.load(GRAMMAR)
    rec = sp.types["rec"]
    names = dict(rec.fields)
    assert names["body"].name == "_body_t" and names["e"].name == "_e_t"
    assert names["inner"].name == "_inner_t"
    assert sp.consts["BLUE"] == 3 and sp.consts["N"] == 16
    cp = sp.plan("rec")
    assert cp.is_var
    assert "bad value of k in _body_t" in cp.messages.values()
    assert "bad value of b in flag" in cp.messages.values()
    assert sp.literals == ["#include <something.h>"]
    t = sp.proc_table()
    assert t.tolist() == [[400000, 1, 0, 0], [400000, 1, 7, 0], [400000, 2, 3, 0]]
    M.Plan(cp).close()  # the C ABI accepts it (host-only validation)


@pytest.mark.parametrize("src,msg", [
    ("union u switch (int x) { default: int a; default: int b; };", "duplicate default"),
    ("struct s { char c; };", "reserved word"),
    ("struct s { nosuch x; };", "unknown type"),
    ("struct s { int x };", "expected"),
    ("struct s { int x[NOPE]; };", "unknown constant"),
    ("struct s { quadruple q; };", "quadruple"),
])
def test_grammar_errors(src, msg):
    with pytest.raises(xdrc.XdrcError, match=msg):
        xdrc.load(src)


def test_emitted_header_compiles_and_creates_plans(tmp_path):
    """The plan emitted at generation time is the plan the runtime builds:
    a C program includes the emitted header, creates every plan through
    libxdrgpu.so (host-only) and prints its info; it must equal the info of
    the same type's runtime-compiled plan."""
    sp = xdrc.load(open(BENCH_X).read() + GRAMMAR)
    types = ["rec128", "recvar", "vecrec", "rec", "tagged"]
    hdr = tmp_path / "plans.h"
    hdr.write_text(xdrc.emit_plan_header(sp, types))
    prog = tmp_path / "main.c"
    body = "\n".join(
        f'  {{ xdrg_plan *p = 0; xdrg_plan_info i; if (xdrg_plan_create_{t}(&p)) return 1;'
        f' xdrg_plan_get_info(p, &i);'
        f' printf("{t} %u %u %u %u %u\\n", i.path, i.native_stride, i.fixed_size, i.max_depth, i.nops);'
        f' xdrg_plan_destroy(p); }}' for t in types)
    prog.write_text('#include <stdio.h>\n#include "plans.h"\nint main(void) {\n' + body +
                    "\n  printf(\"procs %u\\n\", XDRG_EMITTED_NPROCS);\n  return 0;\n}\n")
    exe = tmp_path / "main"
    libdir = os.path.join(ROOT, "xdrpp_amd")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-Wno-unused-const-variable",
                           "-I", os.path.join(ROOT, "include"), "-I", str(tmp_path), "-o", str(exe),
                           str(prog), "-L", libdir, "-lxdrgpu", f"-Wl,-rpath,{libdir}"])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    for t, line in zip(types, out):
        p = M.Plan(sp.plan(t))
        i = A.XdrgPlanInfo()
        A.check(A.lib().xdrg_plan_get_info(p.handle, A.C.byref(i)), "info")
        assert line == f"{t} {i.path} {i.native_stride} {i.fixed_size} {i.max_depth} {i.nops}"
    assert out[len(types)] == f"procs {len(sp.proc_table())}"


def test_cli(tmp_path):
    out = tmp_path / "b.h"
    subprocess.check_call(["python", os.path.join(ROOT, "oracle", "xdrc_front.py"), BENCH_X, "-o",
                           str(out), "rec128"], cwd=ROOT)
    assert "xdrg_plan_create_rec128" in out.read_text()
