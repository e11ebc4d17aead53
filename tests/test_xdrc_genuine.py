"""CPU: genuine xdrc output.  oracle/Makefile drives the reference's own
xdrc back end (xdrc/gen_hh.cc) over the AST oracle/xdrc_front.py builds
from a .x file, then compiles the reference's OWN tests against the
generated tests/xdrtest.hh: if our AST differed from what xdrc's grammar
builds, the generated traits -- and these tests -- would too.  Skipped
where the reference tree (and so oracle/_ref) is absent."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
INC = os.path.join(REF, "gen", "inc")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(INC, "tests", "xdrtest.hh")),
                                reason="oracle/_ref not built (no reference tree)")


@pytest.mark.parametrize("name", ["marshal", "validate", "stacklim", "types"])
def test_reference_tests_pass_on_generated_xdrtest_hh(name):
    """tests/marshal.cc (round trips, sizes, depth checker, containertest
    overflow), validate.cc (user hooks, enum opt-in), stacklim.cc,
    types.cc -- the reference's make-check programs, unmodified."""
    r = subprocess.run([os.path.join(REF, f"reftest_{name}")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_generated_headers_are_xdrc_output():
    for h, must in (("tests/xdrtest.hh", ["struct containertest", "struct test_recursive",
                                          "xdr_traits<::testns::numerics>"]),
                    ("xdrpp/rpc_msg.hh", ["struct rpc_msg", "_xdr_case_values", "namespace xdr"]),
                    ("bench.hh", ["struct rec128", "struct recvar", "struct vecrec"]),
                    ("validated.hh", ["namespace testns_v"])):
        text = open(os.path.join(INC, h)).read()
        assert text.startswith("// -*- C++ -*-\n// Automatically generated from"), h
        for m in must:
            assert m in text, (h, m)
