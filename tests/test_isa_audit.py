"""The pipelined encode windows' explicit wait is right in the compiled
code of the benchmark plans (tools/isa_audit.py: the SW buffer stores, and
nothing else, between the asm payload loads and s_waitcnt vmcnt(SW))."""
import os
import sys
import tempfile

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_audit  # noqa: E402


@pytest.mark.parametrize("schema,want", [("recvar", 1), ("rpc", 1), ("vecrec", 0), ("containertest", 0)])
def test_pipelined_window_wait(schema, want):
    """Every sequence is safe in every encode kernel of the plan (the
    windowed one and the walk-first ones); recvar and rpc overlap their
    loads for real."""
    with tempfile.TemporaryDirectory() as d:
        kernels = isa_audit.kernel_asm(schema, d)
        assert "xdrg_spec_encode" in kernels
        for name, lines in kernels.items():
            checked, effective = isa_audit.audit(lines)
            assert effective >= want, name
