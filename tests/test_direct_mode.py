"""Direct mode of the plan-specialized encode (var_kernels.h
enc_direct_ctx): a wave whose 64 records could pass 2 GiB of stream (a
record of 32 MiB or more, possible only in plans with unbounded fields)
writes its records straight to the stream.  The reference has no record
size limit (xdr_generic_put checks capacity only, xdrpp/marshal.h:84-137);
the C restatement is the checker."""
import numpy as np
import pytest

from xdrpp_amd import objects as OB
from xdrpp_amd.xdr_types import Opaque, String, Struct, UInt, XVector, compile_plan
import oracle_bridge as O

big = Struct("big", [("id", UInt), ("data", Opaque()), ("tags", XVector(String(8)))])
MIB = 1 << 20


def values(sizes):
    rng = np.random.default_rng(5)
    return [{"id": i, "data": rng.integers(0, 256, s, dtype=np.uint8).tobytes(),
             "tags": [b"t%d" % j for j in range(i % 3)]} for i, s in enumerate(sizes)]


def test_oracle_encodes_a_33_mib_record():
    vals = values([3, 33 * MIB + 5, 0])
    nat, heap = OB.stage(big, vals)
    x, offs = O.encode(compile_plan(big), nat, len(vals), heap)
    assert int(offs[2] - offs[1]) == 4 + 4 + 33 * MIB + 8 + 4 + 4 + 4


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [[3, 33 * MIB + 5, 0, 70], [32 * MIB] + [17] * 70, [5] * 130])
def test_gpu_direct_mode_matches_oracle(dev, sizes):
    import torch
    from xdrpp_amd import marshal as M
    vals = values(sizes)
    n = len(vals)
    nat, heap = OB.stage(big, vals)
    cp = compile_plan(big)
    want, woffs = O.encode(cp, nat, n, heap)
    mar = M.Marshaler(M.Plan(big), dev)
    r = mar.encode(torch.from_numpy(nat).to(dev), n, torch.from_numpy(heap).to(dev))
    assert torch.equal(r.offsets.cpu(), torch.from_numpy(woffs.view(np.int64)))
    assert np.array_equal(r.xdr.cpu().numpy(), want)
    nat2, heap2 = mar.decode(r.xdr, n, r.offsets)
    assert OB.unstage(big, nat2.cpu().numpy(), heap2.cpu().numpy(), n) == vals
