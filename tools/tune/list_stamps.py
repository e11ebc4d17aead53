"""Cycle stamps of the wave pass's list decode (sub_kernels.h list_decode,
built with XDRG_LIST_STAMPS): 16 lists of 500 nodes, rp__list, decoded
with the plan-specialized kernels (printf per list: nodes, batches, block
loads, cycles in all / batch checks / batch writes / block loads)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
import test_deep as T  # noqa: E402
import oracle_bridge as O  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402

dev = torch.device("cuda:0")
lens = [500] * 16 + [2, 3]
chains = T.chain_lists(lens)
n, cp = len(chains), T.plan_of("rp__list")
nat, heap = T.stage_chains("rp__list", chains)
x, offs = O.encode(cp, nat, n, heap)
spec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
mar = M.Marshaler(M.Plan(S.rp__list, {"specialize": spec}), dev)
dx, do = torch.from_numpy(x).to(dev), torch.from_numpy(offs.astype(np.int64)).to(dev)
for _ in range(2):
    a, h = mar.decode(dx, n, do)
torch.cuda.synchronize()
onat, oheap = O.decode(cp, x, n, offs)
print("ok", np.array_equal(a.cpu().numpy(), onat) and np.array_equal(h.cpu().numpy(), oheap))
