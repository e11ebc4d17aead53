"""Launch the message path (encode_msgs, index, decode_msgs) a few times on
1M records for rocprofv3 --kernel-trace --stats (per-kernel durations).

    python tools/tune/run_msgs.py recvar rpc
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
for schema in sys.argv[1:] or ["recvar"]:
    n = 1 << 20
    plan = M.Plan(S.ALL[schema])
    mar = M.Marshaler(plan, dev)
    nat_np, heap_np = W.GENERATORS[schema](n)
    nat = torch.from_numpy(nat_np).to(dev)
    heap = torch.from_numpy(heap_np).to(dev) if heap_np.size else None
    res = mar.encode_msgs(nat, n, heap)
    maxlen = min(plan.max_record_bytes, A.INDEX_MAX_MSG)
    for _ in range(5):
        idx = M.index_messages(res.xdr, maxlen)
        mar.decode_msgs(res.xdr, n, idx)
        mar.encode_msgs(nat, n, heap)
    torch.cuda.synchronize()
    assert torch.equal(idx, res.offsets)
    print(schema, "ok", res.xdr.numel())
