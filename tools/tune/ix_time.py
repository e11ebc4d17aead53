"""Record index of an encoded 1M batch, REPS calls (for rocprofv3 --stats):
the walk's kernels and the host gate between them.

    rocprofv3 --kernel-trace --stats -d OUT -- python tools/tune/ix_time.py rpc
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
dev = torch.device("cuda:0")
L = A.lib()
for name in sys.argv[1:] or ["rpc"]:
    n = 1 << 20
    p = M.Plan(S.ALL[name], {"index_fast": int(os.environ.get("FAST", "1"))})
    mar = M.Marshaler(p, dev)
    nat, heap = (torch.from_numpy(a).to(dev) for a in W.GENERATORS[name](n))
    enc = mar.encode(nat, n, heap)
    total = enc.xdr.numel()
    maxlen = min(p.max_record_bytes, A.INDEX_MAX_MSG)
    ws = torch.zeros(L.xdrg_index_workspace_size(total, maxlen), dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(REPS + 3):
        mar.status.init(s)
        e0.record()
        A.check(L.xdrg_index_records(p.handle, enc.xdr.data_ptr(), total, n, maxlen, offs.data_ptr(),
                                     cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index")
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1))
    assert torch.equal(offs, enc.offsets), name
    ts.sort()
    print(name, f"index median {ts[len(ts) // 2]:.4f} ms min {ts[0]:.4f}", flush=True)
