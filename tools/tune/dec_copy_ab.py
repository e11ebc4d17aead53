"""Window decode with a separate decoded heap (the stream copied into it)
vs zero-copy (heap_out == the stream): isolates the cost of the heap
stores.  Interleaved rounds, HIP events, median."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
for name in sys.argv[1:] or ["recvar", "rpc"]:
    n = 1 << 20
    p = M.Plan(S.ALL[name])
    mar = M.Marshaler(p, dev)
    nat_np, heap_np = W.GENERATORS[name](n)
    nat, heap = torch.from_numpy(nat_np).to(dev), torch.from_numpy(heap_np).to(dev)
    res = mar.encode(nat, n, heap)
    xdr, offs = res.xdr, res.offsets
    back = torch.empty_like(nat)
    hout = torch.empty(p.decode_heap_bytes(xdr.numel()), dtype=torch.uint8, device=dev)
    t = {"copy": [], "zero_copy": []}
    for _ in range(20):
        for k, h in (("copy", hout), ("zero_copy", xdr)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mar.launch_decode(xdr, n, back, offsets=offs, heap_out=h)
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1))
    mar.check()
    print(name, {k: round(float(np.median(v)), 4) for k, v in t.items()}, "ms", flush=True)
