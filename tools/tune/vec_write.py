"""Where the vecrec decode's extra writes come from: the same decode with
its own heap (the stream copied verbatim, then the element arrays) and
zero-copy (heap_out == the stream: element arrays only), 5 launches each,
for rocprofv3 --pmc WRITE_SIZE (kernel names: xdrg_spec_decode_copy /
xdrg_spec_decode).    python tools/tune/vec_write.py [schema]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
name = sys.argv[1] if len(sys.argv) > 1 else "vecrec"
n = 1 << 20
plan = M.Plan(S.ALL[name])
mar = M.Marshaler(plan, dev)
nat, heap = (torch.from_numpy(a).to(dev) for a in W.GENERATORS[name](n))
enc = mar.encode(nat, n, heap)
L = enc.xdr.numel()
H = plan.decode_heap_bytes(L)
back = torch.empty_like(nat)
hout = torch.empty(H, dtype=torch.uint8, device=dev)
big = torch.empty(H, dtype=torch.uint8, device=dev)
big[:L].copy_(enc.xdr)
s = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    mar.launch_decode(enc.xdr, n, back, offsets=enc.offsets, heap_out=hout, stream=s)
for _ in range(5):
    mar.launch_decode(big[:L], n, back, offsets=enc.offsets, heap_out=big, stream=s)
torch.cuda.synchronize()
mar.check(s)
print(name, "stream", L, "heap", H, "native", back.numel())
