"""A/B of decode plan options (GPU box): the window decode of one schema,
1M records, per option set of VALS (space-separated sets of name=value,
comma-joined; "-" = the defaults), timed with HIP events over 20 launches
(median), its native records and heap compared with the first set's (both
heaps zeroed first).
    VALS="stage_bytes=0 stage_bytes=8192,window_bytes=8192" python tools/tune/dec_ab.py vecrec
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
name = sys.argv[1] if len(sys.argv) > 1 else "vecrec"
vals = os.environ.get("VALS", "- stage_bytes=0").split()


def opts(v):
    return {} if v == "-" else {k: int(x) for k, x in (kv.split("=") for kv in v.split(","))}


n = 1 << 20
base = M.Plan(S.ALL[name])
m0 = M.Marshaler(base, dev)
nat, heap = (torch.from_numpy(a).to(dev) for a in W.GENERATORS[name](n))
enc = m0.encode(nat, n, heap)
L = enc.xdr.numel()
H = base.decode_heap_bytes(L)
s = torch.cuda.current_stream().cuda_stream
ref = None
for v in vals:
    mar = M.Marshaler(M.Plan(S.ALL[name], opts(v)), dev)
    back = torch.zeros_like(nat)
    hout = torch.zeros(H, dtype=torch.uint8, device=dev)
    mar.status.init(s)
    mar.launch_decode(enc.xdr, n, back, offsets=enc.offsets, heap_out=hout, stream=s)
    try:
        mar.check(s)
    except M.XdrRuntimeError as e:
        print(f"{name} {v} FAILED: {e} record {e.record} op {e.op}", flush=True)
        continue
    same = None
    if ref is None:
        ref = (back.clone(), hout.clone())
    else:
        same = bool(torch.equal(ref[0], back)) and bool(torch.equal(ref[1], hout))
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mar.launch_decode(enc.xdr, n, back, offsets=enc.offsets, heap_out=hout, stream=s)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print(f"{name} {v} decode_ms {ts[len(ts) // 2]:.4f} min {ts[0]:.4f} same_as_first {same}", flush=True)
