"""A/B the var-path kernel families (group-copy vs record-image) in one
process, interleaved (cdna_hip_programming.md §5.4 rule 24)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

# (encode kernel, decode kernel, encode LDS image bytes, decode LDS window
# bytes[, encode unroll, decode read-ahead]) as plan options
# (xdrg_plan_set_option): kernels 0 auto, 1 per-lane, 3 chunk-map image
# (encode) / 2 window (decode); -1 bytes = automatic
VARIANTS = [tuple(int(x) for x in v.split(",")) for v in
            os.environ.get("VARIANTS", "3,2,-1,-1 3,2,4096,4096 3,2,0,4096 3,2,4096,2048 1,1,-1,-1").split()]


def options(v):
    return {"var_encode_kernel": v[0], "var_decode_kernel": v[1], "image_bytes": v[2],
            "window_bytes": v[3], "enc_unroll": v[4] if len(v) > 4 else 8,
            "dec_readahead": v[5] if len(v) > 5 else 1}


dev = torch.device("cuda:0")
out = {}
for schema in sys.argv[1:] or ["recvar", "rpc"]:
    n = 1 << 20
    plan = M.Plan(S.ALL[schema])
    mar = M.Marshaler(plan, dev)
    mars = {v: M.Marshaler(M.Plan(S.ALL[schema], options(v)), dev) for v in VARIANTS}
    nat_np, heap_np = W.GENERATORS[schema](n)
    nat = torch.from_numpy(nat_np).to(dev)
    heap = torch.from_numpy(heap_np).to(dev)
    total = int(mar.serial_sizes(nat, n).to(torch.int64).sum().item())
    xdr = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    back = torch.empty_like(nat)
    hout = torch.empty(plan.decode_heap_bytes(total), dtype=torch.uint8, device=dev)
    ref = None
    s = torch.cuda.current_stream().cuda_stream
    times = {v: ([], []) for v in VARIANTS}
    for v in VARIANTS:  # correctness + warmup
        mar = mars[v]
        mar.status.init(s)
        mar.launch_encode(nat, n, xdr, heap=heap, offsets=offs)
        mar.launch_decode(xdr, n, back, offsets=offs, heap_out=hout)
        mar.check()
        x = xdr.clone()
        ref = x if ref is None else ref
        assert torch.equal(x, ref), f"{schema}: variant {v} encode differs"
        x2 = torch.empty_like(xdr)
        mar.launch_encode(back, n, x2, heap=hout, offsets=offs)
        mar.check()
        assert torch.equal(x2, ref), f"{schema}: variant {v} decode->encode differs"
    for rnd in range(5):
        for v in VARIANTS:
            mar = mars[v]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            for _ in range(5):
                mar.launch_encode(nat, n, xdr, heap=heap, offsets=offs)
            ev[1].record()
            for _ in range(5):
                mar.launch_decode(xdr, n, back, offsets=offs, heap_out=hout)
            ev[2].record()
            torch.cuda.synchronize()
            times[v][0].append(ev[0].elapsed_time(ev[1]) / 5)
            times[v][1].append(ev[1].elapsed_time(ev[2]) / 5)
    for m in mars.values():
        m.check()
    for v in VARIANTS:
        name = f"e{v[0]}d{v[1]}_i{v[2] // 1024}K_w{v[3] // 1024}K" + (f"_u{v[4]}" if len(v) > 4 else "") + (f"_ra{v[5]}" if len(v) > 5 else "")
        e, d = float(np.median(times[v][0])), float(np.median(times[v][1]))
        out[f"{schema}_{name}"] = {"encode_ms": round(e, 4), "decode_ms": round(d, 4),
                                   "gib_s": round(2 * total / 2**30 / ((e + d) * 1e-3), 1)}
        print(schema, name, out[f"{schema}_{name}"])
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "ab_var.json"), "w"), indent=1)
