"""A/B the group-path launch shape (k_fixed_grp) on numerics 1M encode and
decode: U chunks in flight, workgroup cap, nontemporal stores.  Interleaved
rounds in one process; HIP events around each launch, median."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
n = int(os.environ.get("TUNE_N", 1 << 20))
p = M.Plan(S.numerics)
mar = M.Marshaler(p, dev)
nat = torch.from_numpy(W.numerics(n)[0]).to(dev)
xdr = torch.empty(n * 44, dtype=torch.uint8, device=dev)
back = torch.empty_like(nat)
s = torch.cuda.current_stream().cuda_stream
ref = mar.encode(nat, n).xdr.clone()
variants = [(u, b, nt) for u in (1, 2, 4) for b in (1024, 2048, 4096, 8192, 16384) for nt in (0, 1)]
res = {v: ([], []) for v in variants}
mars = {v: M.Marshaler(M.Plan(S.numerics, {"grp_unroll": v[0], "grp_blocks": v[1], "grp_nontemporal": v[2]}),
                       dev) for v in variants}
for rnd in range(15):
    for v in variants:
        m = mars[v]
        for k, f in ((0, lambda: m.launch_encode(nat, n, xdr, stream=s)),
                     (1, lambda: m.launch_decode(xdr, n, back, stream=s))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            res[v][k].append(e0.elapsed_time(e1))
        if rnd == 0:
            assert torch.equal(xdr, ref) and torch.equal(back, nat), v
alg = n * 100
rows = sorted(((np.median(a) + np.median(b)) / 2, v, np.median(a), np.median(b)) for v, (a, b) in res.items())
for t, v, a, b in rows:
    print(f"U={v[0]} blocks={v[1]:5d} nt={v[2]}  enc {a*1e3:6.1f} us  dec {b*1e3:6.1f} us  "
          f"avg {t*1e3:6.1f} us = {alg / (t * 1e-3) / 1e12:.2f} TB/s")
