"""A/B of the var encode's LDS window (plan option image_bytes) on the
plan-specialized kernels, interleaved in one process, bytes checked.
    python tools/tune/ab_img.py recvar rpc   (IMGS="-1 2048 3072")"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
IMGS = [int(x) for x in os.environ.get("IMGS", "-1 2048 3072").split()]
for name in sys.argv[1:] or ["recvar", "rpc"]:
    n = 1 << 20
    nat, heap = (torch.from_numpy(a).to(dev) for a in W.GENERATORS[name](n))
    mars = {i: M.Marshaler(M.Plan(S.ALL[name], {"image_bytes": i}), dev) for i in IMGS}
    ref = mars[IMGS[0]].encode(nat, n, heap)
    out = torch.empty_like(ref.xdr)
    offs = torch.empty_like(ref.offsets)
    s = torch.cuda.current_stream().cuda_stream
    t = {i: [] for i in IMGS}
    for i, m in mars.items():
        m.status.init(s)
        m.launch_encode(nat, n, out, heap=heap, offsets=offs, stream=s)
        m.check(s)
        assert torch.equal(out, ref.xdr) and torch.equal(offs, ref.offsets), (name, i)
    for _ in range(7):
        for i, m in mars.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                m.launch_encode(nat, n, out, heap=heap, offsets=offs, stream=s)
            e1.record()
            torch.cuda.synchronize()
            t[i].append(e0.elapsed_time(e1) / 5)
    print(name, {i: round(float(np.median(v)), 4) for i, v in t.items()}, flush=True)
