"""k_fixed_reg launch shapes (XDRG_OPT_FIXED_STREAM) across batch sizes
past the Infinity Cache: where does the non-temporal 1024-workgroup loop stop
beating the non-temporal one-shot grid?  rec128 encode + decode, HIP events
around each kernel, median of 15 after 2 untimed; random record bytes (the
round trip is checked, not the reference's hash: bench.py does that).

  python tools/gpu/fixed_shape_sweep.py [records_in_M,...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402

SHAPES = {-1: "default", 0: "plain/1024", 1: "nt/one-shot", 2: "plain/one-shot", 3: "nt/1024"}


def main():
    sizes = [float(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,1.5,2,3,4,6,8,16".split(","))]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    for m in sizes:
        n = int(m * (1 << 20))
        nat = torch.randint(0, 256, (n * 128,), dtype=torch.uint8, device=dev)
        xdr = torch.empty_like(nat)
        back = torch.empty_like(nat)
        row = []
        for fs, name in SHAPES.items():
            plan = M.Plan(S.ALL["rec128"], {"fixed_stream": fs} if fs != -1 else None)
            mar = M.Marshaler(plan, dev)
            mar.status.init(s)
            enc, dec = [], []
            for r in range(17):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(stream)
                mar.launch_encode(nat, n, xdr, stream=s)
                ev[1].record(stream)
                mar.launch_decode(xdr, n, back, stream=s)
                ev[2].record(stream)
                torch.cuda.synchronize()
                if r >= 2:
                    enc.append(ev[0].elapsed_time(ev[1]))
                    dec.append(ev[1].elapsed_time(ev[2]))
            mar.check(s)
            ok = bool(torch.equal(back, nat))
            t = (float(np.median(enc)) + float(np.median(dec))) / 2
            row.append(f"{name} {n * 256 / (t * 1e-3) / 1e12:.3f}{'' if ok else '(BAD)'}")
        print(f"{m:5.1f}M ({n * 256 >> 20} MiB in+out): TB/s " + "  ".join(row), flush=True)
        del nat, xdr, back
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
