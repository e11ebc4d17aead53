"""Run one var schema's encode (and decode) repeatedly: a target for
rocprofv3 PC sampling / counters.  python tools/tune/run_enc.py rpc [reps]
OPTS='{"enc_stream": 0}' sets plan options (xdrg_plan_set_option names)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "rpc"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda:0")
n = 1 << 20
p = M.Plan(S.ALL[name], json.loads(os.environ.get("OPTS", "{}")))
mar = M.Marshaler(p, dev)
nat_np, heap_np = W.GENERATORS[name](n)
nat, heap = torch.from_numpy(nat_np).to(dev), torch.from_numpy(heap_np).to(dev)
res = mar.encode(nat, n, heap)
xdr, offs = res.xdr, res.offsets
back = torch.empty_like(nat)
hout = torch.empty(p.decode_heap_bytes(xdr.numel()), dtype=torch.uint8, device=dev)
for _ in range(reps):
    mar.launch_encode(nat, n, xdr, heap=heap, offsets=offs)
    mar.launch_decode(xdr, n, back, offsets=offs, heap_out=hout)
torch.cuda.synchronize()
mar.check()
print("ok", name, reps)
