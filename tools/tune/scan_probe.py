"""How the single-workgroup block scan (launch_block_scan) scales with the
number of block sums: xdrg_rpc_replies over n zero headers runs
k_rpc_reply_sizes, k_scan_blocks over n/256 values, k_rpc_reply_emit.
Run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import rpc as R  # noqa: E402

dev = torch.device("cuda:0")
for n in (1 << 18, 1 << 20, 1 << 22, 1 << 24):
    h = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    w = R.ReplyWriter(dev)
    out = torch.empty(4, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    for _ in range(10):
        w.launch(h, out, offs)
    torch.cuda.synchronize()
    print(n, "ok", flush=True)
