"""A/B of the var encode variants on 1M records, one process, interleaved:
the two-pass encode (size pass + scan + windowed encode), the one-pass
encode (look-back), its sized half alone (bases
from a size pass + scan run beforehand) and both halves timed together
(halves: walk-first record kernel; halves0: the two-pass record kernel).  Prints
ms per call (HIP events on the launch stream, mean of REPS after a warmup)
and checks every variant's bytes against the first.

    python tools/tune/stream_ab.py recvar rpc
    VARIANTS="two_pass lb16k lb8k sized16k" REPS=20 python tools/tune/stream_ab.py rpc
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

VAR_OPTS = {
    "two_pass": {"enc_stream": 0}, "walk_first": {"enc_stream": -1}, "lb": {"enc_stream": 1},
    "sized": {"enc_stream": -1}, "halves": {"enc_stream": -1}, "halves0": {"enc_stream": 0},
    "wf2k": {"image_bytes": 2048}, "wf3k": {"image_bytes": 3072}, "wf6k": {"image_bytes": 6144},
    "wf8k": {"image_bytes": 8192},
    "wf_nolin": {"enc_stream": -1, "size_linear": 0}, "two_pass_nolin": {"enc_stream": 0, "size_linear": 0},
}
VARIANTS = os.environ.get("VARIANTS", "two_pass walk_first lb sized").split()
REPS = int(os.environ.get("REPS", "20"))

dev = torch.device("cuda:0")
for schema in sys.argv[1:] or ["recvar", "rpc"]:
    n = 1 << 20
    nat_np, heap_np = W.GENERATORS[schema](n)
    nat = torch.from_numpy(nat_np).to(dev)
    heap = torch.from_numpy(heap_np).to(dev)
    mars = {v: M.Marshaler(M.Plan(S.ALL[schema], VAR_OPTS[v]), dev) for v in VARIANTS}
    total = int(mars[VARIANTS[0]].serial_sizes(nat, n, heap=heap).to(torch.int64).sum().item())
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    L = A.lib()
    ref = None

    def launch(v):
        mar = mars[v]
        if v.startswith("halves"):  # xdrg_encode_sizes + xdrg_encode_sized, both timed
            ws = mar._workspace(n)
            A.check(L.xdrg_encode_sizes(mar.plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                        A.DEFAULT_STACK_LIMIT, 0, ws.data_ptr(), ws.numel(), mar.status.ptr,
                                        s.cuda_stream), "sizes")
            A.check(L.xdrg_encode_sized(mar.plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                        out.data_ptr(), total, offs.data_ptr(), A.DEFAULT_STACK_LIMIT, 0,
                                        ws.data_ptr(), ws.numel(), mar.status.ptr, s.cuda_stream), "sized")
        elif v.startswith("sized"):
            ws = mar._workspace(n)
            A.check(L.xdrg_encode_sized(mar.plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                        out.data_ptr(), total, offs.data_ptr(), A.DEFAULT_STACK_LIMIT, 0,
                                        ws.data_ptr(), ws.numel(), mar.status.ptr, s.cuda_stream), "sized")
        else:
            mar.launch_encode(nat, n, out, heap=heap, offsets=offs, stream=s.cuda_stream)

    for v in VARIANTS:  # warm + check
        mar = mars[v]
        mar.status.init(s.cuda_stream)
        if v.startswith("sized"):
            ws = mar._workspace(n)
            A.check(L.xdrg_encode_sizes(mar.plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                        A.DEFAULT_STACK_LIMIT, 0, ws.data_ptr(), ws.numel(), mar.status.ptr,
                                        s.cuda_stream), "sizes")
        out.zero_()
        launch(v)
        mar.check(s.cuda_stream)
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), f"{schema} {v}: bytes differ"
    times = {v: [] for v in VARIANTS}
    for _ in range(REPS):
        for v in VARIANTS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch(v)
            e1.record(s)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1))
    for v in VARIANTS:
        t = sorted(times[v])
        print(f"{schema:8s} {v:10s} median {t[len(t) // 2]:.4f} ms  min {t[0]:.4f}", flush=True)
