"""Per-phase cycle shares of the var-length encode / decode kernels
(diagnostic build path: s_memtime stamps, cdna_hip_programming.md §7
In-kernel stamps).  Read the SHARES, not the total (stamps cost time).

    VENC=<0-3> VDEC=<0-3> python tools/tune/stamps_var.py recvar rpc
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

L = A.lib()
L.xdrg__force_var_kernels.argtypes = [C.c_int, C.c_int]
L.xdrg__set_stamps.argtypes = [C.c_void_p]
L.xdrg__set_stamps_enc.argtypes = [C.c_void_p]
L.xdrg__set_window_bytes.argtypes = [C.c_int]
dev = torch.device("cuda:0")
ENC = (["sizes+scan", "tile load+barrier", "walk", "emit", "-"]
       if os.environ.get("VENC", "0") == "2" else ["tile+size pass", "look-back", "walk", "chunk map+copy", "image out"])
DEC = ["window load+copy", "walk (parse)", "tile out", "-", "-"]


def report(tag, st, nwaves, names):
    t = st.cpu().numpy().reshape(nwaves, 8).astype(np.int64)
    d = np.diff(t[:, :6], axis=1)
    tot = d.sum(axis=1)
    print(tag, "median wave lifetime (cycles):", int(np.median(tot)),
          " span first start -> last end:", int(t[:, 5].max() - t[:, 0].min()))
    for i, nm in enumerate(names):
        if nm != "-":
            print(f"  {nm:20s} median {int(np.median(d[:, i])):8d}  share {d[:, i].sum() / tot.sum():.3f}")


for schema in sys.argv[1:] or ["recvar"]:
    n = 1 << 20
    plan = M.Plan(S.ALL[schema])
    mar = M.Marshaler(plan, dev)
    nat_np, heap_np = W.GENERATORS[schema](n)
    nat = torch.from_numpy(nat_np).to(dev)
    heap = torch.from_numpy(heap_np).to(dev)
    total = int(mar.serial_sizes(nat, n).to(torch.int64).sum().item())
    xdr = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    back = torch.empty_like(nat)
    hout = torch.empty(plan.decode_heap_bytes(total), dtype=torch.uint8, device=dev)
    L.xdrg__force_var_kernels(int(os.environ.get('VENC', '0')), int(os.environ.get('VDEC', '0')))
    L.xdrg__set_window_bytes(int(os.environ.get('WIN', '-1')))
    mar.status.init(torch.cuda.current_stream().cuda_stream)
    nwaves = (n + 63) // 64
    se = torch.zeros(nwaves * 8, dtype=torch.int64, device=dev)
    sd = torch.zeros(nwaves * 8, dtype=torch.int64, device=dev)
    L.xdrg__set_stamps_enc(C.c_void_p(se.data_ptr()))
    L.xdrg__set_stamps(C.c_void_p(sd.data_ptr()))
    for _ in range(3):
        mar.launch_encode(nat, n, xdr, heap=heap, offsets=offs)
        mar.launch_decode(xdr, n, back, offsets=offs, heap_out=hout)
    torch.cuda.synchronize()
    L.xdrg__set_stamps(None)
    L.xdrg__set_stamps_enc(None)
    mar.check()
    if se.abs().sum().item():
        report(schema + " encode", se, nwaves, ENC)
    if sd.abs().sum().item():
        report(schema + " decode", sd, nwaves, DEC)
