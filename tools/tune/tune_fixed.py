"""Sweep k_fixed_reg variants vs a plain copy on the rec128 1M workload.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes as C
import itertools
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libtune.so")
if not os.path.exists(SO):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-I", os.path.join(ROOT, "include"), "-o", SO, os.path.join(HERE, "tune_fixed.hip")])
L = C.CDLL(SO)
vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
L.tune_copy.argtypes = [vp, vp, u64, i32, i32, i32, vp]
L.tune_reg.argtypes = [vp, vp, u64, u32, vp, i32, i32, i32, vp]

from xdrpp_amd import marshal as M, schemas as S, workloads as W  # noqa: E402

dev = torch.device("cuda:0")
n = int(os.environ.get("TUNE_N", 1 << 20))
nat = torch.from_numpy(W.rec128(n)[0]).to(dev)
out = torch.empty_like(nat)
nchunks = n * 8
# rec128 encode program per chunk position (ints: in place; u64: pair swap)
prog = np.zeros((8, 4, 6), dtype=np.uint32)
for q in range(8):
    for i in range(4):
        ints = q < 2
        prog[q, i, 0] = (0x00010203 if i % 2 == 0 else 0x04050607) if ints else \
                        (0x04050607 if i % 2 == 0 else 0x00010203)
        prog[q, i, 1] = 1
dprog = torch.from_numpy(prog.reshape(-1).view(np.int32)).to(dev)
s = torch.cuda.current_stream().cuda_stream

# correctness of the harness program vs the product library
mar = M.Marshaler(M.Plan(S.rec128), dev)
ref = mar.encode(nat, n).xdr
assert L.tune_reg(nat.data_ptr(), out.data_ptr(), nchunks, 8, dprog.data_ptr(), 4, 1, 2048, s) == 0
torch.cuda.synchronize()
assert torch.equal(out, ref), "harness program differs from libxdrgpu"

variants = []
for kind, U, nt, blocks in itertools.product(["copy", "reg"], [1, 2, 4, 8], [0, 1],
                                             [512, 1024, 2048, 4096, 8192, 16384]):
    if blocks * 256 * U > nchunks * 2:
        continue
    variants.append((kind, U, nt, blocks))
variants.append(("d2d", 0, 0, 0))


def launch(v):
    kind, U, nt, blocks = v
    if kind == "copy":
        return L.tune_copy(nat.data_ptr(), out.data_ptr(), nchunks, U, nt, blocks, s)
    if kind == "reg":
        return L.tune_reg(nat.data_ptr(), out.data_ptr(), nchunks, 8, dprog.data_ptr(), U, nt, blocks, s)
    out.copy_(nat)
    return 0


times = {v: [] for v in variants}
for v in variants:
    for _ in range(3):
        assert launch(v) == 0
torch.cuda.synchronize()
for rnd in range(int(os.environ.get("TUNE_ROUNDS", 5))):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            launch(v)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 10)
alg = 2 * n * 128
res = []
for v, ts in times.items():
    med = float(np.median(ts))
    res.append({"kind": v[0], "U": v[1], "nt": v[2], "blocks": v[3], "ms": round(med, 4),
                "GBps": round(alg / med / 1e6, 1)})
res.sort(key=lambda r: -r["GBps"])
for r in res[:25]:
    print(r)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"tune_fixed_{n}.json"), "w"), indent=1)
