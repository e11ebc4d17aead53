"""Per-wave phase timestamps of the one-pass var encode (var_kernels.h
var_encode_stream_body).

    python tools/tune/stream_stamps.py build recvar rpc   # here: stamped .co files
    python tools/tune/stream_stamps.py run recvar rpc     # GPU box

`build` compiles the plan's generated source with XDRG_STAMP(k) defined:
lane 0 of every wave writes s_memtime at the phase boundaries into the
output buffer past `cap` (the harness allocates the room; the library never
sees the macro).  `run` attaches the code object (xdrg_plan_load_kernels),
encodes 1M records through xdrg_encode (the look-back) and
xdrg_encode_sized, checks the bytes against the library's, and prints the
median cycles per phase and the wave lifetime.  NOSTAMP=1: the same
without stamps.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, build as B, marshal as M, schemas as S  # noqa: E402

OUT = os.path.join(ROOT, "tools", "tune", "_stamps_stream" + ("n" if os.environ.get("NOSTAMP") else "")
                   + os.environ.get("TAG", ""))
NST = 8
PHASES = ["start->tile", "walk+scans", "tables+lookback", "cap", "assembly+stores"]
STAMP = ("#define XDRG_STAMP(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = "
         "__builtin_amdgcn_s_memtime(); *reinterpret_cast<volatile unsigned long long *>(xdr + "
         "((cap + 15ull) & ~15ull) + (static_cast<unsigned long long>(blockIdx.x) * " + str(NST) +
         "ull + (k)) * 8ull) = t_; } } while (0)\n"
         "#define XDRG_STAMPV(k, v) do { if (threadIdx.x == 0) { *reinterpret_cast<volatile unsigned long long *>(xdr + "
         "((cap + 15ull) & ~15ull) + (static_cast<unsigned long long>(blockIdx.x) * " + str(NST) +
         "ull + (k)) * 8ull) = (v); } } while (0)\n")


def source(plan):
    L = A.lib()
    n = C.c_size_t()
    A.check(L.xdrg_plan_kernel_source(plan.handle, None, 0, C.byref(n)), "xdrg_plan_kernel_source")
    buf = C.create_string_buffer(n.value + 1)
    A.check(L.xdrg_plan_kernel_source(plan.handle, buf, n.value + 1, C.byref(n)), "xdrg_plan_kernel_source")
    return buf.value.decode()


def build(schemas):
    os.makedirs(OUT, exist_ok=True)
    for name in schemas:
        src = os.path.join(OUT, f"{name}.hip")
        with open(src, "w") as f:
            f.write(("" if os.environ.get("NOSTAMP") else STAMP) + source(M.Plan(S.ALL[name])))
        subprocess.check_call([B.hipcc(), "--genco", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17"]
                              + os.environ.get("CFLAGS", "").split()
                              + ["-I", B.CSRC, "-I", os.path.join(ROOT, "include"),
                                 "-o", os.path.join(OUT, f"{name}.co"), src])
        print("built", name)


def run(schemas):
    import torch
    from xdrpp_amd import workloads as W
    dev = torch.device("cuda:0")
    L = A.lib()
    s = torch.cuda.current_stream()
    for name in schemas:
        n = 1 << 20
        nb = (n + 63) // 64
        nat_np, heap_np = W.GENERATORS[name](n)
        nat, heap = torch.from_numpy(nat_np).to(dev), torch.from_numpy(heap_np).to(dev)
        lib_plan = M.Plan(S.ALL[name])
        ref = M.Marshaler(lib_plan, dev).encode(nat, n, heap)
        total = ref.xdr.numel()
        code = open(os.path.join(OUT, f"{name}.co"), "rb").read()
        for hb in [0]:
            plan = M.Plan(S.ALL[name], {"enc_stream": 1})
            A.check(L.xdrg_plan_load_kernels(plan.handle, code, len(code)), "load_kernels")
            mar = M.Marshaler(plan, dev)
            room = ((total + 15) // 16) * 16 + nb * NST * 8
            out = torch.zeros(room, dtype=torch.uint8, device=dev)
            offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
            for mode in ("lookback", "sized"):
                ws = mar._workspace(n)
                if mode == "sized":
                    mar.status.init(s.cuda_stream)
                    A.check(L.xdrg_encode_sizes(plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                                A.DEFAULT_STACK_LIMIT, 0, ws.data_ptr(), ws.numel(),
                                                mar.status.ptr, s.cuda_stream), "sizes")
                    mar.check(s.cuda_stream)

                def go():
                    if mode == "sized":
                        A.check(L.xdrg_encode_sized(plan.handle, nat.data_ptr(), n, heap.data_ptr(), heap.numel(),
                                                    out.data_ptr(), total, offs.data_ptr(), A.DEFAULT_STACK_LIMIT, 0,
                                                    ws.data_ptr(), ws.numel(), mar.status.ptr, s.cuda_stream), "sized")
                    else:
                        mar.launch_encode(nat, n, out[:total], heap=heap, offsets=offs, stream=s.cuda_stream)
                ts = []
                for rep in range(8):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    go()
                    e1.record(s)
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                mar.check(s.cuda_stream)
                if not os.environ.get("NOCHECK"):
                    assert torch.equal(out[:total], ref.xdr), f"{name} {mode}: bytes differ"
                line = f"{name:7s} {mode:8s} {sorted(ts)[len(ts) // 2]:.4f} ms"
                if not os.environ.get("NOSTAMP"):
                    st = out[((total + 15) // 16) * 16:].cpu().numpy().view(np.uint64).reshape(nb, NST)
                    st = st[:, :6].astype(np.int64)
                    d = np.diff(st, axis=1)
                    med = np.median(d, axis=0)
                    life = np.median(st[:, 5] - st[:, 0])
                    line += "  " + "  ".join(f"{p}={m:.0f}" for p, m in zip(PHASES, med)) + f"  life={life:.0f}"
                    if mode == "lookback":
                        pol = out[((total + 15) // 16) * 16:].cpu().numpy().view(np.uint64).reshape(nb, NST)[:, 6]
                        line += f"  polls mean={pol.mean():.2f} max={pol.max()} >1: {(pol > 1).mean():.3f}"
                print(line, flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]](sys.argv[2:])
