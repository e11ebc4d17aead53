"""Per-wave phase timestamps of the plan-specialized var encode.

    python tools/tune/enc_stamps.py build recvar rpc   # here: stamped .co files
    python tools/tune/enc_stamps.py run recvar rpc     # GPU box

NOSTAMP=1 builds and times the same code objects without the stamps, and
U=<n> sets the payload chunks in flight per lane: an A/B of kernel shapes
against the library's default (encode_ms_library vs encode_ms_stamped).

`build` compiles the plan's generated source (xdrg_plan_kernel_source) with
XDRG_STAMP(k) defined: lane 0 of every wave writes s_memtime at the phase
boundaries of var_encode_body into the output buffer past `cap` (the
harness allocates the room; the library never sees the macro).  `run`
attaches that code object to a plan (xdrg_plan_load_kernels), encodes 1M
records, checks the bytes against the unstamped library's, and prints the
median cycles per phase and the wave lifetime (s_memtime deltas within a
wave; the clocks of different XCDs are not comparable).  IMAGES="-1 32768"
also runs larger LDS images (fewer waves per CU): how a wave's phases
stretch with the number of waves sharing the memory system.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, build as B, marshal as M, schemas as S  # noqa: E402

OUT = os.path.join(ROOT, "tools", "tune", "_stamps" + os.environ.get("U", "") + ("n" if os.environ.get("NOSTAMP") else "")
                   + os.environ.get("TAG", ""))
NST = 10
IMAGES = [int(x) for x in os.environ.get("IMAGES", "-1").split()]  # values of plan option OPT (-1 auto)
PHASES = ["sizes+tile+scan", "first walk", "slots+scan", "windows up to the last copy", "last flush"]
STAMP = ("#define XDRG_STAMP(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = "
         "__builtin_amdgcn_s_memtime(); *reinterpret_cast<volatile unsigned long long *>(xdr + "
         "((cap + 15ull) & ~15ull) + (static_cast<unsigned long long>(blockIdx.x) * " + str(NST) +
         "ull + (k)) * 8ull) = t_; } } while (0)\n"
         "#define XDRG_DSTAMP(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = "
         "__builtin_amdgcn_s_memtime(); *reinterpret_cast<volatile unsigned long long *>(native + "
         "((n * stride + 15ull) & ~15ull) + (static_cast<unsigned long long>(blockIdx.x) * " + str(NST) +
         "ull + (k)) * 8ull) = t_; } } while (0)\n")
DPHASES = ["offsets", "window load+heap copy", "walk", "tile out"]


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
        text = source(M.Plan(S.ALL[name]))
        if os.environ.get("U"):  # payload chunks in flight per lane (the library's default: 4)
            text = text.replace(", 4>(plan_walk{}", ", " + os.environ["U"] + ">(plan_walk{}")
        with open(src, "w") as f:
            f.write(("" if os.environ.get("NOSTAMP") else STAMP) + text)
        subprocess.check_call([B.hipcc(), "--genco", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17"]
                              + os.environ.get("CFLAGS", "").split() + ["-I", B.CSRC, "-I", os.path.join(ROOT, "include"),
                               "-o", os.path.join(OUT, f"{name}.co"), src])
        print("built", name)


def run(schemas):
    import torch
    from xdrpp_amd import workloads as W
    dev = torch.device("cuda:0")
    L = A.lib()
    res = {}
    for name, img in [(nm, i) for nm in schemas for i in IMAGES]:
        n = 1 << 20
        ref = M.Marshaler(M.Plan(S.ALL[name]), dev)
        p = M.Plan(S.ALL[name], {os.environ.get("OPT", "image_bytes"): img})
        code = open(os.path.join(OUT, f"{name}.co"), "rb").read()
        A.check(L.xdrg_plan_load_kernels(p.handle, code, len(code)), "xdrg_plan_load_kernels")
        mar = M.Marshaler(p, dev)
        nat_np, heap_np = W.GENERATORS[name](n)
        nat, heap = torch.from_numpy(nat_np).to(dev), torch.from_numpy(heap_np).to(dev)
        want = ref.encode(nat, n, heap)
        total = want.xdr.numel()
        nw = (n + 63) // 64
        big = torch.zeros(((total + 15) & ~15) + nw * NST * 8, dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            mar.status.init(s)
            mar.launch_encode(nat, n, big[:total], heap=heap, offsets=offs)
            mar.check()
        assert torch.equal(big[:total], want.xdr) and torch.equal(offs, want.offsets), name
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        mar.launch_encode(nat, n, big[:total], heap=heap, offsets=offs)
        ev[1].record()
        torch.cuda.synchronize()
        d = {}
        if not os.environ.get("NOSTAMP"):
            st = big[((total + 15) & ~15):].cpu().numpy().view(np.uint64).reshape(nw, NST).astype(np.int64)
            # 0 start, 1 offsets, 2 first walk, 3 slots, 4 last payload window, 5 end
            seq = [(0, 1, "sizes+tile+scan"), (1, 2, "first walk"), (2, 3, "slots"),
                   (3, 4, "windows up to the last copy"), (4, 5, "last flush")]
            for a, b_, ph in seq:
                dd = st[:, b_] - st[:, a]
                d[ph] = [int(np.median(dd)), int(np.percentile(dd, 90))]
            d["wave_lifetime_median"] = int(np.median(st[:, 5] - st[:, 0]))
        d["encode_ms_all_passes"] = round(ev[0].elapsed_time(ev[1]), 4)
        t = {"library": [], "stamped": []}
        for _ in range(5):
            for k, m in (("library", ref), ("stamped", mar)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    m.launch_encode(nat, n, big[:total], heap=heap, offsets=offs)
                e1.record()
                torch.cuda.synchronize()
                t[k].append(e0.elapsed_time(e1) / 5)
        d["encode_ms_library"] = round(float(np.median(t["library"])), 4)
        d["encode_ms_stamped"] = round(float(np.median(t["stamped"])), 4)
        # decode: the same code object's decode_copy, stamps past the natives
        nb_nat = nat.numel()
        nbig = torch.zeros(((nb_nat + 15) & ~15) + nw * NST * 8, dtype=torch.uint8, device=dev)
        hout = torch.empty(p.decode_heap_bytes(total), dtype=torch.uint8, device=dev)
        for _ in range(2):
            mar.status.init(s)
            mar.launch_decode(want.xdr, n, nbig[:nb_nat], offsets=want.offsets, heap_out=hout)
            mar.check()
        if not os.environ.get("NOSTAMP"):
            st = nbig[((nb_nat + 15) & ~15):].cpu().numpy().view(np.uint64).reshape(nw, NST)[:, :5].astype(np.int64)
            for i, ph in enumerate(DPHASES):
                d["dec " + ph] = int(np.median(st[:, i + 1] - st[:, i]))
            d["dec wave_lifetime_median"] = int(np.median(st[:, 4] - st[:, 0]))
        t = {"library": [], "variant": []}
        back = torch.empty_like(nat)
        for _ in range(5):
            for k, m in (("library", ref), ("variant", mar)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    own = (k == "variant") != bool(os.environ.get("SWAP"))  # SWAP: trade output buffers
                    m.launch_decode(want.xdr, n, nbig[:nb_nat] if own else back, offsets=want.offsets,
                                    heap_out=hout)
                e1.record()
                torch.cuda.synchronize()
                t[k].append(e0.elapsed_time(e1) / 5)
        d["decode_ms_library"] = round(float(np.median(t["library"])), 4)
        d["decode_ms_variant"] = round(float(np.median(t["variant"])), 4)
        res[f"{name}_img{img}"] = d
        print(name, img, json.dumps(d))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "enc_stamps.json"), "w"), indent=1)


if __name__ == "__main__":
    (build if sys.argv[1] == "build" else run)(sys.argv[2:] or ["recvar", "rpc", "vecrec"])
