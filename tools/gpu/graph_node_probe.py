"""Do memset and memcpy nodes of a captured hipGraph take effect on every
replay, and do kernels with private (scratch) memory replay correctly?  (The deep plans' graphs -- the only ones of ours with such nodes --
replayed once and faulted on the second replay under ROCm's graph packet
capture; profiles/r05a-d.)  No kernel of ours runs here: each case
captures one runtime call (hipMemsetAsync / hipMemsetD32Async /
hipMemcpyAsync on valid buffers), then before every replay the host resets
the destination to a sentinel and checks afterwards whether the node wrote.
The scratch cases capture one launch of a kernel with a dynamically indexed
private array (tools/gpu/scratch_probe.hip, built here with hipcc) and
compare every replay with an uncaptured launch; the last case launches a
kernel with a 32x larger private array between replays, uncaptured, so the
runtime has to grow its scratch area while the graph holds the old one.

  python tools/gpu/graph_node_probe.py
"""
import ctypes as C

import torch

hip = C.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
hip.hipMemsetD32Async.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]


def case(name, nbytes, call):
    dev = torch.device("cuda:0")
    dst = torch.full((nbytes + 64,), 0xAB, dtype=torch.uint8, device=dev)
    src = torch.arange(nbytes, dtype=torch.int64, device=dev).to(torch.uint8)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        rc = call(dst, src, nbytes, s)
        assert rc == 0, (name, rc)
    res = []
    for it in range(4):
        dst.fill_(0xAB)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        got = dst[:nbytes].cpu()
        want = src.cpu() if "memcpy" in name.lower() else torch.zeros(nbytes, dtype=torch.uint8) if "D32" not in name \
            else torch.full((nbytes // 4,), 0x01020304, dtype=torch.int32).view(torch.uint8)
        ok = bool(torch.equal(got, want)) and bool((dst[nbytes:] == 0xAB).all().item())
        res.append("ok" if ok else "MISSED")
    print(f"{name:28s} {nbytes:8d} B: replays {' '.join(res)}", flush=True)
    return all(r == "ok" for r in res)


def scratch_cases():
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    co = os.path.join(here, "scratch_probe.co")
    src = os.path.join(here, "scratch_probe.hip")
    if not os.path.exists(co) or os.path.getmtime(co) < os.path.getmtime(src):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O3", "-o", co, src])
    hip.hipModuleLoad.argtypes = [C.POINTER(C.c_void_p), C.c_char_p]
    hip.hipModuleGetFunction.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_char_p]
    hip.hipModuleLaunchKernel.argtypes = [C.c_void_p] + [C.c_uint] * 7 + [C.c_void_p, C.c_void_p, C.c_void_p]
    hip.hipFuncGetAttribute.argtypes = [C.POINTER(C.c_int), C.c_int, C.c_void_p]
    mod = C.c_void_p()
    assert hip.hipModuleLoad(C.byref(mod), co.encode()) == 0
    fn = {}
    for name in ("scratch_small", "scratch_big"):
        f = C.c_void_p()
        assert hip.hipModuleGetFunction(C.byref(f), mod, name.encode()) == 0
        priv = C.c_int(-1)
        hip.hipFuncGetAttribute(C.byref(priv), 3, f)  # HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES
        print(f"{name}: private bytes per lane {priv.value}", flush=True)
        fn[name] = f

    def launch(name, out, n, k, stream):
        a_out, a_n, a_k = C.c_void_p(out.data_ptr()), C.c_uint(n), C.c_uint(k)
        args = (C.c_void_p * 3)(C.cast(C.byref(a_out), C.c_void_p), C.cast(C.byref(a_n), C.c_void_p),
                                C.cast(C.byref(a_k), C.c_void_p))
        return hip.hipModuleLaunchKernel(fn[name], (n + 255) // 256, 1, 1, 256, 1, 1, 0, stream, args, None)

    dev = torch.device("cuda:0")
    bad = 0
    for label, cap, n, between in (("scratch_small", "scratch_small", 1 << 20, None),
                                   ("scratch_big", "scratch_big", 1 << 18, None),
                                   ("small, big between replays", "scratch_small", 1 << 16, "scratch_big")):
        want = torch.zeros(n, dtype=torch.int32, device=dev)
        assert launch(cap, want, n, 5, torch.cuda.current_stream().cuda_stream) == 0
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        other = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            assert launch(cap, out, n, 5, torch.cuda.current_stream().cuda_stream) == 0
        res = []
        for it in range(4):
            out.fill_(-1)
            if between:
                assert launch(between, other, 1 << 20, 3, torch.cuda.current_stream().cuda_stream) == 0
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            res.append("ok" if torch.equal(out, want) else "WRONG")
            print(f"  {label}: replay {it} {res[-1]}", flush=True)
        print(f"{label:28s} {n:8d} lanes: replays {' '.join(res)}", flush=True)
        bad += 0 if all(r == "ok" for r in res) else 1
    return bad


def main():
    cases = []
    for n in (4, 8, 16, 24, 256, 4096, 1 << 20):
        cases.append((f"hipMemsetAsync", n, lambda d, s_, n, st: hip.hipMemsetAsync(d.data_ptr(), 0, n, st)))
    for n in (16, 4096):
        cases.append((f"hipMemsetD32Async", n,
                      lambda d, s_, n, st: hip.hipMemsetD32Async(d.data_ptr(), 0x01020304, n // 4, st)))
    for n in (8, 16, 4096, 1 << 20):
        cases.append((f"hipMemcpyAsync D2D", n,
                      lambda d, s_, n, st: hip.hipMemcpyAsync(d.data_ptr(), s_.data_ptr(), n, 3, st)))
    bad = 0
    for name, n, call in cases:
        bad += 0 if case(name, n, call) else 1
    print("all nodes took effect on every replay" if not bad else f"{bad} cases missed replays", flush=True)
    sbad = scratch_cases()
    print("scratch kernels replayed correctly" if not sbad else f"{sbad} scratch cases wrong", flush=True)


if __name__ == "__main__":
    main()
