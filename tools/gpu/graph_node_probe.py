"""Do memset and memcpy nodes of a captured hipGraph take effect on every
replay?  (The deep plans' graphs -- the only ones of ours with such nodes --
replayed once and faulted on the second replay under ROCm's graph packet
capture; profiles/r05a-d.)  No kernel of ours runs here: each case
captures one runtime call (hipMemsetAsync / hipMemsetD32Async /
hipMemcpyAsync on valid buffers), then before every replay the host resets
the destination to a sentinel and checks afterwards whether the node wrote.

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
        want = src.cpu() if "memcpy" in name else torch.zeros(nbytes, dtype=torch.uint8) if "D32" not in name \
            else torch.full((nbytes // 4,), 0x01020304, dtype=torch.int32).view(torch.uint8)
        ok = bool(torch.equal(got, want)) and bool((dst[nbytes:] == 0xAB).all().item())
        res.append("ok" if ok else "MISSED")
    print(f"{name:28s} {nbytes:8d} B: replays {' '.join(res)}", flush=True)
    return all(r == "ok" for r in res)


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
    print("all nodes took effect on every replay" if not bad else f"{bad} cases missed replays")


if __name__ == "__main__":
    main()
