"""Where the speculative walk over a whole stream (rx_windows' first step)
misses on a stream it should hold: XDRG_OPT_INDEX_FAST = 3 runs the walk
alone and leaves its segment records in the workspace; this prints the
segments whose check failed next to the true chain (a tuning tool).  With
a code object built here by `build` (the plan's source with XDRG_LDBG
writing each lane's state past the node lists) it also prints the lanes of
the first failing segments.

    python tools/gpu/rx_whole_diag.py build bigrec|rp_list    # here
    python tools/gpu/rx_whole_diag.py bigrec|rp_list          # GPU box
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from xdrpp_amd import _abi as A, marshal as M, schemas as S, workloads as W  # noqa: E402

SEG, WORDS = 64 * 124 - 8 * 124, 4
DBG = ("#define XDRG_LDBG(k, v) do { *reinterpret_cast<volatile unsigned *>(reinterpret_cast<char *>(nodes) + "
       "static_cast<unsigned long long>(gridDim.x) * (kRxsSeg / 2) + ((static_cast<unsigned long long>(blockIdx.x) "
       "* 64ull + threadIdx.x) * 4ull + (k)) * 4ull) = (v); } while (0)\n")
CO = os.path.join(ROOT, "tools", "tune", "_rxdiag")


def plan_type(which):
    if which == "bigrec":
        import test_record_index as T
        return T.bigrec_type()
    return S.ALL["rp_list"]


def build(which):
    import ctypes as C
    from xdrpp_amd import build as B
    p = M.Plan(plan_type(which))
    L = A.lib()
    n = C.c_size_t()
    A.check(L.xdrg_plan_kernel_source(p.handle, None, 0, C.byref(n)), "source")
    buf = C.create_string_buffer(n.value + 1)
    A.check(L.xdrg_plan_kernel_source(p.handle, buf, n.value + 1, C.byref(n)), "source")
    os.makedirs(CO, exist_ok=True)
    src = os.path.join(CO, f"{which}.hip")
    with open(src, "w") as f:
        f.write(DBG + buf.value.decode())
    import subprocess
    subprocess.check_call([B.hipcc(), "--genco", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-I", B.CSRC,
                           "-I", os.path.join(ROOT, "include"), "-o", os.path.join(CO, f"{which}.co"), src])


def a256(x):
    return (x + 255) // 256 * 256


def main(which):
    dev = torch.device("cuda:0")
    t = plan_type(which)
    if which == "bigrec":
        import test_record_index as T
        x, offs, n = T.long_records_stream(3000, 5)
        dx = torch.from_numpy(x).to(dev)
    else:
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 17
        nat, heap = W.rp_list(n)
        r = M.Marshaler(M.Plan(t), dev).encode(torch.from_numpy(nat).to(dev), n, torch.from_numpy(heap).to(dev))
        dx, offs = r.xdr, r.offsets.cpu().numpy().view(np.uint64)
    plan = M.Plan(t, {"index_fast": 3})
    L = A.lib()
    co = os.path.join(CO, f"{which}.co")
    dbg = os.path.exists(co)
    if dbg:
        code = open(co, "rb").read()
        A.check(L.xdrg_plan_load_kernels(plan.handle, code, len(code)), "xdrg_plan_load_kernels")
    mar = M.Marshaler(plan, dev)
    ln = dx.numel()
    w0 = L.xdrg_index_workspace_size(ln, A.INDEX_MAX_MSG)
    ws = torch.zeros(L.xdrg_index_workspace_size(ln, A.MAX_MSG), dtype=torch.uint8, device=dev)
    o = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    c = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    A.check(L.xdrg_index_records(mar.plan.handle, dx.data_ptr(), ln, n, A.MAX_MSG, o.data_ptr(), c.data_ptr(),
                                 ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index")
    torch.cuda.synchronize()
    w = ws.cpu().numpy()
    nseg = (ln + SEG - 1) // SEG
    flag_at = w0 - 256
    tot_at = flag_at - 256
    base_at = tot_at - a256(nseg * 8)
    cnt_at = base_at - a256(nseg * 8)
    seg_at = cnt_at - a256(nseg * WORDS * 8)
    seg = w[seg_at:seg_at + nseg * WORDS * 8].view(np.uint64).reshape(nseg, WORDS)
    cnt = w[cnt_at:cnt_at + nseg * 8].view(np.uint64)
    flag = int(w[flag_at:flag_at + 4].view(np.uint32)[0])
    print("stream", ln, "bytes", n, "records", nseg, "segments; flag", flag)
    starts = offs[:n + 1].astype(np.int64)
    bad = 0
    for i in range(nseg):
        s0, s1 = i * SEG, min(ln, (i + 1) * SEG)
        inside = starts[(starts >= s0) & (starts < s1)]
        true_cnt = len(inside)
        ex = starts[starts >= s1]
        true_exit = int(ex[0]) if len(ex) else ln
        r1 = int(seg[i][1])
        if int(cnt[i]) != true_cnt or (true_cnt and r1 != true_exit):
            bad += 1
            if bad <= 12:
                r = seg[i]
                print(f"seg {i}: cnt {int(cnt[i])} true {true_cnt}; r0 {int(r[0])} r1 {int(r[1]):#x} r2 {int(r[2])} "
                      f"M {int(r[3])} | s0 {s0} s1 {s1} first {int(inside[0]) if true_cnt else -1} exit {true_exit}")
            if dbg and bad <= 2:
                lo = max(0, s0 - 992)
                d = w[nseg * (SEG // 2):nseg * (SEG // 2) + nseg * 64 * 16].view(np.uint32).reshape(nseg, 64, 4)
                for ln_ in range(64):
                    g0, e0, g1, e1 = (int(v) for v in d[i, ln_])
                    f = lambda v: "-" if v >= 0xfffffffe else (f"L{lo + (v & 0x7fffffff)}" if v & 0x80000000 else str(lo + v))  # noqa: E731
                    print(f"   lane {ln_:2d} [{lo + 124 * ln_ - (0 if s0 == 0 else 0)}]: guess {f(g0)} -> {f(e0)}  final {f(g1)} -> {f(e1)}")
    print("segments whose count differs:", bad)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2])
    else:
        main(sys.argv[1])
