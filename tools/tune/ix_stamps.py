"""Per-wave phase timestamps of the speculative record index walk
(index_kernels.h rxs_walk_body), plan-specialized.

    python tools/tune/ix_stamps.py build recvar rpc   # here: stamped .co files
    python tools/tune/ix_stamps.py run recvar rpc     # GPU box

`build` compiles the plan's generated source with XDRG_XSTAMP(k) defined:
lane 0 of every wave writes s_memtime at the phase boundaries into the
workspace's list area past the node lists (the walk's own scratch; the
library never sees the macro).  `run` attaches the code object to a plan,
indexes an encoded 1M batch, checks the offsets and prints the median and
90th-percentile cycles per phase.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xdrpp_amd import _abi as A, build as B, marshal as M, schemas as S  # noqa: E402

OUT = os.path.join(ROOT, "tools", "tune", os.environ.get("STAMPS_DIR", "_stamps_ix"))
EXTRA = os.environ.get("STAMPS_DEFINES", "")  # e.g. "XDRG_RX_NOPREFIX" (A/B builds)
NST = 8
SEGB = 6944  # kRxsSeg
STAMP = ("#define XDRG_XSTAMP(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = "
         "__builtin_amdgcn_s_memtime(); *reinterpret_cast<volatile unsigned long long *>("
         "reinterpret_cast<char *>(nodes) + static_cast<unsigned long long>(gridDim.x) * (kRxsSeg / 2) + "
         "(static_cast<unsigned long long>(blockIdx.x) * " + str(NST) + "ull + (k)) * 8ull) = t_; } } while (0)\n")
# per lane (first LBLK segments): guess-phase clocks (mask, candidate loop),
# candidates parsed, nodes of the lane's chain
LBLK = 2048
LSTAMP = ("#define XDRG_LCLK() __builtin_amdgcn_s_memtime()\n"
          "#define XDRG_LSTAMP(k, v) do { if (blockIdx.x < " + str(LBLK) + "u) { *reinterpret_cast<volatile unsigned long long *>("
          "reinterpret_cast<char *>(nodes) + static_cast<unsigned long long>(gridDim.x) * (kRxsSeg / 2 + " + str(NST * 8) + ") + "
          "((static_cast<unsigned long long>(blockIdx.x) * 64ull + threadIdx.x) * 4ull + (k)) * 8ull) = (v); } } while (0)\n")
PHASES = ["stage", "guess", "agree", "count", "write"]


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
            f.write("".join(f"#define {d}\n" for d in EXTRA.split()) + STAMP + LSTAMP + source(M.Plan(S.ALL[name])))
        subprocess.check_call([B.hipcc(), "--genco", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17",
                               "-I", B.CSRC, "-I", os.path.join(ROOT, "include"),
                               "-o", os.path.join(OUT, f"{name}.co"), src])
        print("built", name)


def run(schemas):
    import torch
    from xdrpp_amd import workloads as W
    dev = torch.device("cuda:0")
    L = A.lib()
    for name in schemas:
        n = 1 << 20
        p = M.Plan(S.ALL[name])
        code = open(os.path.join(OUT, f"{name}.co"), "rb").read()
        A.check(L.xdrg_plan_load_kernels(p.handle, code, len(code)), "xdrg_plan_load_kernels")
        mar = M.Marshaler(p, dev)
        nat, heap = (torch.from_numpy(a).to(dev) for a in W.GENERATORS[name](n))
        enc = mar.encode(nat, n, heap)
        total = enc.xdr.numel()
        # WHOLE=1: the bound the bench's plain stream passes (records of any
        # length: the whole-stream walk when it is past the index window)
        cap = A.MAX_MSG if os.environ.get("WHOLE") else A.INDEX_MAX_MSG
        maxlen = min(p.max_record_bytes, cap)
        ws = torch.zeros(L.xdrg_index_workspace_size(total, maxlen), dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cnt = torch.empty(1, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            mar.status.init(s)
            A.check(L.xdrg_index_records(p.handle, enc.xdr.data_ptr(), total, n, maxlen, offs.data_ptr(),
                                         cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index")
        torch.cuda.synchronize()
        assert torch.equal(offs, enc.offsets), name
        nseg = (total + SEGB - 1) // SEGB
        o = nseg * (SEGB // 2)
        st = ws[o:o + nseg * NST * 8].cpu().numpy().view(np.uint64).reshape(nseg, NST)[:, :6].astype(np.int64)
        d = {}
        for i, ph in enumerate(PHASES):
            dd = st[:, i + 1] - st[:, i]
            d[ph] = [int(np.median(dd)), int(np.percentile(dd, 90)), int(dd.max())]
        d["wave"] = [int(np.median(st[:, 5] - st[:, 0])), int(np.percentile(st[:, 5] - st[:, 0], 90))]
        print(name, "segments", nseg, "cycles [median, p90, max]:", d, flush=True)
        # the timeline: the kernel's span, the waves' summed time over it (the
        # mean number in flight), and where the slowest waves sit in it
        t0, t1 = st[:, 0].min(), st[:, 5].max()
        dur = st[:, 5] - st[:, 0]
        slow = np.argsort(dur)[-5:]
        print(f"  span {t1 - t0} cycles; mean waves in flight {dur.sum() / (t1 - t0):.1f}; last start at "
              f"{st[:, 0].max() - t0}; slowest waves (start, cycles): "
              f"{[(int(st[i, 0] - t0), int(dur[i])) for i in slow]}", flush=True)
        ends = np.sort(st[:, 5] - t0)
        print(f"  ends: 50% at {ends[len(ends) // 2]}, 90% at {ends[int(len(ends) * 0.9)]}, "
              f"99% at {ends[int(len(ends) * 0.99)]}, last {ends[-1]}", flush=True)
        o2 = nseg * (SEGB // 2 + NST * 8)
        nb = min(nseg, LBLK)
        assert o2 + nb * 64 * 32 <= ws.numel()
        ls = ws[o2:o2 + nb * 64 * 32].cpu().numpy().view(np.uint64).reshape(nb, 64, 4).astype(np.int64)
        lanes = ls[:, 8:, :]  # the segment proper
        for j, nm in enumerate(["mask_clk", "loop_clk", "tries", "nodes"]):
            x = lanes[:, :, j]
            wmax = x.max(axis=1)
            print(f"  {nm}: lane mean {x.mean():.1f} p90 {np.percentile(x, 90):.0f}; wave max median "
                  f"{np.median(wmax):.0f} p90 {np.percentile(wmax, 90):.0f}", flush=True)
        t = lanes[:, :, 2]
        print("  tries histogram", np.bincount(t.ravel().clip(0, 8)).tolist(), flush=True)
        print("  nodes histogram", np.bincount(lanes[:, :, 3].ravel().clip(0, 8)).tolist(), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]](sys.argv[2:])
