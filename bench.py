"""Headline benchmark: device-resident XDR encode+decode of 1M x 128-byte
records (BASELINE.json config 2) on N MI355X GPUs.

One step = encode the rank's batch (native rec128 structs -> XDR stream,
= xdr_to_opaque of the batch) + decode it back (= xdr_from_opaque).
Inputs are resident in HBM before timing.  Multi-GPU: one process per GPU
(torchrun), each rank owns a contiguous range of the global record index
(weak scaling, no collective on the data path); the timed region is
bracketed by barrier + synchronize and the max over ranks is reported.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--records N]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts
the N rank processes itself (torch.distributed.run as a child process,
before anything touches the GPU) and exits with its status; under an
external launcher WORLD_SIZE must equal N.  Records per GPU default to
1,048,576 at N = 1 (BASELINE.json config 2) and 2,097,152 at N > 1
(config 5: 16M records over 8 GPUs, seed 0x5EED0005 over the global
record index).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from xdrpp_amd import _abi as A  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import shard as SH  # noqa: E402
from xdrpp_amd import workloads as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--records", "--n", dest="n", type=int, default=None,
                    help="records per GPU (default 1M at N=1, 2M at N>1: BASELINE.json configs 2 and 5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-large", action="store_true",
                    help="skip the 16M-record fixed-path leg (large_batch_16m)")
    ap.add_argument("--no-shard", action="store_true",
                    help="skip the config-5 per-rank shard leg (shard_2m: rank 0's 2M records of 16M)")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="measure pinned host->device->host rates (PCIe-bound, reported apart; "
                         "on by default for rec128)")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--cold", action="store_true",
                    help="time each kernel alone after evicting the caches (on by default for rec128)")
    ap.add_argument("--no-cold", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the RCCL gather of the encoded shards to rank 0 (timed apart)")
    ap.add_argument("--msgs", action="store_true",
                    help="also time the record-marked message path (xdr_to_msg per record, the "
                         "device record index from the marks, xdr_from_msg per message)")
    ap.add_argument("--rpc", action="store_true",
                    help="also time the RPC header batch (xdrg_rpc_dispatch routing of 1M "
                         "record-marked calls + xdrg_rpc_replies error replies)")
    ap.add_argument("--no-plain", action="store_true",
                    help="var schemas: skip the plain-stream leg (the record index xdr_from_opaque "
                         "needs without offsets, xdrg_index_records)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP events around the kernels of every E-th timed step (1: every step)")
    ap.add_argument("--engine", default=None,
                    help="a file defining Engine, in place of the GPU step (tests only: "
                         "tests/bench_cpu_engine.py rehearses the multi-rank plumbing on CPU over gloo)")
    ap.add_argument("--schema", default="rec128",
                    choices=["rec128", "numerics", "recvar", "rpc", "vecrec", "containertest", "rp_list"],
                    help="rec128 is the headline; numerics/recvar/rpc measure BASELINE.json "
                         "configs 1, 3, 4; vecrec covers xvector<T>/pointer<T>")
    ap.add_argument("--plan-opt", action="append", default=[], metavar="NAME=V",
                    help="a plan option (xdrpp_amd._abi.PLAN_OPTIONS) for A/B runs, e.g. enc_stream=0; "
                         "echoed in config.plan_options")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_command(gpus: int, port: int, argv: list[str]) -> list[str]:
    """The torch.distributed.run command that starts one bench rank per GPU.
    (--n is passed on as --records: torch.distributed.run's own parser would
    take it for an abbreviation of its options.)"""
    argv = ["--records" if a == "--n" else "--records=" + a[4:] if a.startswith("--n=") else a for a in argv]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv


def launch_ranks(args) -> int | None:
    """--gpus N > 1 without a launcher: run the N ranks as a child process
    group and return its exit status (None: this process is a rank)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        return subprocess.call(rank_command(args.gpus, _free_port(), sys.argv[1:]), env=env)
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    return None


def dist_init(args, backend="nccl"):
    """One process per GPU: RCCL ("nccl") between the ranks; the tests'
    CPU engine rehearses the same plumbing over gloo."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return dist, world, rank, local
    return None, 1, 0, local


def barrier(dist):
    if dist is not None:
        dist.barrier()


def host_cpus() -> dict:
    """The host's CPUs as this process sees them: nproc, the affinity mask,
    the cgroup CPU quota (cores), and the model name."""
    info = {"nproc": os.cpu_count() or 1, "affinity": len(os.sched_getaffinity(0)), "cgroup_quota": None,
            "cpu_model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota"] = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def _port_baseline(schema: str, n: int, threads: int, reps: int, nat, heap) -> dict:
    """The committed C restatement (oracle/xdr_oracle.c) on `threads`
    pthreads over contiguous slices (oracle/cpu_bench.c)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as O
    plan = __import__("xdrpp_amd.xdr_types", fromlist=["compile_plan"]).compile_plan(S.ALL[schema])
    L = O.lib()
    vp, u32, u64 = A.C.c_void_p, A.C.c_uint32, A.C.c_uint64
    L.xdro_bench.argtypes = [vp, u32, vp, u32, vp, u64, vp, u64, vp, u64, vp, u32, u32, vp]
    L.xdro_bench.restype = A.C.c_int
    sizes = np.zeros(n, dtype=np.uint32)
    X = n * plan.fixed_size if plan.fixed_size else None
    if X is None:
        X = int(O.sizes(plan, nat, n, heap).astype(np.int64).sum())  # (element arrays live in the heap)
    out = np.zeros(max(X, 4), dtype=np.uint8)
    back = np.zeros(n * plan.stride, dtype=np.uint8)
    res = np.zeros(8, dtype=np.float64)
    p = lambda a: a.ctypes.data if a is not None and a.size else None  # noqa: E731
    rc = L.xdro_bench(p(plan.ops), len(plan.ops), p(plan.table), plan.stride, p(nat), n, p(heap),
                      0 if heap is None else heap.size, p(out), out.size, p(back), threads, reps, p(res))
    if rc != 0:
        raise RuntimeError(f"xdro_bench failed ({rc})")
    del sizes
    gib = res[6] / GIB
    r = {"encode_gib_s": gib / res[0], "decode_gib_s": gib / res[2], "to_opaque_gib_s": gib / res[4],
         "encode_decode_gib_s": 2 * gib / (res[0] + res[2]),
         "encode_decode_gib_s_median": 2 * gib / (res[1] + res[3]), "threads": threads}
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    h = json.load(open(man))["hashes"].get(f"{schema}_{n}") if os.path.exists(man) else None
    if h is not None:
        r["bit_exact_vs_reference"] = hashlib.sha256(out[:X].tobytes()).hexdigest() == h["xdr"]
    return r


def _ref_baseline(schema: str, n: int, threads: int, reps: int) -> dict | None:
    """The real reference (oracle/_ref/ref_golden: xdrpp/marshal.cc compiled
    by build() in the container, shipped with the tree) on `threads`
    std::threads."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
    if not (os.path.exists(ref) and os.access(ref, os.X_OK)):
        return None
    out = subprocess.run([ref, "bench", schema, str(n), str(threads), str(reps)],
                         capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-200:]}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    got = {k: r[k] for k in ("encode_gib_s", "decode_gib_s", "to_opaque_gib_s", "encode_decode_gib_s",
                             "threads")}
    got["encode_decode_gib_s_median"] = 2 * r["xdr_bytes"] / GIB / (r["encode_s_median"] + r["decode_s_median"])
    return got


def cpu_baseline(schema: str, n_records: int, threads: int = 0) -> dict:
    """The reference's CPU marshaler on this host, on the same workload:
    the real reference (oracle/_ref) when the tree carries it, and always
    the committed C restatement (oracle/cpu_bench.c).  One thread per host
    core (the affinity mask; also the cgroup quota when that is smaller),
    best of `reps` over the whole batch; the median of
    the same runs beside it (`value_median`: the best swings with the box)."""
    cpus = host_cpus()
    counts = [threads] if threads else sorted({cpus["affinity"], cpus["cgroup_quota"] or cpus["affinity"], 1})
    reps = 5
    nat, heap = W.GENERATORS[schema](n_records)
    runs = {"port": {}, "reference": {}}
    for t in counts:
        runs["port"][t] = _port_baseline(schema, n_records, t, reps, nat, heap)
        ref = _ref_baseline(schema, n_records, t, reps)
        if ref is not None:
            runs["reference"][t] = ref
    kind = "reference" if runs["reference"] and all("error" not in v for v in runs["reference"].values()) \
        else "port"
    best_t = max(runs[kind], key=lambda t: runs[kind][t]["encode_decode_gib_s"])
    best = runs[kind][best_t]
    return {"value": round(best["encode_decode_gib_s"], 3), "unit": "GiB/s", "cores": best_t, "kind": kind,
            "value_median": round(best["encode_decode_gib_s_median"], 3),
            "sample": f"{schema} x {n_records} (the whole batch): xdr_put / xdr_get streams over {best_t} "
                      f"contiguous slices, one thread each, best of {reps} (value_median: median)",
            "nproc": cpus["nproc"], "affinity_cpus": cpus["affinity"], "cgroup_quota_cpus": cpus["cgroup_quota"],
            "cpu_model": cpus["cpu_model"],
            "encode_gib_s": round(best["encode_gib_s"], 3), "decode_gib_s": round(best["decode_gib_s"], 3),
            "to_opaque_gib_s": round(best["to_opaque_gib_s"], 3),
            "by_threads": {k: {str(t): round(v["encode_decode_gib_s"], 3) for t, v in runs[k].items()}
                           for k in runs if runs[k]},
            "port_bit_exact_vs_reference": runs["port"][best_t if best_t in runs["port"] else counts[0]]
            .get("bit_exact_vs_reference")}


def pcie_ceiling(nbytes: int, dev, reps=5, chunk=16 << 20, nstreams=4) -> dict:
    """Raw pinned hipMemcpyAsync bandwidth on this box, chunked over
    `nstreams` streams like the host-inclusive legs: H2D alone, D2H alone
    and both directions at once (full duplex).  GiB/s, best of reps."""
    h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]

    def run(h2d: bool, d2h: bool) -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ci, o in enumerate(range(0, nbytes, chunk)):
            e = min(o + chunk, nbytes)
            with torch.cuda.stream(streams[ci % nstreams]):
                if h2d:
                    d_a[o:e].copy_(h_src[o:e], non_blocking=True)
                if d2h:
                    h_dst[o:e].copy_(d_b[o:e], non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(True, True)
    g = nbytes / GIB
    h2d = g / min(run(True, False) for _ in range(reps))
    d2h = g / min(run(False, True) for _ in range(reps))
    both = 2 * g / min(run(True, True) for _ in range(reps))
    return {"h2d_gib_s": round(h2d, 2), "d2h_gib_s": round(d2h, 2), "duplex_gib_s": round(both, 2),
            "bytes": nbytes, "chunk_bytes": chunk, "streams": nstreams}


def host_inclusive(mar, plan, nat_dev, n, W_, reps=5, nstreams=4, chunk_records=1 << 15):
    """Pinned host -> device -> encode -> host, chunked over `nstreams`
    streams so that chunk k's D2H runs while chunk k+1's H2D and kernel run
    (both copy directions at once), and the decode mirror.  PCIe-bound;
    reported apart, never as `value`, next to the raw copy ceiling."""
    S_ = plan.stride
    h_nat = torch.empty(n * S_, dtype=torch.uint8, pin_memory=True)
    h_nat.copy_(nat_dev.cpu())
    h_xdr = torch.empty(n * W_, dtype=torch.uint8, pin_memory=True)
    h_back = torch.empty(n * S_, dtype=torch.uint8, pin_memory=True)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    d_nat = [torch.empty(chunk_records * S_, dtype=torch.uint8, device=nat_dev.device) for _ in streams]
    d_xdr = [torch.empty(chunk_records * W_, dtype=torch.uint8, device=nat_dev.device) for _ in streams]
    mars = [M.Marshaler(plan, nat_dev.device) for _ in streams]
    for m in mars:
        m.status.init(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()

    def run(encode: bool) -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ci, r0 in enumerate(range(0, n, chunk_records)):
            k = ci % nstreams
            s = streams[k]
            nr = min(chunk_records, n - r0)
            with torch.cuda.stream(s):
                if encode:
                    d_nat[k][:nr * S_].copy_(h_nat[r0 * S_:(r0 + nr) * S_], non_blocking=True)
                    mars[k].launch_encode(d_nat[k][:nr * S_], nr, d_xdr[k][:nr * W_], stream=s.cuda_stream)
                    h_xdr[r0 * W_:(r0 + nr) * W_].copy_(d_xdr[k][:nr * W_], non_blocking=True)
                else:
                    d_xdr[k][:nr * W_].copy_(h_xdr[r0 * W_:(r0 + nr) * W_], non_blocking=True)
                    mars[k].launch_decode(d_xdr[k][:nr * W_], nr, d_nat[k][:nr * S_], stream=s.cuda_stream)
                    h_back[r0 * S_:(r0 + nr) * S_].copy_(d_nat[k][:nr * S_], non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(True), run(False)
    te = min(run(True) for _ in range(reps))
    td = min(run(False) for _ in range(reps))
    for m in mars:
        m.check(torch.cuda.current_stream().cuda_stream)
    ok = torch.equal(h_back, h_nat)
    xb = n * W_
    return {"encode_gib_s": round(xb / GIB / te, 2), "decode_gib_s": round(xb / GIB / td, 2),
            "encode_decode_gib_s": round(2 * xb / GIB / (te + td), 2), "round_trip_ok": bool(ok),
            "chunk_records": chunk_records, "streams": nstreams,
            "pcie_ceiling": pcie_ceiling(max(n * S_, xb), nat_dev.device, chunk=chunk_records * W_,
                                         nstreams=nstreams)}


def host_inclusive_var(mar, plan, nat_dev, heap_dev, n, reps=3):
    """Var schemas, whole batch on one stream: pinned native records + payload
    heap H2D -> encode -> stream + record index D2H, and the decode mirror
    (stream + index H2D -> decode -> native records + decoded heap D2H).
    PCIe-bound; reported apart, never as `value`."""
    dev = nat_dev.device
    s = torch.cuda.current_stream()
    h_nat = nat_dev.cpu().pin_memory()
    h_heap = heap_dev.cpu().pin_memory()
    X = int(mar.serial_sizes(nat_dev, n, heap=heap_dev).to(torch.int64).sum().item())
    d_nat, d_heap = torch.empty_like(nat_dev), torch.empty_like(heap_dev)
    d_xdr = torch.empty(X, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    h_xdr = torch.empty(X, dtype=torch.uint8, pin_memory=True)
    h_off = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
    d_back = torch.empty_like(nat_dev)
    d_hout = torch.empty(plan.decode_heap_bytes(X), dtype=torch.uint8, device=dev)
    h_back = torch.empty(d_back.numel(), dtype=torch.uint8, pin_memory=True)
    h_hout = torch.empty(d_hout.numel(), dtype=torch.uint8, pin_memory=True)
    mar.status.init(s.cuda_stream)

    def enc():
        d_nat.copy_(h_nat, non_blocking=True)
        d_heap.copy_(h_heap, non_blocking=True)
        mar.launch_encode(d_nat, n, d_xdr, heap=d_heap, offsets=d_off, stream=s.cuda_stream)
        h_xdr.copy_(d_xdr, non_blocking=True)
        h_off.copy_(d_off, non_blocking=True)

    def dec():
        d_xdr.copy_(h_xdr, non_blocking=True)
        d_off.copy_(h_off, non_blocking=True)
        mar.launch_decode(d_xdr, n, d_back, offsets=d_off, heap_out=d_hout, stream=s.cuda_stream)
        h_back.copy_(d_back, non_blocking=True)
        h_hout.copy_(d_hout, non_blocking=True)

    def timed(f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    timed(enc), timed(dec)
    te = min(timed(enc) for _ in range(reps))
    td = min(timed(dec) for _ in range(reps))
    mar.check(s.cuda_stream)
    x2 = torch.empty_like(d_xdr)
    mar.launch_encode(d_back, n, x2, heap=d_hout, offsets=torch.empty_like(d_off), stream=s.cuda_stream)
    mar.check(s.cuda_stream)
    return {"encode_gib_s": round(X / GIB / te, 2), "decode_gib_s": round(X / GIB / td, 2),
            "encode_decode_gib_s": round(2 * X / GIB / (te + td), 2),
            "round_trip_ok": bool(torch.equal(x2, d_xdr)), "streams": 1,
            "note": "whole batch, copies and kernel serialized on one stream"}


def cold_cache(mar, nat, xdr, back, n, alg_bytes, reps=5):
    """Each kernel timed alone after a 1 GiB streaming READ that evicts the
    256 MiB Infinity Cache and the L2s without leaving dirty lines whose
    write-back would land inside the timed kernel."""
    scratch = torch.ones(1 << 27, dtype=torch.int64, device=nat.device)  # 1 GiB
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    enc, dec = [], []
    for r in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        sink = scratch.sum()
        ev[0].record(stream)
        mar.launch_encode(nat, n, xdr, stream=s)
        ev[1].record(stream)
        sink = sink + scratch.sum()
        ev[2].record(stream)
        mar.launch_decode(xdr, n, back, stream=s)
        ev[3].record(stream)
        torch.cuda.synchronize()
        enc.append(ev[0].elapsed_time(ev[1]))
        dec.append(ev[2].elapsed_time(ev[3]))
    del scratch
    e, d = float(np.median(enc)), float(np.median(dec))
    xb = xdr.numel()  # XDR bytes of the batch
    return {"encode_ms": round(e, 4), "decode_ms": round(d, 4),
            "encode_decode_gib_s": round(2 * xb / GIB / ((e + d) * 1e-3), 2),
            "achieved_GBps": round(alg_bytes / ((e + d) / 2 * 1e-3) / 1e9, 1),
            "protocol": "1 GiB read sweep before each kernel, HIP events around the kernel, "
                        f"median of {reps}"}


def plan_linear(plan) -> bool:
    """Var plans whose walk never branches size without a walk (k_size_linear):
    scalars, opaque[n] and opaque<>/string<> fields only, at most 8 of them."""
    ops = plan.cp.ops
    k = ops["kind"]
    nvar = int(((k == A.OP_VAROPAQUE) | (k == A.OP_STRING)).sum())
    return not plan.is_fixed and nvar <= 8 and not np.isin(k, [A.OP_UNION, A.OP_JUMP, A.OP_VECTOR]).any()


def large_batch(mar, dev, reps=5, n=1 << 24):
    """The fixed path at 16M records (2 GiB in, 2 GiB out per kernel): a
    working set eight times the 256 MiB Infinity Cache, so the rate is HBM's,
    not the cache's (the 1M headline fits in it).  Synthetic record bytes
    made on the device; parity at this size is tests/test_gpu_parity.py
    (test_config5_16m_sharded)."""
    S_ = mar.plan.stride
    nat = torch.randint(0, 256, (n * S_,), dtype=torch.uint8, device=dev)
    xdr = torch.empty(n * mar.plan.fixed_size, dtype=torch.uint8, device=dev)
    back = torch.empty_like(nat)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    mar.status.init(s)
    enc, dec = [], []
    for r in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        mar.launch_encode(nat, n, xdr, stream=s)
        ev[1].record(stream)
        mar.launch_decode(xdr, n, back, stream=s)
        ev[2].record(stream)
        torch.cuda.synchronize()
        if r:
            enc.append(ev[0].elapsed_time(ev[1]))
            dec.append(ev[1].elapsed_time(ev[2]))
    mar.check(s)
    ok = bool(torch.equal(back, nat))
    e, d = float(np.median(enc)), float(np.median(dec))
    alg = n * (S_ + mar.plan.fixed_size)  # bytes in + out per kernel
    ach = alg / ((e + d) / 2 * 1e-3) / 1e9
    del nat, xdr, back
    return {"records": n, "encode_ms": round(e, 4), "decode_ms": round(d, 4),
            "encode_decode_gib_s": round(2 * n * mar.plan.fixed_size / GIB / ((e + d) * 1e-3), 2),
            "achieved_GBps": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4), "round_trip_ok": ok,
            "protocol": f"HIP events around each kernel, median of {reps}, device-made record bytes"}


SHARD_SHAPES = {-1: "default (by working set)", 0: "plain, 1024 workgroups", 1: "non-temporal, one-shot grid",
                2: "plain, one-shot grid", 3: "non-temporal, 1024 workgroups"}


def shard_leg(dev, reps=20, world=8, n=1 << 21) -> dict:
    """Config 5's per-rank work on one GPU: rank 0's shard of the 16M-record
    batch (2M rec128 records, seed 0x5EED0005 over the global record index;
    256 MiB per buffer, 512 MiB in+out per kernel -- past the 256 MiB
    Infinity Cache), encode + decode back to back with HIP events around
    each kernel, median of `reps`.  Bit-exact against the reference's hash of
    the 16M stream's first 2M records (manifest rec128_mgpu_2097152).  Every
    k_fixed_reg launch shape (XDRG_OPT_FIXED_STREAM) is timed beside the
    default, which is the leg's result."""
    nat_np, _ = SH.shard_inputs("rec128", n, 0, world)
    nat = torch.from_numpy(nat_np).to(dev)
    del nat_np
    W_ = 128  # rec128: 128 wire bytes, native stride 128
    xdr = torch.empty(n * W_, dtype=torch.uint8, device=dev)
    back = torch.empty_like(nat)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    alg = n * (128 + W_)  # bytes in + out per kernel
    shapes = {}
    for fs in SHARD_SHAPES:
        plan = M.Plan(S.ALL["rec128"], {"fixed_stream": fs} if fs != -1 else None)
        mar = M.Marshaler(plan, dev)
        mar.status.init(s)
        enc, dec = [], []
        for r in range(reps + 2):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(stream)
            mar.launch_encode(nat, n, xdr, stream=s)
            ev[1].record(stream)
            mar.launch_decode(xdr, n, back, stream=s)
            ev[2].record(stream)
            torch.cuda.synchronize()
            if r >= 2:
                enc.append(ev[0].elapsed_time(ev[1]))
                dec.append(ev[1].elapsed_time(ev[2]))
        mar.check(s)
        e, d = float(np.median(enc)), float(np.median(dec))
        ach = alg / ((e + d) / 2 * 1e-3) / 1e9
        shapes[fs] = {"shape": SHARD_SHAPES[fs], "encode_ms": round(e, 4), "decode_ms": round(d, 4),
                      "achieved_GBps": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                      "round_trip_ok": bool(torch.equal(back, nat))}
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    h = json.load(open(man))["hashes"].get(f"rec128_mgpu_{n}") if os.path.exists(man) else None
    bit_exact = None if h is None else hashlib.sha256(xdr.cpu().numpy().tobytes()).hexdigest() == h["xdr"]
    best = shapes[-1]
    res = {"records": n, "shard": f"rank 0 of {world} (config 5: {n * world} records, seed 0x5EED0005)",
           "encode_ms": best["encode_ms"], "decode_ms": best["decode_ms"],
           "encode_decode_gib_s": round(2 * n * W_ / GIB / ((best["encode_ms"] + best["decode_ms"]) * 1e-3), 2),
           "achieved_GBps": best["achieved_GBps"], "frac": best["frac"],
           "round_trip_ok": best["round_trip_ok"], "bit_exact_vs_reference": bit_exact,
           "shapes": {SHARD_SHAPES[k]: {kk: vv for kk, vv in v.items() if kk != "shape"} for k, v in shapes.items()},
           "protocol": f"HIP events around each kernel, median of {reps} after 2 untimed"}
    del nat, xdr, back
    torch.cuda.empty_cache()
    ceil = copy_ceiling(n * W_ >> 20)  # the same bytes per buffer
    if ceil is not None:
        res["copy_ceiling"] = ceil
        if "best_tb_s" in ceil:
            res["frac_of_copy_ceiling"] = round(res["achieved_GBps"] / (ceil["best_tb_s"] * 1e3), 4)
    return res


def copy_ceiling(mib: int) -> dict | None:
    """The box's device-copy ceiling past the Infinity Cache: the best of
    four plain 16-byte copy shapes (tools/probe/copy_ceiling.hip, built by
    build(); run as a child process), `mib` MiB per buffer, median of 7."""
    probe = os.path.join(ROOT, "tools", "probe", "copy_ceiling")
    if not os.access(probe, os.X_OK):
        return None
    out = subprocess.run([probe, "--json", str(mib)], capture_output=True, text=True, timeout=120)
    if out.returncode != 0:
        return {"error": out.stdout[-200:] + out.stderr[-200:]}
    return json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])


def messages_leg(schema, plan, mar, nat, heap, n, reps=20):
    """Record-marked messages (message_t, RFC 5531): encode_msgs = xdr_to_msg
    per record, the device index of the stream's marks (read_message framing),
    decode_msgs = xdr_from_msg per message.  Each timed alone with HIP events
    on the launch stream; reported apart from the headline."""
    dev = nat.device
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    X = n * plan.fixed_size if plan.is_fixed else \
        int(mar.serial_sizes(nat, n, heap=heap).to(torch.int64).sum().item())
    total = X + 4 * n
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    idx = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    back = torch.empty(n * plan.stride, dtype=torch.uint8, device=dev)
    hout = None if plan.is_fixed else torch.empty(plan.decode_heap_bytes(total), dtype=torch.uint8,
                                                  device=dev)
    L = A.lib()
    maxlen = min(plan.max_record_bytes, A.INDEX_MAX_MSG)
    ws = torch.empty(max(L.xdrg_index_workspace_size(total, maxlen), 16), dtype=torch.uint8, device=dev)
    st = M.Status(dev)
    st.init(s)
    mar.status.init(s)

    def index():
        A.check(L.xdrg_index_msgs(out.data_ptr(), total, maxlen, n, idx.data_ptr(), cnt.data_ptr(),
                                  ws.data_ptr(), ws.numel(), st.ptr, s), "xdrg_index_msgs")

    legs = {"encode_msgs": lambda: mar.launch_encode_msgs(nat, n, out, offs, heap=heap, stream=s),
            "index_msgs": index,
            "decode_msgs": lambda: mar.launch_decode_msgs(out, n, back, idx, heap_out=hout, stream=s)}
    for f in legs.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in legs}
    for _ in range(reps):
        for k, f in legs.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            f()
            ev[1].record(stream)
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]))
    mar.check(s)
    e = st.read(s)
    ok_index = e.code == 0 and int(cnt.item()) == n and bool(torch.equal(idx, offs))
    x2 = torch.empty_like(out)
    o2 = torch.empty_like(offs)
    mar.status.init(s)
    mar.launch_encode_msgs(back, n, x2, o2, heap=hout if hout is not None else heap, stream=s)
    mar.check(s)
    r = {k: round(float(np.mean(v)), 4) for k, v in times.items()}
    ms = r["encode_msgs"] + r["index_msgs"] + r["decode_msgs"]
    res = {"stream_bytes": total,
           "encode_msgs_ms": r["encode_msgs"], "index_msgs_ms": r["index_msgs"],
           "decode_msgs_ms": r["decode_msgs"],
           "encode_index_decode_gib_s": round(2 * total / GIB / (ms * 1e-3), 2),
           "index_gb_s": round((total + 8 * (n + 1)) / (r["index_msgs"] * 1e-3) / 1e9, 1),
           "index_ok": ok_index, "round_trip_ok": bool(torch.equal(x2, out)),
           "protocol": f"HIP events around each launch, mean of {reps}"}
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    if os.path.exists(man):
        h = json.load(open(man))["hashes"].get(f"{schema}_{n}", {})
        if "msgs" in h:
            res["bit_exact_vs_reference"] = (
                hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == h["msgs"])
    return res


def plain_stream_leg(schema, engine, dec_ms, reps=10):
    """xdr_from_opaque of a plain concatenated stream (marshal.h:299-306):
    the record index the decode needs when no offsets came with the bytes
    (xdrg_index_records), timed with HIP events around the call -- the
    speculative walk, whose verdict the host waits for (the gap counts), and
    beside it the list ranking alone (XDRG_OPT_INDEX_FAST = 0) -- then the
    decode it feeds.  The offsets must equal the encoder's."""
    dev = engine.nat.device
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    xdr, want, n = engine.xdr, engine.offsets, engine.n
    L = A.lib()
    res = {}
    for label, fast in (("index", 1), ("index_list_ranking", 0)):
        plan = M.Plan(S.ALL[schema], {"index_fast": fast})
        mar = M.Marshaler(plan, dev)
        # records past one index window (rp_list's 500-node lists) take the
        # windowed index (include/xdrgpu.h xdrg_index_records)
        maxlen = max(min(plan.max_record_bytes, A.MAX_MSG), 16)
        total = xdr.numel()
        ws = torch.empty(max(L.xdrg_index_workspace_size(total, maxlen), 16), dtype=torch.uint8, device=dev)
        flag_at = L.xdrg_index_workspace_size(total, min(maxlen, A.INDEX_MAX_MSG)) - 256
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        cnt = torch.empty(1, dtype=torch.int64, device=dev)
        mar.status.init(s)

        def run():
            A.check(L.xdrg_index_records(plan.handle, xdr.data_ptr(), total, n, maxlen, offs.data_ptr(),
                                         cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s),
                    "xdrg_index_records")
        run()
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            run()
            ev[1].record(stream)
            torch.cuda.synchronize()
            t.append(ev[0].elapsed_time(ev[1]))
        ok = mar.status.read(s).code == 0 and int(cnt.item()) == n and bool(torch.equal(offs, want))
        res[label + "_ms"] = round(float(np.mean(t)), 4)
        res[label + "_ok"] = ok
        if fast:
            res["walk_held"] = int(ws[flag_at:flag_at + 4].cpu().numpy().view(np.uint32)[0]) == 1
            res["windowed"] = maxlen > A.INDEX_MAX_MSG and not res["walk_held"]
    res["decode_ms"] = dec_ms
    res["index_over_decode"] = round(res["index_ms"] / dec_ms, 3)
    res["protocol"] = f"HIP events around each xdrg_index_records call, mean of {reps}; decode: the headline's"
    return res


def rpc_leg(dev, n=1 << 20, reps=20):
    """RPC header batches: xdrg_rpc_dispatch over n
    record-marked CALL messages (workloads.rpc_calls: mixed routes and
    malformed headers) and xdrg_rpc_replies of the batch's error replies.
    HIP events on the launch stream, mean of reps; reported apart from the
    headline.  Algorithmic bytes of dispatch: the header bytes each lane
    reads (mark .. end of header) + its two offsets + the 64-byte record."""
    from xdrpp_amd import rpc as R
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    sb, ob = W.rpc_calls(n)
    st = torch.from_numpy(sb).to(dev)
    od = torch.from_numpy(ob.view(np.int64)).to(dev)
    procs = torch.from_numpy(W.RPC_PROCS.view(np.int32)).to(dev)
    hd = torch.empty(n * A.RPC_HDR_BYTES, dtype=torch.uint8, device=dev)
    rw = R.ReplyWriter(dev)
    rout = torch.empty(36 * n, dtype=torch.uint8, device=dev)
    roffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    L = A.lib()
    rw.status.init(s)

    def disp():
        A.check(L.xdrg_rpc_dispatch(st.data_ptr(), st.numel(), od.data_ptr(), n, procs.data_ptr(),
                                    procs.numel() // 4, hd.data_ptr(), s), "xdrg_rpc_dispatch")

    legs = {"dispatch": disp, "replies": lambda: rw.launch(hd, rout, roffs, s)}
    for f in legs.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in legs}
    for _ in range(reps):
        for k, f in legs.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            f()
            ev[1].record(stream)
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]))
    e = rw.status.read(s)
    h = hd.cpu().numpy().view(R.HDR_DTYPE)
    hdr_bytes = int(np.where(h["err"] == 0, h["body_off"] - ob[:-1], h["end"] - ob[:-1]).sum())
    r = {k: round(float(np.mean(v)), 4) for k, v in times.items()}
    alg = hdr_bytes + 16 * n + A.RPC_HDR_BYTES * n
    res = {"messages": n, "stream_bytes": int(sb.size), "dispatch_ms": r["dispatch"],
           "replies_ms": r["replies"], "reply_bytes": int(e.total_bytes),
           "dispatch_mmsg_s": round(n / (r["dispatch"] * 1e-3) / 1e6, 1),
           "dispatch_alg_bytes": alg, "dispatch_gb_s": round(alg / (r["dispatch"] * 1e-3) / 1e9, 1),
           "protocol": f"HIP events around each launch, mean of {reps}"}
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    if os.path.exists(man):
        hh = json.load(open(man))["hashes"].get(f"rpccall_{n}", {})
        if "hdrs" in hh:
            res["bit_exact_vs_reference"] = (
                hashlib.sha256(h.tobytes()).hexdigest() == hh["hdrs"] and
                hashlib.sha256(rout[:int(e.total_bytes)].cpu().numpy().tobytes()).hexdigest()
                == hh["replies"])
    return res


def setup(schema, n, dev, rank, world, opts=None):
    """Plan, resident inputs and preallocated outputs for one rank."""
    plan = M.Plan(S.ALL[schema], opts or None)
    mar = M.Marshaler(plan, dev)
    nat_np, heap_np = SH.shard_inputs(schema, n, rank, world)
    nat = torch.from_numpy(nat_np).to(dev)
    heap = torch.from_numpy(heap_np).to(dev) if heap_np.size else None
    back = torch.empty(n * plan.stride, dtype=torch.uint8, device=dev)
    if plan.is_fixed:
        xdr = torch.empty(n * plan.fixed_size, dtype=torch.uint8, device=dev)
        return plan, mar, nat, heap, xdr, back, None, None
    total = int(mar.serial_sizes(nat, n, heap=heap).to(torch.int64).sum().item())
    xdr = torch.empty(total, dtype=torch.uint8, device=dev)
    offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
    heap_out = torch.empty(plan.decode_heap_bytes(total), dtype=torch.uint8, device=dev)
    return plan, mar, nat, heap, xdr, back, offsets, heap_out


def plan_opts(args) -> dict:
    """--plan-opt NAME=V pairs as a plan options dict."""
    out = {}
    for kv in getattr(args, "plan_opt", []) or []:
        k, v = kv.split("=", 1)
        out[k] = int(v)
    return out


def walk_first(plan) -> bool:
    """Word-list plans encode with the walk-first record kernel
    (xdrg_spec_encode_pre, XDRG_OPT_ENC_STREAM default): its generated source
    defines it."""
    L = A.lib()
    n = A.C.c_size_t(0)
    if L.xdrg_plan_kernel_source(plan.handle, None, 0, A.C.byref(n)) != A.OK:
        return False
    buf = A.C.create_string_buffer(n.value + 1)
    A.check(L.xdrg_plan_kernel_source(plan.handle, buf, n.value + 1, A.C.byref(n)), "xdrg_plan_kernel_source")
    return b"xdrg_spec_encode_pre" in buf.value


class GpuEngine:
    """One rank's marshal step on its GPU: encode the rank's batch, decode it
    back (libxdrgpu through xdrpp_amd.marshal), with HIP events around the
    kernels of the steps the caller marks.  The multi-rank plumbing of
    main() only sees this interface (tests/bench_cpu_engine.py gives it a
    CPU stand-in to rehearse that plumbing over gloo)."""

    backend = "nccl"

    def __init__(self, args, n, rank, world, local):
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.schema, self.n = args.schema, n
        (self.plan, self.mar, self.nat, self.heap, self.xdr, self.back, self.offsets,
         self.heap_out) = setup(args.schema, n, self.dev, rank, world, plan_opts(args))
        self.enc_stream = plan_opts(args).get("enc_stream", -1)
        self.size_linear = plan_opts(args).get("size_linear", -1)
        self.fixed_path = plan_opts(args).get("fixed_path", 0)
        self.stream = torch.cuda.current_stream()
        self.s = self.stream.cuda_stream
        self.mar.status.init(self.s)
        self.evs = []

    def sync(self):
        torch.cuda.synchronize()

    # HIP events bracket the kernels of every E-th step of the timed region
    # (--event-every E): before its encode, between encode and decode, after
    # its decode.  An event between two kernels is itself a command on the
    # stream that widens the gap between them; the other steps run without.
    def step(self, record=False):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if record else None
        if ev is not None:
            ev[0].record(self.stream)
        self.mar.launch_encode(self.nat, self.n, self.xdr, heap=self.heap, offsets=self.offsets, stream=self.s)
        if ev is not None:
            ev[1].record(self.stream)
        self.mar.launch_decode(self.xdr, self.n, self.back, offsets=self.offsets, heap_out=self.heap_out,
                               stream=self.s)
        if ev is not None:
            ev[2].record(self.stream)
            self.evs.append(ev)

    def launch_ms(self):
        """(encode ms, decode ms) of every recorded step."""
        return ([e[0].elapsed_time(e[1]) for e in self.evs], [e[1].elapsed_time(e[2]) for e in self.evs])

    def check(self):
        self.mar.check(self.s)

    def round_trip_ok(self) -> bool:
        """decode(encode(x)) == x (fixed) or encode(decode(encode(x))) ==
        encode(x) (var)."""
        if self.plan.is_fixed:
            return bool(torch.equal(self.back, self.nat))
        x2 = torch.empty_like(self.xdr)
        o2 = torch.empty_like(self.offsets)
        self.mar.status.init(self.s)
        self.mar.launch_encode(self.back, self.n, x2, heap=self.heap_out, offsets=o2, stream=self.s)
        self.mar.check(self.s)
        return bool(torch.equal(x2, self.xdr))

    def dominant(self, enc_ms, dec_ms):
        """The dominant kernel (or phase) and its algorithmic bytes per launch
        (DESIGN.md §4), and the launch times it is timed by."""
        plan, n, S_, X = self.plan, self.n, self.plan.stride, self.xdr.numel()
        info = A.XdrgPlanInfo()
        A.check(A.lib().xdrg_plan_get_info(plan.handle, A.C.byref(info)), "xdrg_plan_get_info")
        if plan.is_fixed:
            # encode and decode are the same kernel with the encode / decode
            # permutation programs: read one side, write the other
            # (non-identity layouts: the tile kernel for records of up to 16
            # words each way, xdrgpu.hip run_fixed)
            tile = self.fixed_path == 0 and S_ <= 64 and plan.fixed_size <= 64
            kern = ("k_fixed_reg" if plan.path == A.PATH_FIXED_REG else
                    "k_fixed_tile" if tile else
                    "k_fixed_grp" if info.group_records and self.fixed_path != 2 else "k_fixed_lds")
            return kern, n * S_ + X, enc_ms + dec_ms
        # dominant phase: encode (size pass + block scan + window encode) vs
        # decode (window decode).  Encode reads the native records and the
        # payload heap and writes the stream + record index; decode reads
        # stream + index and writes the native records, the heap (= the
        # stream verbatim) and the decoded element arrays past it (the
        # element area the decode filled: every container's elements, read
        # back from the decoded records' refs).  Scratch (sizes, block sums)
        # is excluded.
        H = 0 if self.heap is None else self.heap.numel()
        enc_alg = n * S_ + H + X + 8 * (n + 1)
        dec_alg = X + 8 * (n + 1) + n * S_ + X + self.element_bytes()
        spec = bool(info.specialized)  # plan-specialized kernels ran (built at warmup)
        sub = bool((plan.cp.ops["flags"] & A.F_SUB).any())  # element subroutines: the frame walk
        deep = A.lib().xdrg_deep_workspace_size(plan.handle, 1) > 0  # recursive: frame walks only
        if deep:  # the frame walks (+ their deep passes), generated or interpreted
            size_k, enc_k, dec_k = (("xdrg_spec_sub_size", "xdrg_spec_sub_encode", "xdrg_spec_sub_decode") if spec
                                    else ("k_sub_size", "k_sub_encode", "k_sub_decode"))
        else:
            # (a linear plan sizes with the generated walk when it has one,
            # XDRG_OPT_SIZE_LINEAR -1; 1 forces k_size_linear)
            size_k = ("k_sub_size" if sub and not spec
                      else "k_size_linear" if plan_linear(plan) and (self.size_linear == 1 or
                                                                    (not spec and self.size_linear != 0))
                      else "xdrg_spec_size" if spec else "k_var_size")
            enc_k = (("xdrg_spec_encode_pre" if walk_first(plan) and self.enc_stream != 0 else "xdrg_spec_encode")
                     if spec
                     else "k_sub_encode" if sub else "k_var_encode_i")
            dec_k = "xdrg_spec_decode_copy" if spec else "k_sub_decode" if sub else "k_var_decode_w"
        if np.mean(enc_ms) >= np.mean(dec_ms):
            return f"{size_k}+k_scan_blocks+{enc_k}", enc_alg, enc_ms
        return dec_k, dec_alg, dec_ms

    def element_bytes(self) -> int:
        """Native bytes of the element arrays a decode writes: count x stride
        of every xvector/pointer field of every record (plans whose
        containers hold fixed-size elements, read from the decoded records)."""
        if self.schema == "rp_list":  # every node past a list's first is an element image
            return int(W.rp_list_nodes(self.n).sum() - self.n) * self.plan.stride
        ops = self.plan.cp.ops
        vec = np.nonzero(ops["kind"] == A.OP_VECTOR)[0]
        if not vec.size:
            return 0
        nat = self.back.view(-1, self.plan.stride)
        total = 0
        for i in vec:
            off, stride = int(ops["noff"][i]), int(ops["arg1"][i])
            cnt = nat[:, off + 8:off + 12].contiguous().view(torch.int32)
            total += int(cnt.to(torch.int64).sum().item()) * stride
        return total

    def shard(self):
        """The rank's encoded stream and record index (for the gather)."""
        return self.xdr, self.offsets


def load_engine(path: str):
    """--engine FILE: a module defining Engine (the tests' CPU stand-in)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_engine", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Engine


def measure(engine, args):
    """Warmup, then exactly args.steps steps bracketed by barrier + sync;
    events around the kernels of every E-th.  Returns (elapsed s, encode
    ms, decode ms)."""
    for _ in range(args.warmup):
        engine.step()
    engine.sync()
    engine.check()
    E = max(1, args.event_every)
    timed = {k for k in range(args.steps) if k % E == E - 1} or {args.steps - 1}
    barrier(engine.dist)
    engine.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        engine.step(k in timed)
    engine.sync()
    barrier(engine.dist)
    elapsed = time.perf_counter() - t0
    engine.check()
    enc_ms, dec_ms = engine.launch_ms()
    return elapsed, enc_ms, dec_ms


def rank_rows(dist, world, mine: list[float], dev):
    """Every rank's row [elapsed, encode ms, decode ms, XDR bytes, achieved
    GB/s, round trip ok] on every rank (one all_gather)."""
    t = torch.tensor(mine, dtype=torch.float64, device=dev)
    if dist is None:
        return t.cpu().numpy()[None, :]
    allr = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allr, t)
    return torch.stack(allr).cpu().numpy()


def gather_leg(engine, dist, rank, world, X_all, X, rows, hashes, key):
    """The one collective: every shard's stream (and
    record index) to rank 0, timed apart from the marshal step.  Rank 0
    gets the report dict; the others None."""
    xdr, offsets = engine.shard()
    engine.sync()
    barrier(dist)
    g0 = time.perf_counter()
    g_stream, g_index = SH.gather_streams(dist, xdr, offsets, rank, world)
    engine.sync()
    g_s = time.perf_counter() - g0
    t = torch.tensor([g_s], dtype=torch.float64, device=engine.dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    g_s = float(t.item())
    if rank != 0:
        return None
    recv = X_all - X
    sha = hashlib.sha256(g_stream.cpu().numpy().tobytes()).hexdigest()
    gather = {"gather_ms": round(g_s * 1e3, 3), "bytes_to_root": recv, "stream_bytes": int(g_stream.numel()),
              "root_inbound_gib_s": round(recv / GIB / g_s, 2),
              "encode_plus_gather_gib_s": round(X_all / GIB / (float(rows[:, 1].max()) * 1e-3 + g_s), 2),
              "sha256": sha,
              "collective": f"exact-size point-to-point sends to rank 0 ({engine.backend}; RCCL over xGMI on "
                            "MI355X)"}
    if g_index is not None:
        gather["index_sha256"] = hashlib.sha256(g_index.cpu().numpy().tobytes()).hexdigest()
    if key in hashes:
        gather["bit_exact_vs_reference"] = sha == hashes[key]["xdr"]
    return gather


def report(args, engine, world, rows, X, kern, alg_bytes, launches, enc_ms, dec_ms, bit_exact, gather):
    """Rank 0's JSON line (the bench contract) from the per-rank rows."""
    n, S_ = engine.n, engine.plan.stride
    elapsed = float(rows[:, 0].max())
    X_all = int(rows[:, 3].sum())
    value = 2 * X_all / GIB / (elapsed / args.steps)
    avg = float(np.mean(launches))
    achieved = alg_bytes / (avg * 1e-3) / 1e9
    E = max(1, args.event_every)
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            tab = tj.get("hbm_bytes_per_launch", {})
            parts = [tab.get(f"{args.schema}:{k}") for k in kern.split("+")]
            if tj.get("records") == n and all(p is not None for p in parts):
                traffic = int(sum(parts))  # multi-kernel phases: sum of their launches
        except Exception:
            traffic = None
    wl = {"rec128": "rec128: fixed-width 128-byte XDR records",
          "numerics": "numerics (tests/xdrtest.x) fixed 44-byte records, 56-byte native",
          "recvar": "recvar: opaque<256> + string<64> variable-length records",
          "rpc": "rpc_msg (xdrpp/rpc_msg.x) nested discriminated unions",
          "vecrec": "vecrec: int<16>, mismatch_info *, vpair<8> counted/optional containers",
          "containertest": "containertest (tests/xdrtest.x): u_4_12 uvec<> (variable-size union "
                           "elements, element subroutines) + string sarr[2]",
          "rp_list": "rp_list (xdrpp/rpcb_prot.x rp__list, the RPCBPROC_DUMP reply): linked lists of rpcb "
                     "entries, 1-4 nodes, a 500-node list every 65536 (recursive element subroutine)"}[args.schema]
    line = {
        "metric": ("XDR encode+decode GiB/s (device-resident, 1M×128B records) + %HBM roofline"
                   if args.schema == "rec128" else
                   f"XDR encode+decode GiB/s (device-resident, {args.schema}) + %HBM roofline"),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 seeds 0x5EED000x per SURVEY.md §8(d); FP fields as raw bit patterns)",
        "config": {"workload": f"{wl}, {n} records per GPU x {world} GPU(s), encode (xdr_to_opaque) + "
                               "decode (xdr_from_opaque), device-resident",
                   "schema": args.schema, "records_per_gpu": n, "records_total": n * world,
                   "xdr_bytes_per_gpu": X, "native_stride": S_, "parallelism": f"dp{world}",
                   **({"plan_options": plan_opts(args)} if plan_opts(args) else {})},
        "encode_ms": round(float(np.mean(enc_ms)), 4),
        "decode_ms": round(float(np.mean(dec_ms)), 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": kern, "median_launch_ms": round(float(np.median(launches)), 4),
                     "alg_bytes_per_launch": alg_bytes,
                     "timed_launches": len(launches),
                     "protocol": f"HIP events on the launch stream around both kernels of every {E}th timed step"},
        "round_trip_ok": bool(rows[:, 5].all()),
        "bit_exact_vs_reference": bit_exact,
    }
    if world > 1:
        line["per_rank"] = [{"rank": r, "gib_s": round(2 * row[3] / GIB / (row[0] / args.steps), 2),
                             "encode_ms": round(row[1], 4), "decode_ms": round(row[2], 4),
                             "roofline_frac": round(row[4] / HBM_PEAK_GBS, 4)}
                            for r, row in enumerate(rows)]
    if gather is not None:
        line["gather"] = gather
    return line


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    Engine = load_engine(args.engine) if args.engine else GpuEngine
    dist, world, rank, local = dist_init(args, Engine.backend)
    n = args.n if args.n is not None else (1 << 20 if world == 1 else 1 << 21)
    engine = Engine(args, n, rank, world, local)
    engine.dist = dist
    elapsed, enc_ms, dec_ms = measure(engine, args)

    # correctness of what was timed; on the 1-GPU headline config the stream
    # also hashes to the reference's output
    ok_rt = engine.round_trip_ok()
    xdr, _ = engine.shard()
    X = xdr.numel()
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    hashes = json.load(open(man))["hashes"] if os.path.exists(man) else {}
    bit_exact = None
    if world == 1 and f"{args.schema}_{n}" in hashes:
        bit_exact = hashlib.sha256(xdr.cpu().numpy().tobytes()).hexdigest() == hashes[f"{args.schema}_{n}"]["xdr"]

    kern, alg_bytes, launches = engine.dominant(enc_ms, dec_ms)
    achieved = alg_bytes / (float(np.mean(launches)) * 1e-3) / 1e9
    rows = rank_rows(dist, world, [elapsed, float(np.mean(enc_ms)), float(np.mean(dec_ms)), float(X), achieved,
                                   float(ok_rt)], engine.dev)
    X_all = int(rows[:, 3].sum())
    gather = None
    if dist is not None and not args.no_gather:
        gather = gather_leg(engine, dist, rank, world, X_all, X, rows, hashes, f"{args.schema}_mgpu_{n * world}")
        if gather is not None and "bit_exact_vs_reference" in gather:
            bit_exact = gather["bit_exact_vs_reference"]
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    line = report(args, engine, world, rows, X, kern, alg_bytes, launches, enc_ms, dec_ms, bit_exact, gather)
    if isinstance(engine, GpuEngine) and world == 1:
        extra_legs(args, engine, line, alg_bytes)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def extra_legs(args, engine, line, alg_bytes):
    """The legs beside the headline (1 GPU): the fixed path past the cache,
    cold caches, record-marked messages, RPC headers, host-inclusive rates
    with the PCIe ceiling, and the CPU reference on this host's cores."""
    plan, mar, nat, heap, n = engine.plan, engine.mar, engine.nat, engine.heap, engine.n
    if plan.is_fixed and args.schema == "rec128" and not args.no_large:
        try:
            line["large_batch_16m"] = large_batch(mar, nat.device)
            torch.cuda.empty_cache()
            ceil = copy_ceiling(2048)  # the same bytes per buffer as 16M records
            if ceil is not None:
                lb = line["large_batch_16m"]
                lb["copy_ceiling"] = ceil
                lb["frac_of_copy_ceiling"] = round(lb["achieved_GBps"] / (ceil["best_tb_s"] * 1e3), 4)
        except Exception as e:  # reported, never fatal
            line["large_batch_16m"] = {"error": str(e)[:200]}
    if plan.is_fixed and args.schema == "rec128" and not args.no_shard:
        try:
            line["shard_2m"] = shard_leg(nat.device)
        except Exception as e:  # reported, never fatal
            line["shard_2m"] = {"error": str(e)[:200]}
    headline = args.schema == "rec128"
    if (args.cold or headline) and not args.no_cold and plan.is_fixed:
        line["cold_cache"] = cold_cache(mar, nat, engine.xdr, engine.back, n, alg_bytes)
        engine.check()
    if not plan.is_fixed and not args.no_plain:
        try:
            line["plain_stream"] = plain_stream_leg(args.schema, engine, line["decode_ms"])
        except Exception as e:  # reported, never fatal
            line["plain_stream"] = {"error": str(e)[:200]}
    if args.msgs:
        line["messages"] = messages_leg(args.schema, plan, mar, nat, heap, n)
    if args.rpc:
        line["rpc_headers"] = rpc_leg(nat.device)
    if (args.host_inclusive or headline) and not args.no_host_inclusive:
        try:
            line["host_inclusive"] = (host_inclusive(mar, plan, nat, n, plan.fixed_size) if plan.is_fixed
                                      else host_inclusive_var(mar, plan, nat, heap, n))
        except Exception as e:  # reported, never fatal
            line["host_inclusive"] = {"error": str(e)[:200]}
    if not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(args.schema, n, args.cpu_threads)
        except Exception as e:
            line["cpu_baseline"] = {"error": str(e)[:200]}


if __name__ == "__main__":
    main()
