"""Headline benchmark: device-resident XDR encode+decode of 1M x 128-byte
records (BASELINE.json config 2) on N MI355X GPUs.

One step = encode the rank's batch (native rec128 structs -> XDR stream,
= xdr_to_opaque of the batch) + decode it back (= xdr_from_opaque).
Inputs are resident in HBM before timing.  Multi-GPU: one process per GPU
(torchrun), each rank owns a contiguous range of the global record index
(weak scaling, no collective on the data path); the timed region is
bracketed by barrier + synchronize and the max over ranks is reported.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n RECORDS]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
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
from xdrpp_amd import workloads as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=1 << 20, help="records per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="also time an RCCL gather of encoded shards to rank 0 (reported apart)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def dist_init(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, world, rank, local
    torch.cuda.set_device(local)
    return None, 1, 0, local


def barrier(dist):
    if dist is not None:
        dist.barrier()


def cpu_baseline(n_records: int, threads: int) -> dict | None:
    """The reference's CPU marshaler on this host: oracle/_ref/ref_golden
    (xdrpp/marshal.cc compiled from the reference sources) when present,
    else the C restatement in oracle/ (single thread)."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        reps = 10
        out = subprocess.run([ref, "bench", "rec128", str(n_records), str(threads), str(reps)],
                             capture_output=True, text=True, timeout=600)
        if out.returncode == 0:
            r = json.loads(out.stdout.strip().splitlines()[-1])
            return {"value": round(r["encode_decode_gib_s"], 4), "unit": "GiB/s", "cores": threads,
                    "kind": "reference",
                    "sample": f"rec128 x {n_records} (the full batch), xdr_put/xdr_get streams over "
                              f"{threads} contiguous slices, best of {reps}; per-record "
                              f"xdr_to_opaque {r['to_opaque_gib_s']:.3f} GiB/s",
                    "encode_gib_s": round(r["encode_gib_s"], 4),
                    "decode_gib_s": round(r["decode_gib_s"], 4)}
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as O

    plan = __import__("xdrpp_amd.xdr_types", fromlist=["compile_plan"]).compile_plan(S.rec128)
    ns = min(n_records, 1 << 18)
    nat, _ = W.rec128(ns)
    t0 = time.perf_counter()
    x, _ = O.encode(plan, nat, ns)
    t1 = time.perf_counter()
    O.decode(plan, x, ns)
    t2 = time.perf_counter()
    return {"value": round(2 * x.size / GIB / (t2 - t0), 4), "unit": "GiB/s", "cores": 1,
            "kind": "port", "sample": f"rec128 x {ns}, oracle/xdr_oracle.c, 1 thread",
            "encode_gib_s": round(x.size / GIB / (t1 - t0), 4),
            "decode_gib_s": round(x.size / GIB / (t2 - t1), 4)}


def host_inclusive(mar, plan, nat_dev, n, W_, reps=5, nstreams=2, chunk_records=1 << 17):
    """Pinned host -> device -> encode -> host, chunked over streams (and the
    decode direction).  PCIe-bound; reported apart, never as `value`."""
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
            "chunk_records": chunk_records, "streams": nstreams}


def main():
    args = parse()
    dist, world, rank, local = dist_init(args)
    dev = torch.device("cuda", local)
    n = args.n
    plan = M.Plan(S.rec128)
    W_ = plan.fixed_size
    S_ = plan.stride
    mar = M.Marshaler(plan, dev)
    seed = W.SEED_REC128 if world == 1 else W.SEED_REC128_MGPU
    nat_np, _ = W.rec128(n, seed=seed, first=rank * n)
    nat = torch.from_numpy(nat_np).to(dev)
    xdr = torch.empty(n * W_, dtype=torch.uint8, device=dev)
    back = torch.empty(n * S_, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    mar.status.init(s)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        mar.launch_encode(nat, n, xdr, stream=s)
        if ev is not None:
            ev[1].record(stream)
        mar.launch_decode(xdr, n, back, stream=s)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    mar.check(s)

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    mar.check(s)
    enc_ms = [e[0].elapsed_time(e[1]) for e in evs]
    dec_ms = [e[1].elapsed_time(e[2]) for e in evs]

    # correctness of what was timed: decode(encode(x)) == x everywhere, and
    # on rank 0 of the 1-GPU config the stream hashes to the reference's.
    ok_rt = bool(torch.equal(back, nat))
    bit_exact = None
    man = os.path.join(ROOT, "tests", "golden", "manifest.json")
    if world == 1 and n == (1 << 20) and os.path.exists(man):
        want = json.load(open(man))["hashes"]["rec128_1048576"]["xdr"]
        bit_exact = hashlib.sha256(xdr.cpu().numpy().tobytes()).hexdigest() == want

    gather_ms = None
    if args.gather and dist is not None:
        gl = [torch.empty_like(xdr) for _ in range(world)] if rank == 0 else None
        torch.cuda.synchronize()
        barrier(dist)
        g0 = time.perf_counter()
        dist.gather(xdr, gl, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    xdr_bytes_step = 2 * n * W_ * world
    value = xdr_bytes_step / GIB / (elapsed / args.steps)
    # dominant kernel: k_fixed_reg (encode and decode are the same kernel
    # with the encode / decode permutation programs)
    alg_bytes = n * (S_ + W_)  # read one side + write the other, per launch
    med = float(np.median(enc_ms + dec_ms))
    avg = float(np.mean(enc_ms + dec_ms))
    achieved = alg_bytes / (avg * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get("records") == n and tj.get("kernel", "").startswith("k_fixed_reg"):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    line = {
        "metric": "XDR encode+decode GiB/s (device-resident, 1M×128B records) + %HBM roofline",
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
        "data": "synthetic (splitmix64 seed 0x5EED0002 / 0x5EED0005, FP fields as raw bit patterns)",
        "config": {"workload": "rec128: 1M fixed-width 128-byte XDR records per GPU, "
                               "encode (xdr_to_opaque) + decode (xdr_from_opaque), device-resident",
                   "records_per_gpu": n, "record_bytes": W_, "native_stride": S_,
                   "parallelism": f"dp{world}"},
        "encode_ms": round(float(np.mean(enc_ms)), 4),
        "decode_ms": round(float(np.mean(dec_ms)), 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": "k_fixed_reg", "median_launch_ms": round(med, 4),
                     "alg_bytes_per_launch": alg_bytes},
        "round_trip_ok": ok_rt,
        "bit_exact_vs_reference": bit_exact,
    }
    if gather_ms is not None:
        line["gather_ms"] = round(gather_ms, 3)
    if world == 1 and not args.no_host_inclusive:
        try:
            line["host_inclusive"] = host_inclusive(mar, plan, nat, n, W_)
        except Exception as e:  # reported, never fatal
            line["host_inclusive"] = {"error": str(e)[:200]}
    if world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        try:
            line["cpu_baseline"] = cpu_baseline(n, threads)
        except Exception as e:
            line["cpu_baseline"] = {"error": str(e)[:200]}
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
