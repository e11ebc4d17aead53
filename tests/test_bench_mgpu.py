"""bench.py's multi-rank path, rehearsed on CPU at world size 2 over gloo.

`bench.py --gpus 2` starts its own ranks (launch_ranks ->
torch.distributed.run), times the step on every rank, gathers the per-rank
rows and the encoded shards to rank 0 (xdrpp_amd.shard.gather_streams:
exact-size point-to-point sends) and prints the report line -- here with
tests/bench_cpu_engine.py (the C restatement) in place of the GPU step.
The gathered stream must be the single-process encoding of the whole
batch (contiguous shards, no collective on the data
path), byte for byte.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

import oracle_bridge as O
from xdrpp_amd import schemas as S
from xdrpp_amd import shard as SH
from xdrpp_amd import workloads as W
from xdrpp_amd.xdr_types import compile_plan

N = 700


@pytest.mark.parametrize("schema", ["rec128", "recvar"])
def test_bench_two_ranks(schema):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--n", str(N), "--steps", "3",
           "--warmup", "1", "--event-every", "1", "--schema", schema,
           "--engine", os.path.join(ROOT, "tests", "bench_cpu_engine.py")]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["records_total"] == 2 * N
    assert [r["rank"] for r in line["per_rank"]] == [0, 1]
    assert line["round_trip_ok"] is True
    # the whole batch, encoded in one process
    cp = compile_plan(S.ALL[schema])
    nat, heap = W.GENERATORS[schema](2 * N, seed=SH.seed_for(schema, 2))
    want, woffs = O.encode(cp, nat, 2 * N, heap)
    g = line["gather"]
    r1_bytes = len(want) - int(woffs[N]) if cp.is_var else N * cp.fixed_size
    assert g["bytes_to_root"] == r1_bytes
    assert g["stream_bytes"] == len(want)
    assert g["sha256"] == hashlib.sha256(bytes(want)).hexdigest()
    if cp.is_var:
        assert g["index_sha256"] == hashlib.sha256(woffs.view(np.int64).tobytes()).hexdigest()
    X_all = len(want)
    assert line["value"] == pytest.approx(2 * X_all / 2**30 / (line["ms_per_step"] * 1e-3), rel=0.01, abs=0.01)


@pytest.mark.parametrize("schema", ["rp_list", "containertest", "recvar", "rpc"])
def test_port_baseline_runs(schema):
    """bench.py's cpu_baseline port leg (oracle/cpu_bench.c) on a small
    batch of every variable-length bench schema, two threads: the decode of
    plans with element arrays (rp_list, containertest) gets a heap of its
    own per thread and decodes what the encode wrote."""
    sys.path.insert(0, ROOT)
    import bench
    n = 3000
    nat, heap = W.GENERATORS[schema](n)
    r = bench._port_baseline(schema, n, 2, 1, nat, heap)
    assert r["encode_gib_s"] > 0 and r["decode_gib_s"] > 0 and r["threads"] == 2
