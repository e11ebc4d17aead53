"""A CPU stand-in for bench.py's GPU step (TEST INFRASTRUCTURE ONLY).

`python bench.py --gpus 2 --engine tests/bench_cpu_engine.py` runs
bench.py's own multi-rank path -- launch_ranks (torch.distributed.run),
the timed loop, the per-rank rows, the gather of the shards to rank 0 and
the report line -- with each rank's encode and decode done by the C
restatement (oracle/) on CPU tensors over gloo, so that the plumbing the
8-GPU run depends on is exercised on a CPU host (tests/test_bench_mgpu.py).
bench.py never imports this file on its own.
"""
from __future__ import annotations

import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import oracle_bridge as O  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import shard as SH  # noqa: E402
from xdrpp_amd.xdr_types import compile_plan  # noqa: E402


class Engine:
    backend = "gloo"

    def __init__(self, args, n, rank, world, local):
        self.dev = torch.device("cpu")
        self.schema, self.n = args.schema, n
        self.cp = compile_plan(S.ALL[args.schema])
        self.nat, self.heap = SH.shard_inputs(args.schema, n, rank, world)
        self.plan = types.SimpleNamespace(stride=self.cp.stride, is_fixed=not self.cp.is_var)
        self.times = []
        self.x = self.offs = self.back = None

    def sync(self):
        pass

    def step(self, record=False):
        t0 = time.perf_counter()
        self.x, self.offs = O.encode(self.cp, self.nat, self.n, self.heap)
        t1 = time.perf_counter()
        self.back = O.decode(self.cp, self.x, self.n, self.offs if self.cp.is_var else None)
        t2 = time.perf_counter()
        if record:
            self.times.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))

    def launch_ms(self):
        return [t[0] for t in self.times], [t[1] for t in self.times]

    def check(self):
        pass  # the oracle raises on a data error

    def round_trip_ok(self) -> bool:
        nat2, heap2 = self.back
        if not self.cp.is_var:
            return bool(np.array_equal(nat2, self.nat))
        x2, _ = O.encode(self.cp, nat2, self.n, heap2)
        return bool(np.array_equal(x2, self.x))

    def dominant(self, enc_ms, dec_ms):
        return "cpu-oracle (test stand-in)", self.n * self.cp.stride + int(self.x.size), enc_ms + dec_ms

    def shard(self):
        offs = torch.from_numpy(self.offs.view(np.int64).copy()) if self.cp.is_var else None
        return torch.from_numpy(np.ascontiguousarray(self.x)), offs
