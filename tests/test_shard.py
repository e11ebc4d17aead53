"""CPU, world_size 2 over gloo: the multi-GPU data-parallel path.

Each rank builds its shard (xdrpp_amd.shard.shard_inputs), marshals it --
here with the oracle, standing in for the GPU on a CPU host -- and the
shards are gathered to rank 0 with the same gather_streams the bench uses
over RCCL.  Rank 0 checks that the concatenated stream and rebased record
index equal the single-process encoding of the whole batch: sharding is
exact by construction, with no collective on the data path.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from xdrpp_amd import shard as SH  # noqa: E402

N_PER_RANK = 300
WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, schema, result_dir):
    import oracle_bridge as O
    from xdrpp_amd import schemas as S
    from xdrpp_amd.xdr_types import compile_plan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cp = compile_plan(S.ALL[schema])
        nat, heap = SH.shard_inputs(schema, N_PER_RANK, rank, world)
        x, offs = O.encode(cp, nat, N_PER_RANK, heap)
        xt = torch.from_numpy(x.copy())
        ot = torch.from_numpy(offs.view(np.int64).copy()) if cp.is_var else None
        stream, index = SH.gather_streams(dist, xt, ot, rank, world)
        if rank == 0:
            np.save(os.path.join(result_dir, "stream.npy"), stream.numpy())
            if index is not None:
                np.save(os.path.join(result_dir, "index.npy"), index.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("schema", ["rec128", "numerics", "recvar", "rpc"])
def test_sharded_encode_equals_whole_batch(tmp_path, schema):
    import oracle_bridge as O
    from xdrpp_amd import schemas as S
    from xdrpp_amd import workloads as W
    from xdrpp_amd.xdr_types import compile_plan

    mp.start_processes(_worker, args=(WORLD, _free_port(), schema, str(tmp_path)),
                       nprocs=WORLD, join=True, start_method="spawn")
    stream = np.load(tmp_path / "stream.npy")
    cp = compile_plan(S.ALL[schema])
    whole_nat, whole_heap = W.GENERATORS[schema](N_PER_RANK * WORLD,
                                                  seed=SH.seed_for(schema, WORLD))
    want, woffs = O.encode(cp, whole_nat, N_PER_RANK * WORLD, whole_heap)
    assert np.array_equal(stream, want)
    if cp.is_var:
        index = np.load(tmp_path / "index.npy")
        assert np.array_equal(index.view(np.uint64), woffs)


def test_shard_range():
    assert SH.shard_range(0, 4, 10) == (0, 10)
    assert SH.shard_range(3, 4, 10) == (30, 10)
    with pytest.raises(ValueError):
        SH.shard_range(4, 4, 10)


def test_mgpu_seed():
    from xdrpp_amd import workloads as W
    assert SH.seed_for("rec128", 1) == W.SEED_REC128
    assert SH.seed_for("rec128", 8) == W.SEED_REC128_MGPU
    assert SH.seed_for("recvar", 8) == W.SEED_RECVAR
