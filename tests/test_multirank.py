"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): env sharding by global env
index and the single episode-record all-gather (bench.py / mxabides.shard).  The per-env
records come from the C oracle here (CPU); on the GPU box the same code runs over RCCL with
the HIP engine producing the records."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


import pyoracle
from mxabides import shard

CONFIG = "sparse_zi_100"
N_PER_RANK = 3
MAX_POPS = 4000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _records(seeds):
    ev, hs, _ = pyoracle.run_batch(CONFIG, seeds, 1, MAX_POPS)
    rec = np.zeros((len(seeds), shard.RECORD_WORDS), dtype=np.int64)
    rec[:, 0] = ev
    rec[:, 1] = hs.view(np.int64)
    return torch.from_numpy(rec)


def _worker(rank, world, port, batch, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seeds = shard.env_seeds(batch, rank, world, N_PER_RANK)
        allrec = shard.gather_records(_records(seeds), world)
        if rank == 0:
            np.save(out_path, allrec.numpy())
    finally:
        dist.destroy_process_group()


def test_env_seeds_independent_of_world_size():
    one = np.concatenate([shard.env_seeds(1, 0, 1, 8)])
    two = np.concatenate([shard.env_seeds(1, r, 2, 4) for r in range(2)])
    four = np.concatenate([shard.env_seeds(1, r, 4, 2) for r in range(4)])
    assert (one == two).all() and (one == four).all()
    assert one[0] == (shard.SEED0 + 8) & 0xFFFFFFFF


def test_gloo_world2_gather_matches_single_process(tmp_path):
    world, batch = 2, 1
    out = tmp_path / "rec.npy"
    mp.start_processes(_worker, args=(world, _free_port(), batch, str(out)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    seeds = shard.env_seeds(batch, 0, 1, world * N_PER_RANK)
    want = _records(seeds).numpy()
    assert got.shape == (world * N_PER_RANK, shard.RECORD_WORDS)
    assert (got == want).all()
