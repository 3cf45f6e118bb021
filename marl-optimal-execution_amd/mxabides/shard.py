"""Env sharding across ranks (one process per GPU) and the episode-record exchange.

Envs are independent markets, so a batch shards with no data-path collective: rank r of W
owns global envs [r*n, (r+1)*n) of every episode batch, and env g always gets seed
(SEED0 + g) mod 2**32 — results never depend on the world size.  The only
collective is one all-gather of the per-env episode records
(RECORD_WORDS int64 words: events, hash, status, time, ...) at episode end: over RCCL/xGMI on the GPU path
(backend "nccl"), over gloo in the CPU tests.
"""
import numpy as np
import torch
import torch.distributed as dist

SEED0 = 123456789
RECORD_WORDS = 12  # mxa_write_records (include/mxa.h MXA_RECORD_WORDS), int64 each
R_EVENTS, R_HASH, R_STATUS, R_TIME, R_ERR, R_SEED, R_LAST, R_OCNT, R_CASH, R_HOLD, R_GAIN, R_RETURN = range(12)


def env_seeds(batch, rank, world, n_per_rank, seed0=SEED0):
    """uint32 seeds of this rank's envs in episode batch `batch` (weak scaling: n per rank)."""
    first = seed0 + (batch * world + rank) * n_per_rank
    return (np.arange(first, first + n_per_rank, dtype=np.int64) & 0xFFFFFFFF).astype(np.uint32)


def gather_records(local, world):
    """All-gather the [n, RECORD_WORDS] int64 episode records of every rank -> [world * n, RECORD_WORDS], rank-major
    (= global env order).  One collective per episode batch."""
    if world == 1:
        return local
    out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local)
    else:
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
        torch.cat(parts, out=out)
    return out
