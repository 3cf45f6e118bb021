#!/usr/bin/env python3
"""Capacity proof for a configuration's compile-time queue / book sizes: runs the C oracle
(test infrastructure) over EVERY seed that `bench.py --gpus N` (N <= 8) draws with the default
warmup + steps (batches 0..3, shard.env_seeds(batch, rank, 8, envs)) and records the maxima of
pending events and resting orders (ora_run_batch_stats).  A capacity is proven for the bench
when the maxima stay below it.

    python tools/capacity_sweep.py CONFIG ENVS [THREADS] -> profiles/r04/capacity_<CONFIG>.json
    python tools/capacity_sweep.py CONFIG ENVS THREADS B0 B1 -> batches B0..B1-1 instead of 0..3,
        written to profiles/r05/capacity_<CONFIG>_b<B0>_<B1>.json (a longer --steps / --warmup run)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "marl-optimal-execution_amd")]
import pyoracle  # noqa: E402
from mxabides import shard  # noqa: E402

cfg, envs = sys.argv[1], int(sys.argv[2])
threads = int(sys.argv[3]) if len(sys.argv) > 3 else os.cpu_count()
b0, b1 = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (0, 4)
seeds = np.unique(np.concatenate([shard.env_seeds(b, r, 8, envs) for b in range(b0, b1) for r in range(8)]))
t0 = time.time()
st = pyoracle.batch_stats(cfg, seeds, threads)
out = {"config": cfg, "envs_per_gpu": envs, "seed_sets": "shard.env_seeds(batch %d-%d, rank 0-7, world 8)" % (b0, b1 - 1),
       "n_seeds": int(len(seeds)), "max_pending_events": int(st[:, 0].max()), "max_resting_orders": int(st[:, 1].max()),
       "max_open_orders_one_agent": int(st[:, 2].max()), "max_tx_records": int(st[:, 3].max()),
       "argmax_seed_pending": int(seeds[st[:, 0].argmax()]), "argmax_seed_resting": int(seeds[st[:, 1].argmax()]),
       "seconds": time.time() - t0}
dst = (os.path.join(ROOT, "profiles", "r04", "capacity_%s.json" % cfg) if (b0, b1) == (0, 4) else
       os.path.join(ROOT, "profiles", "r05", "capacity_%s_b%d_%d.json" % (cfg, b0, b1)))
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out))
