"""bench.py's multi-rank launcher on CPU (VERDICT r02 "missing" 1): `bench.py --gpus 2` starts two
rank processes itself (no torchrun), they rendezvous over gloo, time the same loop (barrier,
max over ranks), all-gather the per-env episode records, and rank 0 prints one JSON line.  The
stub engine stands in for the HIP market (records derived from the env seeds), so the checks
are about the harness: world size, global env count, gathered rows in global env order."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub"] + list(extra), env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_launcher_world2_gathers_in_global_env_order():
    out = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--envs", "3")
    assert out["n_gpus"] == 2
    assert out["config"]["global_envs"] == 6 and out["config"]["envs_per_gpu"] == 3
    assert out["config"]["gathered_records"] == {"own_rows_in_place": True, "global_env_order": True}
    sys.path.insert(0, os.path.join(ROOT, "marl-optimal-execution_amd"))
    from mxabides import shard
    # events of the two timed batches (1, 2) of all 6 global envs: 1000 + seed % 997
    seeds = np.concatenate([shard.env_seeds(k, r, 2, 3) for k in (1, 2) for r in range(2)]).astype(np.int64)
    assert out["config"]["events_per_step"] * 2 == (1000 + seeds % 997).sum()
    assert out["value"] > 0 and out["scaling"] == "weak"


def test_bench_launcher_single_rank():
    out = _bench("--steps", "1", "--warmup", "0", "--envs", "5")
    assert out["n_gpus"] == 1 and out["config"]["global_envs"] == 5
    assert out["config"]["gathered_records"]["global_env_order"]
