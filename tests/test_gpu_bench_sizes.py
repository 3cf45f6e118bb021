"""Parity at the bench sizes of every `bench.py --config` workload (VERDICT r02 "weak" 1): every
env of the exact bench batches is compared with the C oracle, including WHICH envs end in an
error and with which code.  The reference raises where the oracle fails (a pandas / numpy /
TypeError crash path of the reference itself); a device-only capacity error would be a
divergence and fails these tests.

Workloads (seeds as bench.py draws them, shard.env_seeds(batch, rank 0, world 1, n)):
* rmsc02 x4096, batches 0-2 (bench: warmup 1 + 2 timed steps), obi_rmsc02 x4096, rmsc01 x4096,
  random_fund_value / random_fund_diverse x2048, sparse_zi_1000 x1024 (rank 0 batch 0 and rank 7
  of 8 batch 3) — Kernel.runner configs (Kernel.py:190-292);
* rmsc03 with a SpreadBasedMarketMakerAgent (subscribe / polling) x4096: 899 polling envs end in
  the agent's own UnboundLocalError (oracle -18, device 28);
* rmsc03_rl x4096 — GymKernel.stepRunner (GymKernel.py:158-306) with a fixed host action stream of
  the bench's distribution (x ~ U(0, 0.01), level shares U(0, 1));
* marketreplay IBM 2003-01-14 and GOOG 2012-06-21 x512 — ABIDESEnv.step over a whole episode.
"""
import os

import numpy as np
import pytest

import pyoracle
from mxabides import shard, tape

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)
GOLD = os.path.join(os.path.dirname(__file__), "golden")

# oracle fail() code -> device env error code (mxa_layout.h ERR_*) for the reference's own crash paths
ORACLE_TO_DEVICE = {-3: 6, -5: 5, -6: 7, -7: 13, -8: 14, -11: 17, -13: 19, -14: 21, -16: 23, -18: 28}
GYM_ERR = {-8: (14, 15)}  # get_observation/get_reward (14) or ExecutionAgent.kernelStopping (15)


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def _check_batch(s, ev, hs, er):
    dev_err = np.where(s["status"] == 2, s["err"], 0)
    want = np.array([ORACLE_TO_DEVICE.get(int(x), 1000 + int(x)) if x else 0 for x in er])
    bad = np.nonzero(dev_err != want)[0]
    assert len(bad) == 0, "env (device err, oracle err): %s" % [(int(i), int(dev_err[i]), int(er[i])) for i in bad[:20]]
    assert (s["status"][er == 0] == 1).all()
    assert (s["events"] == ev).all(), np.nonzero(s["events"] != ev)[0][:20]
    assert (s["hash"] == hs).all(), np.nonzero(s["hash"] != hs)[0][:20]


# (batch, rank, world) seed sets of shard.env_seeds: batch 0 of rank 0 everywhere; rmsc02's three
# bench batches; sparse_zi_1000 also the last batch of rank 7 of 8 (bench.py --gpus 8, warmup 1 +
# steps 3), whose capacities are sized close to the oracle maximum
B0 = ((0, 0, 1),)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg,n,sets", [("rmsc02", 4096, ((0, 0, 1), (1, 0, 1), (2, 0, 1))), ("obi_rmsc02", 4096, B0),
                                        ("rmsc01", 4096, B0), ("random_fund_value", 2048, B0),
                                        ("random_fund_diverse", 2048, B0), ("hist_fund_value", 2048, B0),
                                        ("hist_fund_diverse", 2048, B0), ("rmsc03_sbmm", 4096, B0),
                                        ("rmsc03_sbmm_poll", 4096, B0),
                                        ("sparse_zi_1000", 1024, ((0, 0, 1), (3, 7, 8)))])
def test_gpu_bench_batches_equal_oracle(mx, cfg, n, sets):
    from golden_util import market_kw
    m = mx.VecMarket(cfg, shard.env_seeds(*sets[0], n), **market_kw(cfg))
    for bset in sets:
        seeds = shard.env_seeds(*bset, n)
        m.set_seeds(seeds)
        m.reset()
        m.run()
        s = m.summary()
        ev, hs, er, _ = pyoracle.run_batch_err(cfg, seeds, THREADS)
        _check_batch(s, ev, hs, er)


def _gym_compare(v, r, n_steps, acts):
    """step every env through the device, compare per env with the oracle batch r"""
    n = v.n_envs
    alive = np.ones(n, dtype=bool)
    last_obs = np.zeros((n, 9))
    steps = np.zeros(n, dtype=np.int32)
    for i in range(n_steps):
        obs, done, valid, err = v.step(acts[i])
        upd = alive & valid & ~err
        last_obs[upd] = obs[upd]
        steps[alive] += 1
        alive &= ~(done | err)
        if not alive.any():
            break
    s = v.summary()
    dev_err = np.where(s["status"] == 2, s["err"], 0)
    for e in range(n):
        o = int(r["err"][e])
        ok = dev_err[e] in GYM_ERR[o] if o else dev_err[e] == 0
        assert ok, (e, int(dev_err[e]), o)
    assert (steps == r["steps"]).all(), np.nonzero(steps != r["steps"])[0][:20]
    assert (s["events"] == r["events"]).all(), np.nonzero(s["events"] != r["events"])[0][:20]
    assert (s["hash"] == r["hash"]).all(), np.nonzero(s["hash"] != r["hash"])[0][:20]
    np.testing.assert_allclose(last_obs, r["obs"], rtol=1e-9, atol=1e-12)
    return dev_err


@pytest.mark.timeout(600)
def test_gpu_rmsc03_rl_bench_size_equals_oracle(mx):
    from mxabides.gym import VecABIDESEnv
    n, n_steps = 4096, 27
    seeds = shard.env_seeds(0, 0, 1, n)
    rs = np.random.RandomState(2024)
    acts = rs.uniform(0, 1, (n_steps, n, 3))
    acts[:, :, 0] *= 0.01
    r = pyoracle.gym_batch(acts, THREADS, seeds=seeds)
    v = VecABIDESEnv(seeds=seeds)
    dev_err = _gym_compare(v, r, n_steps, acts)
    assert 0 < (dev_err != 0).sum() < n  # the reference's ValueError path is reached, and not everywhere


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tname", ["IBM_2003-01-14", "GOOG_2012-06-21"])
def test_gpu_replay_bench_size_equals_oracle(mx, tname):
    from mxabides.gym import VecABIDESEnv
    tp = tape.Tape.load(os.path.join(GOLD, "tape_%s.npz" % tname))
    n, n_steps = 512, 761
    rs = np.random.RandomState(99)
    acts = rs.uniform(0, 1, (n_steps, n, 3))
    acts[:, :, 0] *= 0.01
    r = pyoracle.gym_batch(acts, THREADS, tape=tp)
    v = VecABIDESEnv(tp, n)
    _gym_compare(v, r, n_steps, acts)
