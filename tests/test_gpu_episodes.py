"""Consecutive episodes of one process on the GPU:
a GymKernel handle's mxa_reset continues Order.order_id / Order._order_ids from the env's
previous episode (util/order/Order.py:8-9, 27-42; ABIDESEnv.py:51-57).  Against the reference's
own multi-episode fixtures (tests/golden/gen_episodes_fixtures.py) and the C oracle."""
import os

import numpy as np
import pytest

import pyoracle
from mxabides.gym import VecABIDESEnv
from test_oracle_episodes import EPISODE_FIXTURES, GOLD, OBS_RTOL, agents_match, fixture_tape, load_eps

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", EPISODE_FIXTURES)
def test_gpu_consecutive_episodes_match_reference(name):
    if not os.path.exists(os.path.join(GOLD, name + ".json")):
        pytest.skip("fixture not generated")
    d, z = load_eps(name)
    tp = fixture_tape(d)
    cap = max(len(z["trace_%d" % (k + 1)]) for k in range(len(d["episodes"])))
    v = None
    for k, ep in enumerate(d["episodes"]):
        acts, trace = z["actions_%d" % (k + 1)], z["trace_%d" % (k + 1)]
        if v is None:
            v = VecABIDESEnv(tp, 1, trace_cap=cap) if tp is not None else VecABIDESEnv(seeds=[ep["seed"]], trace_cap=cap)
        else:
            v.reset(seeds=None if tp is not None else [ep["seed"]])
        for i, a in enumerate(acts):
            obs, done, valid, err = v.step(np.asarray(a)[None])
            st = ep["steps"][i]
            assert v.summary()["events"][0] == st["events"], (k, i)
            if "error" in st:
                assert err[0]
                break
            assert not err[0], v.summary()["err"]
            assert int(done[0]) == st["done"], (k, i)
            if st["obs"]:
                np.testing.assert_allclose(obs[0], st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="episode %d step %d" % (k, i))
        s = v.summary()
        assert s["events"][0] == ep["events"]
        assert "%016x" % s["hash"][0] == ep["hash"], k
        assert (v.trace(0)[:len(trace)] == trace).all(), k
        assert v.book(0, 0) == ep["bids"] and v.book(0, 1) == ep["asks"], k
        assert s["order_counter"][0] == ep["order_id_counter"] + 1, k
        agents_match(ep, v.agents(0), d.get("ticker"))


def test_gpu_rl_episodes_equal_oracle_and_fresh_mode():
    """8 envs x 3 episodes with per-env seed sequences and bigger orders; then the same first
    episode with persistence off reproduces a fresh process"""
    n, eps = 8, 3
    rs = np.random.RandomState(17)
    seeds = (rs.randint(0, 2 ** 31, (eps, n))).astype(np.int64)
    acts = rs.uniform(0, 1, (eps, 27, n, 3))
    acts[..., 0] *= 0.02
    v = VecABIDESEnv(seeds=seeds[0])
    oras = [pyoracle.OracleGymEnv(seed=int(seeds[0, e])) for e in range(n)]
    for k in range(eps):
        if k:
            v.reset(seeds=seeds[k])
            for e in range(n):
                oras[e].reset(seed=int(seeds[k, e]))
        alive = np.ones(n, dtype=bool)
        for i in range(27):
            obs, done, valid, err = v.step(acts[k, i])
            for e in np.nonzero(alive)[0]:
                o_obs, o_done, rc = oras[e].step(acts[k, i, e])
                assert bool(err[e]) == (rc != 0), (k, i, e)
                if rc:
                    alive[e] = False
                    continue
                if o_obs is not None:
                    np.testing.assert_allclose(obs[e], o_obs, rtol=OBS_RTOL, atol=1e-12)
                alive[e] = not o_done
            if not alive.any():
                break
        s = v.summary()
        for e in range(n):
            assert s["events"][e] == oras[e].events and s["hash"][e] == oras[e].hash, (k, e)
            assert s["order_counter"][e] == oras[e].order_counter, (k, e)
    assert s["order_counter"].max() > 2 * 38000  # ids continued over three episodes
    v.set_id_persistence(False)
    v.reset(seeds=seeds[0])
    f = [pyoracle.OracleGymEnv(seed=int(seeds[0, e])) for e in range(n)]
    for i in range(27):
        v.step(acts[0, i])
        for e in range(n):
            f[e].step(acts[0, i, e])
    s = v.summary()
    assert all(s["hash"][e] == f[e].hash for e in range(n))
