"""rmsc03 + DummyRL (BASELINE.json configs[3]) on the GPU: libmxa mxa_create(MXA_RMSC03_RL) +
mxa_step against the reference fixtures (first envs: the reference's own seeds and actions,
one of them ending in the reference's ValueError) and against the C oracle (every env; the
extra envs use other seeds and bigger actions, so the RL orders fill).  Bit-exact for events,
hashes, traces, books and holdings; observations (float64) within the north_star tolerance."""
import numpy as np
import pytest

import pyoracle
from mxabides.gym import VecABIDESEnv
from test_oracle_rl import FIXTURES, OBS_RTOL, load_rl

pytestmark = pytest.mark.gpu
ERR_OBS = 14  # ERR_RP_OBS: get_observation / get_reward on missing or None data (the reference raises)


def test_gpu_rl_matches_reference_and_oracle():
    fx = [load_rl(name) for name, _ in FIXTURES]
    n_ref = len(fx)
    seeds = [seed for _, seed in FIXTURES] + [7, 123, 2 ** 32 - 5]
    n_envs = len(seeds)
    n_steps = 27
    acts = np.zeros((n_steps, n_envs, 3))
    for e, (_, a, _) in enumerate(fx):
        acts[:len(a), e] = a
    rs = np.random.RandomState(11)
    for e in range(n_ref, n_envs):  # up to several thousand shares per step: executions, partial fills
        acts[:, e, 0] = rs.uniform(0, 0.1 * (e - 1), n_steps)
        acts[:, e, 1:] = rs.uniform(0, 1, (n_steps, 2))
    acts[3:6, n_ref, 1:] = 0.0  # zero level shares -> equal split branch
    v = VecABIDESEnv(seeds=seeds, trace_cap=max(len(f[2]) for f in fx))
    oras = [pyoracle.OracleGymEnv(seed=s) for s in seeds]
    alive = np.ones(n_envs, dtype=bool)
    errored = []
    for i in range(n_steps):
        obs, done, valid, err = v.step(acts[i])
        summ = v.summary()
        ev = summ["events"]
        for e in np.nonzero(alive)[0]:
            o_obs, o_done, rc = oras[e].step(acts[i, e])
            assert ev[e] == oras[e].events, (i, e)
            st = fx[e][0]["steps"][i] if e < n_ref else None
            if st is not None:
                assert ev[e] == st["events"], (i, e)
                assert ("error" in st) == (rc != 0), (i, e)
            if rc:  # the reference raises here (get_observation on an empty book side)
                assert err[e] and summ["err"][e] == ERR_OBS, (i, e, rc, summ["err"][e])
                alive[e] = False
                errored.append(int(e))
                continue
            assert not err[e], (i, e, summ["err"][e])
            assert bool(done[e]) == o_done, (i, e)
            assert valid[e]
            np.testing.assert_allclose(obs[e], o_obs, rtol=OBS_RTOL, atol=1e-12, err_msg="step %d env %d" % (i, e))
            if st is not None:
                assert int(done[e]) == st["done"], (i, e)
                np.testing.assert_allclose(obs[e], st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="step %d env %d" % (i, e))
        if (done | ~alive).all():
            break
    assert (done | ~alive).all()
    assert errored == [2]  # the reference's ValueError episode
    s = v.summary()
    for e, (d, _, trace) in enumerate(fx):
        assert "%016x" % s["hash"][e] == d["hash"], e
        assert s["events"][e] == d["events"]
        assert (v.trace(e)[:len(trace)] == trace).all(), e
        assert v.book(e, 0) == d["bids"] and v.book(e, 1) == d["asks"], e
        ag = v.agents(e)
        for ref in d["agents"]:
            assert ag[ref["id"]] == (ref["cash"], ref["shares"], ref["n_open"]), (e, ref["id"])
    for e in range(n_envs):
        assert s["hash"][e] == oras[e].hash, e
        assert v.book(e, 0) == oras[e].book(0) and v.book(e, 1) == oras[e].book(1), e
        assert v.agents(e)[1:] == [tuple(x) for x in oras[e].agents()][1:], e  # 0 = exchange (no holdings)
    assert min(oras[e].rl_state()[0] for e in range(n_ref, n_envs)) < 100000  # RL orders filled


def test_gpu_rl_reset_with_new_seeds_reproduces():
    d, a, _ = load_rl(FIXTURES[0][0])
    v = VecABIDESEnv(seeds=[1, 2])
    v.reset(seeds=[FIXTURES[0][1], FIXTURES[0][1]])
    for i in range(len(a)):
        obs, done, valid, err = v.step(np.stack([a[i], a[i]]))
        assert not err.any()
    s = v.summary()
    assert ["%016x" % x for x in s["hash"]] == [d["hash"]] * 2
