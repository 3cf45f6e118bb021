"""ABIDESEnv / market replay on the GPU (libmxa mxa_create_replay + mxa_step) against the
reference fixture (env 0: the reference's own actions) and against the C oracle (other envs:
other action streams).  Bit-exact for events, hashes, traces, books and holdings; observations
(float64) within the north_star tolerance."""
import json
import os

import numpy as np
import pytest

import pyoracle
from mxabides import tape
from mxabides.gym import VecABIDESEnv, ABIDESEnv

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TAPE = os.path.join(GOLD, "tape_IBM_2003-01-14.npz")
# (ticker, date): IBM 2003-01-14 has explicit ids only; GOOG 2012-06-21 has 3,913 ORDER_ID 0
# records (hidden executions) that take auto ids interleaved with DummyRL's
EPISODES = [("IBM", "2003-01-14"), ("GOOG", "2012-06-21"), ("IBM", "2003-01-13"), ("YHOO", "2003-01-14")]
OBS_RTOL = 1e-9


def _actions(n_envs, fixture_actions):
    acts = np.zeros((len(fixture_actions), n_envs, 3))
    acts[:, 0] = fixture_actions
    rs = np.random.RandomState(7)
    for e in range(1, n_envs):  # bigger orders than the fixture: they fill, exercising executions
        acts[:, e, 0] = rs.uniform(0, 0.05 * e, len(fixture_actions))
        acts[:, e, 1:] = rs.uniform(0, 1, (len(fixture_actions), 2))
    acts[5:9, 1, 1:] = 0.0  # zero level shares -> equal split branch
    return acts


@pytest.mark.parametrize("ticker,date", EPISODES)
def test_gpu_replay_matches_reference_and_oracle(ticker, date):
    fix = os.path.join(GOLD, "mr_%s_%s_789_1" % (ticker, date))
    with open(fix + ".json") as f:
        d = json.load(f)
    z = np.load(fix + ".npz", allow_pickle=False)
    tp = tape.Tape.load(os.path.join(GOLD, "tape_%s_%s.npz" % (ticker, date)))
    n_envs = 4
    acts = _actions(n_envs, z["actions"])
    v = VecABIDESEnv(tp, n_envs, trace_cap=len(z["trace"]))
    oras = [pyoracle.OracleGymEnv(tp) for _ in range(n_envs)]
    for i in range(len(acts)):
        obs, done, valid, err = v.step(acts[i])
        assert not err.any(), (i, v.summary()["err"])
        ev = v.summary()["events"]
        st = d["steps"][i]
        assert ev[0] == st["events"], i
        assert int(done[0]) == st["done"], i
        if st["obs"]:
            assert valid[0]
            np.testing.assert_allclose(obs[0], st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="step %d" % i)
        for e in range(1, n_envs):
            o_obs, o_done, rc = oras[e].step(acts[i, e])
            assert rc == 0
            assert ev[e] == oras[e].events, (i, e)
            assert bool(done[e]) == o_done, (i, e)
            if o_obs is not None:
                np.testing.assert_allclose(obs[e], o_obs, rtol=OBS_RTOL, atol=1e-12, err_msg="step %d env %d" % (i, e))
        if done.all():
            break
    s = v.summary()
    assert "%016x" % s["hash"][0] == d["hash"]
    assert s["events"][0] == d["events"]
    assert (v.trace(0) == z["trace"]).all()
    assert v.book(0, 0) == d["bids"] and v.book(0, 1) == d["asks"]
    ag = v.agents(0)
    for k, ref in enumerate(d["agents"], start=1):
        assert ag[k][0] == ref["holdings"]["CASH"] and ag[k][1] == ref["holdings"].get(ticker, 0)
        assert ag[k][2] == len(ref["open_orders"])
    for e in range(1, n_envs):
        assert s["hash"][e] == oras[e].hash, e
        assert v.book(e, 0) == oras[e].book(0) and v.book(e, 1) == oras[e].book(1), e
        assert v.agents(e) == [tuple(x) for x in oras[e].agents()], e


def test_gpu_abidesenv_surface():
    env = ABIDESEnv("IBM", "2003-01-14", seed=789, tape=tape.Tape.load(TAPE))
    env.reset()
    obs, rew, done, info = env.step([0.0, 0.5, 0.5])
    assert rew is None and info is None and done == 0 and len(obs) == 9
    assert obs[0] == 760.0 and obs[1] == 100000.0


def test_gpu_replay_truncated_goog_tape_equals_oracle():
    """a short tape (first 3,000 GOOG records, 217 of them ORDER_ID 0): the replay agent runs
    out of records early and DummyRL keeps trading against what is left"""
    full = tape.Tape.load(os.path.join(GOLD, "tape_GOOG_2012-06-21.npz"))
    k = 3000
    tp = tape.Tape(full.t[:k], full.oid[:k], full.price[:k], full.size[:k], full.buy[:k])
    n_envs = 6
    rs = np.random.RandomState(11)
    acts = np.stack([rs.uniform(0, 0.03, (761, n_envs)), rs.uniform(0, 1, (761, n_envs)),
                     rs.uniform(0, 1, (761, n_envs))], 2)
    v = VecABIDESEnv(tp, n_envs)
    oras = [pyoracle.OracleGymEnv(tp) for _ in range(n_envs)]
    done_o = [False] * n_envs
    for i in range(761):
        obs, done, valid, err = v.step(acts[i])
        for e in range(n_envs):
            if done_o[e]:
                continue
            o_obs, o_done, rc = oras[e].step(acts[i, e])
            assert bool(err[e]) == (rc != 0), (i, e)
            done_o[e] = o_done or rc != 0
            if o_obs is not None and not err[e]:
                np.testing.assert_allclose(obs[e], o_obs, rtol=OBS_RTOL, atol=1e-12, err_msg="step %d env %d" % (i, e))
        if all(done_o):
            break
    s = v.summary()
    for e in range(n_envs):
        assert s["events"][e] == oras[e].events and s["hash"][e] == oras[e].hash, e
        assert v.book(e, 0) == oras[e].book(0) and v.book(e, 1) == oras[e].book(1), e
