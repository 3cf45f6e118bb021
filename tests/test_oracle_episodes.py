"""Consecutive episodes in one process: Order.order_id and
Order._order_ids are class attributes (util/order/Order.py:8-9, 27-42), so an ABIDESEnv.reset
(ABIDESEnv.py:51-57) continues the auto ids of the previous episode and skips every id used
before.  The C oracle's OracleGymEnv.reset (ora_gym_reset) against reference fixtures of
several episodes run in ONE reference process (tests/golden/gen_episodes_fixtures.py)."""
import json
import os

import numpy as np
import pytest

import pyoracle
from mxabides import tape

GOLD = os.path.join(os.path.dirname(__file__), "golden")
OBS_RTOL = 1e-9
EPISODE_FIXTURES = ["eps_rl_5_123456789_2024_7", "eps_mr_IBM_2003-01-14_789_3", "eps_mr_GOOG_2012-06-21_789_4"]


def load_eps(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        d = json.load(f)
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return d, z


def fixture_tape(d):
    return tape.Tape.load(os.path.join(GOLD, "tape_%s_%s.npz" % (d["ticker"], d["date"]))) if "ticker" in d else None


def agents_match(d_ep, ag, mr):
    for k, ref in enumerate(d_ep["agents"]):
        if mr:
            c, s, n = ag[ref["id"]]
            assert c == ref["holdings"]["CASH"] and s == ref["holdings"].get(mr, 0), ref["id"]
            assert n == len(ref["open_orders"]), ref["id"]
        else:
            assert tuple(ag[ref["id"]]) == (ref["cash"], ref["shares"], ref["n_open"]), ref["id"]


@pytest.mark.parametrize("name", EPISODE_FIXTURES)
def test_oracle_consecutive_episodes_match_reference(name):
    if not os.path.exists(os.path.join(GOLD, name + ".json")):
        pytest.skip("fixture not generated")
    d, z = load_eps(name)
    tp = fixture_tape(d)
    e = None
    for k, ep in enumerate(d["episodes"]):
        acts, trace = z["actions_%d" % (k + 1)], z["trace_%d" % (k + 1)]
        if e is None:
            e = pyoracle.OracleGymEnv(tp, trace_cap=len(trace), seed=ep.get("seed"))
        else:
            e.reset(seed=ep.get("seed"), trace_cap=len(trace))
        for i, a in enumerate(acts):
            obs, done, rc = e.step(a)
            st = ep["steps"][i]
            assert e.events == st["events"], (k, i)
            if "error" in st:
                assert rc != 0 and i == len(acts) - 1
                break
            assert rc == 0, e.error
            assert int(done) == st["done"], (k, i)
            if st["obs"]:
                np.testing.assert_allclose(obs, st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="episode %d step %d" % (k, i))
        assert e.events == ep["events"]
        assert "%016x" % e.hash == ep["hash"], k
        assert (e.trace() == trace).all(), k
        assert e.book(0) == ep["bids"] and e.book(1) == ep["asks"], k
        assert e.order_counter == ep["order_id_counter"] + 1, k
        agents_match(ep, e.agents(), d.get("ticker"))
    assert len(d["episodes"]) >= 2 and d["episodes"][1]["order_id_counter_start"] > 0
