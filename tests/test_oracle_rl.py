"""C oracle vs the reference rmsc03 + DummyRL composition (BASELINE.json configs[3]): the 64
rmsc03 agents plus DummyRLExecutionAgent 64 under a GymKernel, stepped with seeded actions.
Per step: observation, done flag, event count; then the trace head, whole-episode hash, final
book and every agent's holdings.  Fixtures produced by tests/golden/gen_rl_fixtures.py from
the reference itself."""
import json
import os

import numpy as np
import pytest

import pyoracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# the third episode ends in the reference's own ValueError (get_observation on an empty book side)
FIXTURES = [("rl_rmsc03_123456789_1", 123456789), ("rl_rmsc03_2024_7", 2024), ("rl_rmsc03_99991_3", 99991)]
OBS_RTOL = 1e-9  # observations are float64 (numpy log/tanh/std vs glibc): north_star tolerance


def load_rl(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        d = json.load(f)
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return d, z["actions"], z["trace"]


@pytest.mark.parametrize("name,seed", FIXTURES)
def test_oracle_rl_episode_matches_reference(name, seed):
    d, actions, trace = load_rl(name)
    e = pyoracle.OracleGymEnv(seed=seed, trace_cap=len(trace))
    for i, a in enumerate(actions):
        obs, done, rc = e.step(a)
        st = d["steps"][i]
        assert e.events == st["events"], i
        if "error" in st:  # the reference raised on this step: the oracle stops with an error too
            assert rc != 0 and i == len(actions) - 1
            break
        assert rc == 0, e.error
        assert int(done) == st["done"], i
        np.testing.assert_allclose(obs, st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="step %d" % i)
    assert done or "error" in d["steps"][-1]
    assert e.events == d["events"]
    assert "%016x" % e.hash == d["hash"]
    assert (e.trace() == trace).all()
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert e.order_counter == d["order_id_counter"] + 1
    ag = e.agents()
    assert len(ag) == 65
    for ref in d["agents"]:
        c, s, n = ag[ref["id"]]
        assert (c, s, n) == (ref["cash"], ref["shares"], ref["n_open"]), ref["id"]
    rl = e.rl_state()
    assert rl[0] == d["rl"]["rem_quantity"] and rl[2] == int(d["rl"]["trade"])
