"""C oracle vs the reference ABIDESEnv (Exchange + MarketReplayAgent + DummyRL on the IBM
2003-01-14 LOBSTER tape): every step's observation, done flag and event count, the event
trace head, the whole-episode hash, the final book and holdings.  Fixture produced by
tests/golden/gen_mr_fixtures.py from the reference itself."""
import json
import os

import numpy as np
import pytest

import pyoracle
from mxabides import tape

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIX = os.path.join(GOLD, "mr_IBM_2003-01-14_789_1")
TAPE = os.path.join(GOLD, "tape_IBM_2003-01-14.npz")
CSV = "/root/reference/data/lobster/LOBSTER_SampleFile_IBM_1/IBM_2003-01-14_34200000_57600000_message_1.csv"
OBS_RTOL = 1e-9  # observations are float64 (numpy log/tanh/std vs glibc): north_star tolerance


@pytest.fixture(scope="module")
def fx():
    with open(FIX + ".json") as f:
        d = json.load(f)
    z = np.load(FIX + ".npz", allow_pickle=False)
    return d, z["actions"], z["trace"]


def test_tape_fixture_well_formed():
    t = tape.Tape.load(TAPE)
    assert len(t) == 38311 and (np.diff(t.t) >= 0).all()


@pytest.mark.skipif(not os.path.exists(CSV), reason="reference data not present (GPU box)")
def test_tape_loader_matches_committed_tape():
    a, b = tape.load_lobster(CSV, "2003-01-14"), tape.Tape.load(TAPE)
    for k in ("t", "oid", "price", "size", "buy"):
        assert (getattr(a, k) == getattr(b, k)).all(), k


def test_oracle_replay_episode_matches_reference(fx):
    d, actions, trace = fx
    e = pyoracle.OracleGymEnv(tape.Tape.load(TAPE), trace_cap=len(trace))
    for i, a in enumerate(actions):
        obs, done, rc = e.step(a)
        st = d["steps"][i]
        assert rc == 0, e.error
        assert e.events == st["events"], i
        assert int(done) == st["done"], i
        if st["obs"]:
            np.testing.assert_allclose(obs, st["obs"], rtol=OBS_RTOL, atol=1e-12, err_msg="step %d" % i)
    assert done
    assert e.events == d["events"]
    assert "%016x" % e.hash == d["hash"]
    assert (e.trace() == trace).all()
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert e.order_counter == d["order_id_counter"] + 1  # next id (Order.order_id is the last)
    ag = e.agents()
    for k, ref in enumerate(d["agents"], start=1):
        assert ag[k][0] == ref["holdings"]["CASH"]
        assert ag[k][1] == ref["holdings"].get("IBM", 0)
        assert ag[k][2] == len(ref["open_orders"])
    rl = e.rl_state()
    assert rl[0] == d["rl"]["rem_quantity"] and rl[2] == int(d["rl"]["trade"])
