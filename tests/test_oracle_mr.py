"""C oracle vs the reference ABIDESEnv (Exchange + MarketReplayAgent + DummyRL on a LOBSTER
tape): every step's observation, done flag and event count, the event trace head, the
whole-episode hash, the final book and holdings.  Four episodes: IBM 2003-01-14 (explicit
order ids only) and GOOG 2012-06-21 (3,913 ORDER_ID 0 records, which take auto ids from the
counter DummyRL also uses), plus IBM 2003-01-13 and YHOO 2003-01-14 (round 2).  Fixtures produced by tests/golden/gen_mr_fixtures.py from the
reference itself (LOBSTER CSV path; the reference's processed pickles are never loaded)."""
import json
import os

import numpy as np
import pytest

import pyoracle
from mxabides import tape

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TAPE = os.path.join(GOLD, "tape_IBM_2003-01-14.npz")
LOB = "/root/reference/data/lobster/LOBSTER_SampleFile_%s_1/%s_%s_34200000_57600000_message_1.csv"
EPISODES = [("IBM", "2003-01-14"), ("GOOG", "2012-06-21"), ("IBM", "2003-01-13"), ("YHOO", "2003-01-14")]
OBS_RTOL = 1e-9  # observations are float64 (numpy log/tanh/std vs glibc): north_star tolerance


def _tape(ticker, date):
    return os.path.join(GOLD, "tape_%s_%s.npz" % (ticker, date))


@pytest.fixture(scope="module", params=EPISODES, ids=["%s_%s" % e for e in EPISODES])
def fx(request):
    ticker, date = request.param
    fix = os.path.join(GOLD, "mr_%s_%s_789_1" % (ticker, date))
    with open(fix + ".json") as f:
        d = json.load(f)
    z = np.load(fix + ".npz", allow_pickle=False)
    return d, z["actions"], z["trace"], ticker, date


def test_tape_fixture_well_formed():
    t = tape.Tape.load(TAPE)
    assert len(t) == 38311 and (np.diff(t.t) >= 0).all()


@pytest.mark.parametrize("ticker,date", EPISODES)
def test_tape_loader_matches_committed_tape(ticker, date):
    csv = LOB % (ticker, ticker, date)
    if not os.path.exists(csv):
        pytest.skip("reference data not present (GPU box)")
    a, b = tape.load_lobster(csv, date), tape.Tape.load(_tape(ticker, date))
    for k in ("t", "oid", "price", "size", "buy"):
        assert (getattr(a, k) == getattr(b, k)).all(), k


def test_goog_tape_has_auto_id_records():
    t = tape.Tape.load(_tape("GOOG", "2012-06-21"))
    assert len(t) == 49482 and t.n_auto == 3913


def test_oracle_replay_episode_matches_reference(fx):
    d, actions, trace, ticker, date = fx
    e = pyoracle.OracleGymEnv(tape.Tape.load(_tape(ticker, date)), trace_cap=len(trace))
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
        assert ag[k][1] == ref["holdings"].get(ticker, 0)
        assert ag[k][2] == len(ref["open_orders"])
    rl = e.rl_state()
    assert rl[0] == d["rl"]["rem_quantity"] and rl[2] == int(d["rl"]["trade"])
