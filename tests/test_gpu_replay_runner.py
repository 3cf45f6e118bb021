"""config/marketreplay.py under Kernel.runner on the device (VecMarket("marketreplay_runner", tape=)):
libmxa's replay kernels against the reference fixtures (tests/golden/marketreplay_*) and the C
oracle's OracleReplayRunner.  Bit-exact: trace records, event count, parity hash, both books
(every resting order, FIFO), the agent's holdings and open orders, report and summary log."""
import numpy as np
import pytest

import pyoracle
from test_oracle_replay_runner import REPLAY_FIXTURES, TWAP_FIXTURES, load_replay

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


@pytest.mark.parametrize("ticker,date", REPLAY_FIXTURES)
def test_gpu_replay_runner_matches_reference(mx, ticker, date):
    d, summ, trace, tp = load_replay(ticker, date)
    m = mx.VecMarket("marketreplay_runner", [0], tape=tp, symbol=ticker, trace_cap=len(trace))
    m.run()
    s = m.summary()
    assert s["status"][0] == 1, "env error %d" % s["err"][0]
    assert (m.trace(0) == trace).all()
    assert int(s["events"][0]) == d["events"]
    assert "%016x" % int(s["hash"][0]) == d["hash"]
    assert m.book(0, 0) == d["bids"] and m.book(0, 1) == d["asks"]
    (ag,) = d["agents"]
    a = m.agents(0)[ag["id"]]
    assert (a["cash"], a["shares"], a["n_open"]) == (ag["cash"], ag["shares"], len(ag["open_orders"]))
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"] and means == d["mean_lines"]
    got = m.summary_log(0)
    assert got == summ and all(type(x["Event"]) is type(y["Event"]) for x, y in zip(got, summ))


@pytest.mark.parametrize("ticker,date", REPLAY_FIXTURES)
def test_gpu_replay_runner_batch_and_chunks_equal_oracle(mx, ticker, date):
    """a batch of identical replays (nothing draws) run in many short launches: every env equals the
    oracle's single run, so save/restore of the replay state is exact"""
    _, _, _, tp = load_replay(ticker, date)
    o = pyoracle.OracleReplayRunner(tp, symbol=ticker)
    o.run()
    m = mx.VecMarket("marketreplay_runner", np.zeros(130, dtype=np.int64), tape=tp, symbol=ticker)
    m.run(chunk=9973)
    s = m.summary()
    assert (s["status"] == 1).all()
    assert (s["events"] == o.events).all() and (s["hash"] == o.hash).all()
    assert m.book(129, 0) == o.book(0) and m.book(129, 1) == o.book(1)
    m.reset()
    m.run()
    assert (m.summary()["hash"] == o.hash).all()


def test_gpu_replay_runner_rejects_missing_tape(mx):
    with pytest.raises(ValueError):
        mx.VecMarket("marketreplay_runner", [0])


@pytest.mark.parametrize("ticker,date,trade", TWAP_FIXTURES)
def test_gpu_twap_execution_matches_reference(mx, ticker, date, trade):
    """config/execution/marketreplay/execution_marketreplay.py on the device: the replay plus
    TWAP_EXECUTION_AGENT, passive (no -e) or trading (-e: the reference's KeyError at 10:00 is
    env error 25 after the same pops)"""
    d, summ, trace, tp = load_replay(ticker, date, "twap_e" if trade else "twap")
    cfg = "marketreplay_twap_e" if trade else "marketreplay_twap"
    m = mx.VecMarket(cfg, [0, 0], tape=tp, symbol=ticker, trace_cap=len(trace))
    m.run(chunk=50000)
    s = m.summary()
    assert (s["events"] == d["events"]).all()
    assert ("%016x" % int(s["hash"][0])) == d["hash"] and s["hash"][0] == s["hash"][1]
    assert (m.trace(1) == trace).all()
    assert m.book(1, 0) == d["bids"] and m.book(1, 1) == d["asks"]
    for ag in d["agents"]:
        a = m.agents(1)[ag["id"]]
        assert (a["cash"], a["shares"], a["n_open"]) == (ag["cash"], ag["shares"], len(ag["open_orders"]))
    if trade:
        assert (s["status"] == 2).all() and (s["err"] == 25).all()
        assert (s["current_time"] == d["final_time"]).all()
        return
    assert (s["status"] == 1).all()
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"] and means == d["mean_lines"]
    got = m.summary_log(0)
    assert got == summ and all(type(x["Event"]) is type(y["Event"]) for x, y in zip(got, summ))
