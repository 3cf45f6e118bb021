"""config/marketreplay.py under Kernel.runner (config/marketreplay.py:60-140): the exchange and the
MarketReplayAgent replaying a LOBSTER tape, midnight to 16:01, no oracle and no random draws.
The C oracle's OracleReplayRunner against reference fixtures of that script
(tests/golden/gen_fixtures.py "marketreplay:TICKER:DATE"; the tape is the reference's own LOBSTER
sample message file, parsed by LOBSTEROrdersProcessor, mxabides.tape)."""
import json
import os

import numpy as np
import pytest

import pyoracle
from mxabides import tape

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REPLAY_FIXTURES = [("IBM", "2003-01-14"), ("GOOG", "2012-06-21")]


TWAP_FIXTURES = [(t, d, trade) for t, d in REPLAY_FIXTURES for trade in (False, True)]
# oracle fail() codes of the TWAP agent's crash path (ExecutionAgent.placeOrders KeyError)
TWAP_KEYERROR = -17


def load_replay(ticker, date, prefix="marketreplay"):
    name = "%s_%s_%s_1" % (prefix, ticker, date)
    with open(os.path.join(GOLD, name + ".json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLD, name + "_summary.json")) as f:
        summ = json.load(f)
    trace = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)["trace"]
    tp = tape.Tape.load(os.path.join(GOLD, "tape_%s_%s.npz" % (ticker, date)))
    return d, summ, trace, tp


@pytest.mark.parametrize("ticker,date", REPLAY_FIXTURES)
def test_oracle_replay_runner_matches_reference(ticker, date):
    d, summ, trace, tp = load_replay(ticker, date)
    e = pyoracle.OracleReplayRunner(tp, symbol=ticker, trace_cap=len(trace))
    e.run()
    assert e.error[0] == 0, e.error
    assert (e.trace() == trace).all()
    assert e.events == d["events"]
    assert "%016x" % e.hash == d["hash"]
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert e.last_trade == d["last_trade"]
    # Order.order_id holds the last auto id taken (0 before any, util/order/Order.py:8, 35-42);
    # the oracle's counter the next candidate
    assert max(e.order_counter - 1, 0) == d["order_id_counter"]
    (ag,) = d["agents"]
    assert e.agents()[ag["id"]] == (ag["cash"], ag["shares"], len(ag["open_orders"]))
    e.finish()
    rep = e.report()
    assert [l for l in rep if l.startswith("Final holdings")] == d["final_holdings_lines"]
    assert [l for l in rep if not l.startswith("Final holdings")] == d["mean_lines"]
    got = e.summary_log()
    assert got == summ and all(type(a["Event"]) is type(b["Event"]) for a, b in zip(got, summ))


@pytest.mark.parametrize("ticker,date,trade", TWAP_FIXTURES)
def test_oracle_twap_execution_matches_reference(ticker, date, trade):
    """config/execution/marketreplay/execution_marketreplay.py: the replay plus TWAP_EXECUTION_AGENT.
    Without -e it only learns the market hours and wakes at 10:00; with -e its first placeOrders
    raises KeyError (a 30 s Interval looked up in the 60 s schedule, execution_agent.py:118,
    twap_agent.py:50-55) and the reference run ends there"""
    d, summ, trace, tp = load_replay(ticker, date, "twap_e" if trade else "twap")
    e = pyoracle.OracleReplayRunner(tp, symbol=ticker, trace_cap=len(trace), twap=trade)
    e.run()
    assert (e.trace() == trace).all()
    assert e.events == d["events"] and "%016x" % e.hash == d["hash"]
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert max(e.order_counter - 1, 0) == d["order_id_counter"]
    for ag in d["agents"]:
        assert e.agents()[ag["id"]] == (ag["cash"], ag["shares"], len(ag["open_orders"]))
    if trade:
        assert d["stop_error"].startswith("KeyError: Interval(") and e.error[0] == TWAP_KEYERROR
        assert d["final_time"] == 10 * 3600 * 10 ** 9
        # kernelStarting's rows only: the crash skips kernelStopping
        assert summ == [{"AgentID": a, "AgentStrategy": t, "EventType": "STARTING_CASH", "Event": 0}
                        for a, t in ((1, "MarketReplayAgent"), (2, "ExecutionAgent"))]
        return
    assert e.error[0] == 0 and d["stop_error"] is None
    e.finish()
    rep = e.report()
    assert [l for l in rep if l.startswith("Final holdings")] == d["final_holdings_lines"]
    assert [l for l in rep if not l.startswith("Final holdings")] == d["mean_lines"]
    got = e.summary_log()
    assert got == summ and all(type(a["Event"]) is type(b["Event"]) for a, b in zip(got, summ))
