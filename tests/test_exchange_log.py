"""The exchange's own log, ExchangeAgent.log (EXCHANGE_AGENT.bz2), against the reference's.

Fixtures tests/golden/<cfg>_<seed>_exlog.npz (gen_fixtures.py exlog) hold the log of a reference
run: one row per Agent.logEvent call of the exchange (agent/Agent.py:97-110) -- AGENT_TYPE, every
message it logs on receipt with its sender (ExchangeAgent.py:162-167), with log_orders the order of
each LIMIT_ORDER / CANCEL_ORDER and of each ORDER_ACCEPTED / _CANCELLED / _EXECUTED it sends
(:163-165, 477-482), and OrderBook.handleLimitOrder's BEST_BID / BEST_ASK / LAST_TRADE
(util/OrderBook.py:112-141) -- the first 40,000 verbatim and all of them in one digest.  Here the
CPU oracle's record stream (the device's format, include/mxa.h MXA_BL_EV_*) is rebuilt on the host
(mxabides.booklog.exchange_log) and compared; tests/test_gpu_exchange_log.py checks the device
stream against the oracle's.  The order Events' string form (jsons 0.8.8, not importable here) is
parity unpinned; their fields are pinned.
"""
import os

import numpy as np
import pandas as pd
import pytest

import golden_util as gu
import pyoracle
from mxabides import booklog as bl

# log_orders on (sparse_zi_100, rmsc03) and off (sparse_zi_1000, value_noise)
EXLOG_FIXTURES = [("sparse_zi_100", 123456789), ("rmsc03", 123456789), ("sparse_zi_1000", 123456789),
                  ("value_noise", 7)]


def recs(a):
    r = np.zeros(len(a), dtype=bl.REC_DTYPE)
    r["t"], r["price"], r["qty"] = a[:, 0], a[:, 1], a[:, 2]
    return r


def oracle_records(cfg, seed, exlog=True):
    o = pyoracle.OracleEnv(cfg, seed)
    o.set_book_log()
    o.set_exchange_log(exlog)
    o.run()
    return o, recs(o.book_records())


@pytest.mark.parametrize("cfg,seed", EXLOG_FIXTURES)
def test_oracle_exchange_log_equals_reference(cfg, seed):
    n, digest, head, z = gu.exlog_fixture("%s_%d" % (cfg, seed))
    _, r = oracle_records(cfg, seed)
    rows = bl.exchange_log(r, str(z["symbol"]))
    assert len(rows) == n
    got = [gu.exlog_row_tuple(x) for x in rows[:len(head)]]
    bad = [i for i, (a, b) in enumerate(zip(got, head)) if a != b]
    assert not bad, (bad[0], got[bad[0]], head[bad[0]])
    assert gu.exlog_digest(rows) == digest
    assert (any(isinstance(x[2], dict) for x in rows)) == bool(z["log_orders"])


@pytest.mark.parametrize("cfg,seed", [("rmsc03", 123456789), ("value_noise", 7)])
def test_exchange_log_records_leave_the_book_rows_unchanged(cfg, seed):
    """the exchange-log records (and the order records after them) are not book changes: the
    book_log rows replayed from the stream equal the oracle's own rows with the log on or off"""
    o, r = oracle_records(cfg, seed)
    assert np.array_equal(bl.rows_from_records(r), o.book_log())
    _, r0 = oracle_records(cfg, seed, exlog=False)
    assert np.array_equal(bl.rows_from_records(r0), o.book_log())
    assert len(r) > len(r0)
    assert np.array_equal(r[bl.book_mask(r)], r0[bl.book_mask(r0)])
    assert np.array_equal(r[~bl.exlog_mask(r)], r0)


def test_replay_exchange_log_equals_reference_but_duplicate_id_times():
    """config/marketreplay.py's exchange log (log_orders=True): every row's time, type, sender and
    order fields equal the reference's except time_placed where the tape re-uses an order id
    through modifyOrder (the reference keeps each order object's own creation time; the host
    takes the id's latest placement) -- documented in DESIGN.md §1d"""
    from mxabides import tape
    n, digest, head, z = gu.exlog_fixture("marketreplay_IBM_2003-01-14_1")
    tp = tape.Tape.load(os.path.join(gu.GOLDEN, "tape_IBM_2003-01-14.npz"))
    o = pyoracle.OracleReplayRunner(tp, symbol=tp.symbol)
    o.set_book_log()
    o.set_exchange_log()
    o.run()
    rows = bl.exchange_log(recs(o.book_records()), tp.symbol)
    assert len(rows) == n
    got = [gu.exlog_row_tuple(x) for x in rows[:len(head)]]

    def drop_tp(r):
        return r[:5] + ((r[5][0],) + r[5][2:],)
    assert [drop_tp(a) for a in got] == [drop_tp(b) for b in head]
    differ = [i for i, (a, b) in enumerate(zip(got, head)) if a != b]
    assert len(differ) < len(head) // 10
    assert all(head[i][1] in ("ORDER_EXECUTED", "ORDER_CANCELLED", "CANCEL_ORDER", "ORDER_ACCEPTED") for i in differ)


def test_exchange_log_frame_and_file(tmp_path):
    """Agent.kernelTerminating's frame: pd.DataFrame(log).set_index("EventTime") (NaT for the
    AGENT_TYPE row), Event ints, strings and jsons-dumped order dicts; pickled with bz2 as
    Kernel.writeLog does"""
    _, r = oracle_records("sparse_zi_100", 123456789)
    rows = bl.exchange_log(r, "JPM")
    df = bl.exchange_log_frame(rows)
    assert df.index.name == "EventTime" and list(df.columns) == ["EventType", "Event"]
    assert pd.isna(df.index[0]) and df["EventType"].iloc[0] == "AGENT_TYPE" and df["Event"].iloc[0] == "ExchangeAgent"
    assert str(df.index.dtype) == "datetime64[ns]"
    lim = df[df["EventType"] == "LIMIT_ORDER"]["Event"].iloc[0]
    assert list(lim) == ["agent_id", "time_placed", "symbol", "quantity", "is_buy_order", "order_id", "fill_price",
                         "limit_price"]
    assert lim["time_placed"].startswith("2019-06-28T") and lim["time_placed"].endswith("Z") and lim["fill_price"] is None
    ex = df[df["EventType"] == "ORDER_EXECUTED"]["Event"].iloc[0]
    assert isinstance(ex["fill_price"], int)
    p = os.path.join(str(tmp_path), "ExchangeAgent0.bz2")
    df.to_pickle(p, compression="bz2")
    back = pd.read_pickle(p, compression="bz2")
    assert len(back) == len(rows) and back["EventType"].tolist() == df["EventType"].tolist()


def test_jsons_time_placed_format():
    """jsons 0.8.8's datetime form (parity unpinned): seconds, microseconds only when non-zero"""
    d = {"agent_id": 1, "time_placed": 34200 * 10**9, "symbol": "ABM", "quantity": 5, "is_buy_order": True,
         "order_id": 3, "fill_price": None, "limit_price": 100000}
    assert bl.jsons_dump_order(d)["time_placed"] == "2019-06-28T09:30:00Z"
    d["time_placed"] += 1234567
    assert bl.jsons_dump_order(d)["time_placed"] == "2019-06-28T09:30:00.001234Z"


@pytest.mark.parametrize("code", [bl.BL_EV_RX + bl.K_LIMIT, bl.BL_EV_RX + bl.K_CANCEL, bl.BL_EV_NT + 1])
def test_truncated_exchange_log_raises(code):
    """an order row whose order record was cut off (a full log, ERR_BOOK_LOG_FULL) is a clear error"""
    rec = np.zeros(2, dtype=bl.REC_DTYPE)
    rec[0] = (34200 * 10**9, bl.BL_EV_PLACE, 5)
    rec[1] = (34200 * 10**9, code, 3)
    with pytest.raises(ValueError, match="truncated"):
        bl.exchange_log(rec, "JPM")
