"""The exchange's order-book outputs (mxabides.booklog) against the reference's own.

Fixtures tests/golden/<cfg>_<seed>_booklog.npz (gen_fixtures.py booklog) hold, from the reference
run with book_freq 0: every OrderBook.book_log row (OrderBook.py:151-168), the exchange's
BEST_BID / BEST_ASK / LAST_TRADE log events (OrderBook.py:114-141), and the DataFrames
ExchangeAgent.logOrderBookSnapshots hands to writeLog (ExchangeAgent.py:389-469) for the first
300 rows, narrow and wide_book.  The CPU oracle's rows and the host formatting are checked here;
tests/test_gpu_booklog.py checks the device log against the oracle.
"""
import os

import numpy as np
import pandas as pd
import pytest

import pyoracle
from mxabides import booklog as bl

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BOOKLOG_FIXTURES = [("value_noise", 7), ("rmsc03", 123456789)]
MIDNIGHT = pd.Timestamp(bl.SESSION_DATE).value
EV_TYPES = ("BEST_BID", "BEST_ASK", "LAST_TRADE")


def fixture(cfg, seed):
    path = os.path.join(GOLDEN, "%s_%d_booklog.npz" % (cfg, seed))
    if not os.path.exists(path):
        pytest.skip("no fixture %s" % path)
    return np.load(path)


_oracle_rows = {}


def oracle_rows(cfg, seed):
    if (cfg, seed) not in _oracle_rows:
        o = pyoracle.OracleEnv(cfg, seed)
        o.set_book_log()
        o.run()
        _oracle_rows[(cfg, seed)] = o.book_log()
    return _oracle_rows[(cfg, seed)]


def head_rows(flat, n):
    i = 0
    for _ in range(n):
        i += 4 + 2 * int(flat[i + 1])
    return flat[:i]


@pytest.mark.parametrize("cfg,seed", BOOKLOG_FIXTURES)
def test_oracle_book_log_rows_equal_reference(cfg, seed):
    z = fixture(cfg, seed)
    rows = bl.strip_executions(oracle_rows(cfg, seed))
    assert len(rows) == len(z["rows"])
    assert np.array_equal(rows, z["rows"])


@pytest.mark.parametrize("cfg,seed", BOOKLOG_FIXTURES)
def test_exchange_events_equal_reference(cfg, seed):
    z = fixture(cfg, seed)
    sym = "ABM" if cfg == "rmsc03" else "JPM"
    ev = bl.exchange_events(oracle_rows(cfg, seed), sym)
    ref = list(zip(z["ev_t"].tolist(), [EV_TYPES[k] for k in z["ev_type"].tolist()], z["ev_text"].tolist()))
    assert len(ev) == len(ref)
    assert ev == ref
    df = bl.exchange_events_frame(oracle_rows(cfg, seed)[:4000], sym)
    assert df.index.name == "EventTime" and list(df.columns) == ["EventType", "Event"]


@pytest.mark.parametrize("cfg,seed", BOOKLOG_FIXTURES)
def test_orderbook_full_frames_equal_reference(cfg, seed):
    z = fixture(cfg, seed)
    sub = head_rows(oracle_rows(cfg, seed), int(z["full_rows"]))
    d = bl.orderbook_full(sub)
    assert list(d.index.names) == ["time", "quote"] and list(d.columns) == ["Volume"]
    assert str(d["Volume"].dtype) == str(z["full_dtype"])
    assert np.array_equal(d.index.get_level_values(0).asi8 - MIDNIGHT, z["full_time"])
    assert np.array_equal(np.asarray(d.index.get_level_values(1), dtype=np.int64), z["full_quote"])
    assert np.array_equal(d["Volume"].to_numpy(), z["full_volume"], equal_nan=True)
    w = bl.orderbook_full(sub, wide_book=True)
    assert np.array_equal(w.index.asi8 - MIDNIGHT, z["wide_time"])
    assert np.array_equal(np.asarray(w.columns, dtype=np.int64), z["wide_cols"])
    assert [str(x) for x in w.dtypes] == z["wide_dtypes"].tolist()
    assert np.array_equal(w.to_numpy(dtype=np.float64), z["wide_values"], equal_nan=True)


@pytest.mark.parametrize("cfg,seed", [("value_noise", 7), ("rmsc03", 123456789), ("sparse_zi_100", 123456789)])
def test_records_replay_into_oracle_rows(cfg, seed):
    """the host replay of the record stream (limit orders and cancellations only) rebuilds
    every book_log row, executions included"""
    o = pyoracle.OracleEnv(cfg, seed)
    o.set_book_log()
    o.run()
    r = o.book_records()
    rec = np.zeros(len(r), dtype=bl.REC_DTYPE)
    rec["t"], rec["price"], rec["qty"] = r[:, 0], r[:, 1], r[:, 2]
    assert np.array_equal(bl.rows_from_records(rec), o.book_log())


@pytest.mark.parametrize("cfg,seed", BOOKLOG_FIXTURES)
def test_oracle_fundamental_log_equals_reference(cfg, seed):
    """SparseMeanRevertingOracle.f_log after the run and its kernelStopping pass, and the frame
    written as fundamental_<sym>.bz2"""
    z = fixture(cfg, seed)
    o = pyoracle.OracleEnv(cfg, seed)
    o.set_book_log()
    o.run()
    o.finish()
    r = o.book_records()
    rec = np.zeros(len(r), dtype=bl.REC_DTYPE)
    rec["t"], rec["price"], rec["qty"] = r[:, 0], r[:, 1], r[:, 2]
    t, v = bl.fundamental_log(rec)
    assert np.array_equal(t, z["fund_time"]) and np.array_equal(v, z["fund_value"])
    df = bl.fundamental_frame(rec)
    assert df.index.name == "FundamentalTime" and list(df.columns) == ["FundamentalValue"]
    assert str(df["FundamentalValue"].dtype) == str(z["fund_dtype"])
    assert np.array_equal(df.index.asi8 - MIDNIGHT, z["fund_time"])
    # the book rows ignore the f_log records
    assert np.array_equal(bl.rows_from_records(rec), o.book_log())


def test_records_replay_edge_cases():
    """the host replay of limit/cancel records: crossing sweeps, partial fills, resting
    remainders, cancellations (no row of their own), python rounding of the average price"""
    rec = np.array([(5, 100, -3),      # sell 3 @ 100 rests (the first row: one ask level)
                    (6, 99, 4),        # buy 4 @ 99 rests
                    (7, 101, -2),      # another ask level
                    (8, 101, 4),       # buy 4 @ 101: 3 @ 100 + 1 @ 101, nothing rests
                    (9, -99, 4),       # cancel the bid level
                    (10, 102, 5),      # buy 5 @ 102: 1 @ 101, 4 rest at 102
                    (11, 1, -2),       # sell 2 @ 1: fills 2 @ 102
                    (12, 103, -1), (13, 103, -2), (14, -103, -1)], dtype=bl.REC_DTYPE)
    rows = bl.rows_from_records(rec).tolist()
    assert rows == [5, 1, 0, 0, 100, 3,
                    6, 2, 0, 0, 99, -4, 100, 3,
                    7, 3, 0, 0, 99, -4, 100, 3, 101, 2,
                    8, 2, 4, 100, 99, -4, 101, 1,     # int(round(401 / 4)) = 100
                    10, 1, 1, 101, 102, -4,
                    11, 1, 2, 102, 102, -2,
                    12, 2, 0, 0, 102, -2, 103, 1,
                    13, 2, 0, 0, 102, -2, 103, 3]
    ev = bl.exchange_events(np.array(rows), "JPM")
    assert ev[:3] == [(5, "BEST_ASK", "JPM,100,3"), (6, "BEST_BID", "JPM,99,4"), (6, "BEST_ASK", "JPM,100,3")]
    assert (8, "LAST_TRADE", "4,$100.0000") in ev and (10, "LAST_TRADE", "1,$101.0000") in ev
    # round half to even, as python's round: 2 @ 100 + 2 @ 101 -> 100.5 -> 100
    r2 = bl.rows_from_records(np.array([(1, 100, -2), (2, 101, -2), (3, 101, 4)], dtype=bl.REC_DTYPE))
    assert r2.tolist()[-4:] == [3, 0, 4, 100]
    assert len(bl.rows_from_records(np.zeros(0, dtype=bl.REC_DTYPE))) == 0


def test_duplicate_timestamps_keep_last_row(tmp_path):
    """logOrderBookSnapshots keeps the last row of a timestamp (ExchangeAgent.py:415), and the
    pickle round-trips as Kernel.writeLog writes it"""
    rows = np.array([5, 1, 0, 0, 100, -3,
                     5, 2, 0, 0, 100, -3, 102, 2,
                     6, 1, 0, 0, 102, 2], dtype=np.int64)
    d = bl.orderbook_full(rows)
    assert d.index.get_level_values(0).nunique() == 2
    assert d.loc[(pd.Timestamp(bl.SESSION_DATE) + pd.Timedelta(5, "ns"), 102), "Volume"] == 2
    assert d.loc[(pd.Timestamp(bl.SESSION_DATE) + pd.Timedelta(6, "ns"), 100), "Volume"] == 0
    p = tmp_path / "ORDERBOOK_JPM_FULL.bz2"
    d.to_pickle(p, compression="bz2")
    back = pd.read_pickle(p, compression="bz2")
    assert back.equals(d)


# ---- config/marketreplay.py (book_freq 0: ORDERBOOK_<sym>_FULL of the replay's book) and the
# ExternalFileOracle's f_log (fundamental_JPM of hist_fund_*), pinned by reference runs
# (gen_fixtures.py booklog marketreplay / flog): every book_log row and the exchange's events as
# digests, the first rows verbatim
REPLAY_TAPES = ["IBM_2003-01-14", "GOOG_2012-06-21"]


def _recs(rows3):
    r = np.zeros(len(rows3), dtype=bl.REC_DTYPE)
    r["t"], r["price"], r["qty"] = rows3[:, 0], rows3[:, 1], rows3[:, 2]
    return r


@pytest.mark.parametrize("tname", REPLAY_TAPES)
def test_oracle_replay_book_log_equals_reference(tname):
    """the oracle's replay rows equal the reference's (all rows by digest, the first ones word by
    word); its book-update records (limit, cancel and the modifyOrder head-replace as a volume
    change) replay on the host to exactly those rows"""
    import golden_util as gu
    from mxabides import tape
    z = np.load(os.path.join(GOLDEN, "marketreplay_%s_1_booklog.npz" % tname))
    tp = tape.Tape.load(os.path.join(GOLDEN, "tape_%s.npz" % tname))
    o = pyoracle.OracleReplayRunner(tp, symbol=tp.symbol)
    o.set_book_log()
    o.run()
    flat = o.book_log()
    assert np.array_equal(np.asarray(gu.book_row_digests(flat), dtype=np.uint64), z["row_digests"])
    head = bl.strip_executions(flat)[:len(z["rows"])]
    assert np.array_equal(head, z["rows"])
    ev = bl.exchange_events(flat, tp.symbol)
    assert len(ev) == int(z["n_events"]) and gu.event_digest(ev) == int(z["ev_digest"])
    rec = _recs(o.book_records())
    assert (rec["price"] < 0).sum() > 1000  # the replay's modifies / cancels are in the stream
    assert np.array_equal(bl.rows_from_records(rec), flat)


@pytest.mark.parametrize("cfg", ["hist_fund_value", "hist_fund_diverse"])
def test_oracle_external_file_oracle_f_log_equals_reference(cfg):
    """ExternalFileOracle.f_log (ExternalFileOracle.py:19, 97) after kernelStopping: one entry per
    getPriceAtTime inside the series, as (low, high) word record pairs of the interpolated double"""
    z = np.load(os.path.join(GOLDEN, "%s_7_flog.npz" % cfg))
    o = pyoracle.OracleEnv(cfg, 7)
    o.set_book_log()
    o.run()
    o.finish()
    t, v = bl.fundamental_log(_recs(o.book_records()), external=True)
    assert np.array_equal(t, z["fund_time"]) and np.array_equal(v, z["fund_value"])
    f = bl.fundamental_frame(_recs(o.book_records()), external=True)
    assert str(f["FundamentalValue"].dtype) == str(z["fund_dtype"]) and len(f) == len(t)
