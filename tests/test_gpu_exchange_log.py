"""GPU parity of the exchange's own log (include/mxa.h mxa_set_exchange_log): the device's
book-update stream with the exchange log on is record for record the oracle's, and the host rebuild
of it (mxabides.booklog.exchange_log) is the reference's ExchangeAgent.log
(tests/golden/*_exlog.npz, gen_fixtures.py exlog) -- the EXCHANGE_AGENT.bz2 of Agent.kernelTerminating
(agent/Agent.py:86-95).  Logging leaves the simulation (pop count, parity hash) unchanged."""
import os

import numpy as np
import pandas as pd
import pytest

import golden_util as gu
import pyoracle
from mxabides import booklog as bl

pytestmark = pytest.mark.gpu
CAP = 1 << 20


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def oracle_recs(cfg, seed):
    o = pyoracle.OracleEnv(cfg, seed)
    o.set_book_log()
    o.set_exchange_log()
    o.run()
    a = o.book_records()
    r = np.zeros(len(a), dtype=bl.REC_DTYPE)
    r["t"], r["price"], r["qty"] = a[:, 0], a[:, 1], a[:, 2]
    return o, r


# log_orders on: rmsc03, sparse_zi_100, rmsc02, random_fund_value, rmsc03_sbmm; off: value_noise,
# sparse_zi_1000, rmsc01, obi_rmsc02 (seed 30: its OBI agents trade) -- ADVICE r05
@pytest.mark.parametrize("cfg,seeds", [("rmsc03", [123456789, 7, 1008]), ("sparse_zi_100", [123456789, 5]),
                                       ("value_noise", [7, 123456789]), ("sparse_zi_1000", [123456789]),
                                       ("rmsc02", [7]), ("rmsc01", [7]), ("obi_rmsc02", [30]),
                                       ("random_fund_value", [7]), ("rmsc03_sbmm", [7])])
def test_gpu_exchange_log_records_equal_oracle(mx, cfg, seeds):
    m = mx.VecMarket(cfg, seeds, book_log=CAP * (8 if cfg == "rmsc01" else 1), exchange_log=True)
    m.run()
    s = m.summary()
    for i, sd in enumerate(seeds):
        o, r = oracle_recs(cfg, sd)
        assert s["status"][i] == 1, (s["status"][i], s["err"][i])
        assert s["events"][i] == o.events and s["hash"][i] == o.hash
        d = m.book_log_records(i)
        assert len(d) == len(r)
        assert np.array_equal(d, r)


@pytest.mark.parametrize("cfg,seed", [("sparse_zi_100", 123456789), ("rmsc03", 123456789),
                                      ("sparse_zi_1000", 123456789), ("value_noise", 7)])
def test_gpu_exchange_log_equals_reference_fixture(mx, cfg, seed, tmp_path):
    n, digest, head, z = gu.exlog_fixture("%s_%d" % (cfg, seed))
    m = mx.VecMarket(cfg, [seed], book_log=CAP, exchange_log=True)
    m.run()
    rows = m.exchange_log(0)
    assert len(rows) == n and gu.exlog_digest(rows) == digest
    assert [gu.exlog_row_tuple(x) for x in rows[:len(head)]] == head
    paths = m.write_logs(0, str(tmp_path))
    name = "%s.bz2" % str(z["name"]).replace(" ", "")
    assert name in [os.path.basename(p) for p in paths]
    back = pd.read_pickle(os.path.join(str(tmp_path), name), compression="bz2")
    assert len(back) == n and back.index.name == "EventTime" and back["EventType"].iloc[0] == "AGENT_TYPE"


def test_gpu_exchange_log_chunked_launches_and_reset(mx):
    """records survive launch boundaries, and the switch survives mxa_reset"""
    seeds = [123456789, 7]
    m = mx.VecMarket("rmsc03", seeds, book_log=CAP, exchange_log=True)
    m.run(chunk=2999)
    for i, sd in enumerate(seeds):
        assert np.array_equal(m.book_log_records(i), oracle_recs("rmsc03", sd)[1])
    m.reset()
    m.run()
    for i, sd in enumerate(seeds):
        assert np.array_equal(m.book_log_records(i), oracle_recs("rmsc03", sd)[1])


def test_gpu_exchange_log_off_keeps_the_book_log(mx):
    """without the switch the stream is the book-update log alone; with it the book rows are
    the same"""
    a = mx.VecMarket("rmsc03", [123456789], book_log=CAP)
    a.run()
    b = mx.VecMarket("rmsc03", [123456789], book_log=CAP, exchange_log=True)
    b.run()
    ra, rb = a.book_log_records(0), b.book_log_records(0)
    assert len(rb) > 4 * len(ra)
    assert np.array_equal(ra, rb[~bl.exlog_mask(rb)])  # the book and f_log records, unchanged
    assert np.array_equal(a.book_log_rows(0), b.book_log_rows(0))
    with pytest.raises(ValueError):
        mx.VecMarket("rmsc03", [1], exchange_log=True)


def test_gpu_replay_exchange_log_equals_oracle(mx):
    """config/marketreplay.py (log_orders=True) on the IBM tape: the device stream equals the
    oracle's record for record"""
    from mxabides import tape
    tp = tape.Tape.load(os.path.join(gu.GOLDEN, "tape_IBM_2003-01-14.npz"))
    m = mx.VecMarket("marketreplay_runner", [1, 2], tape=tp, book_log=CAP, exchange_log=True)
    m.run()
    o = pyoracle.OracleReplayRunner(tp, symbol=tp.symbol)
    o.set_book_log()
    o.set_exchange_log()
    o.run()
    a = o.book_records()
    for i in range(2):
        d = m.book_log_records(i)
        assert len(d) == len(a)
        assert np.array_equal(d["t"], a[:, 0]) and np.array_equal(d["price"], a[:, 1]) and np.array_equal(d["qty"], a[:, 2])
    n, digest, head, z = gu.exlog_fixture("marketreplay_IBM_2003-01-14_1")
    assert len(m.exchange_log(0)) == n
