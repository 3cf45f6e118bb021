"""GPU parity of the book-update log (include/mxa.h mxa_set_book_log): the device's records,
replayed on the host (mxabides.booklog), give exactly the oracle's OrderBook.book_log rows and
the reference's own rows (tests/golden/*_booklog.npz); logging leaves the simulation itself
(pop count, parity hash) unchanged although it turns the exchange's event runs off."""
import os

import numpy as np
import pytest

import pyoracle
from mxabides import booklog as bl

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAP = 1 << 18


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def oracle(cfg, seed):
    o = pyoracle.OracleEnv(cfg, seed)
    o.set_book_log()
    o.run()
    return o


@pytest.mark.parametrize("cfg,seeds", [("rmsc03", [123456789, 7, 1008]), ("value_noise", [7, 123456789]),
                                       ("sparse_zi_100", [123456789]), ("rmsc01", [7])])
def test_gpu_book_log_equals_oracle(mx, cfg, seeds):
    m = mx.VecMarket(cfg, seeds, book_log=CAP * (16 if cfg == "rmsc01" else 1))
    m.run()
    s = m.summary()
    for i, sd in enumerate(seeds):
        o = oracle(cfg, sd)
        assert s["status"][i] == 1, (s["status"][i], s["err"][i])
        assert s["events"][i] == o.events and s["hash"][i] == o.hash
        rows = m.book_log_rows(i)
        ref = o.book_log()
        assert len(rows) == len(ref)
        assert np.array_equal(rows, ref)


@pytest.mark.parametrize("cfg,seed", [("rmsc03", 123456789), ("value_noise", 7)])
def test_gpu_book_log_equals_reference_fixture(mx, cfg, seed, tmp_path):
    z = np.load(os.path.join(GOLDEN, "%s_%d_booklog.npz" % (cfg, seed)))
    m = mx.VecMarket(cfg, [seed], book_log=CAP)
    m.run()
    rows = m.book_log_rows(0)
    assert np.array_equal(bl.strip_executions(rows), z["rows"])
    ev = m.exchange_events(0)
    assert len(ev) == len(z["ev_t"]) and ev["Event"].tolist() == z["ev_text"].tolist()
    import pandas as pd
    path = m.write_orderbook_log(0, str(tmp_path))
    assert os.path.basename(path) == "ORDERBOOK_%s_FULL.bz2" % ("ABM" if cfg == "rmsc03" else "JPM")
    back = pd.read_pickle(path, compression="bz2")
    assert list(back.columns) == ["Volume"] and back.index.names == ["time", "quote"]
    times = {t for t, _, _, _, _ in bl.iter_rows(rows)}
    assert back.index.get_level_values(0).nunique() == len(times)


def test_gpu_book_log_chunked_launches(mx):
    """records and their count survive launch boundaries"""
    m = mx.VecMarket("rmsc03", [123456789, 7], book_log=CAP)
    m.run(chunk=3001)
    for i, sd in enumerate([123456789, 7]):
        assert np.array_equal(m.book_log_rows(i), oracle("rmsc03", sd).book_log())


def test_gpu_book_log_overflow_is_an_env_error(mx):
    m = mx.VecMarket("rmsc03", [123456789, 7], book_log=1000)
    m.run()
    s = m.summary()
    assert (s["status"] == 2).all() and (s["err"] == 20).all()
    assert len(m.book_log_records(0, partial=True)) == 1000
    with pytest.raises(mx.MxaError, match="overflow"):
        m.book_log_records(0)


def test_gpu_book_log_off_after_reset(mx):
    """set_book_log(0) frees the log; the next episode runs with the event runs again"""
    m = mx.VecMarket("value_noise", [7], book_log=CAP)
    m.run()
    m.set_book_log(0)
    m.reset()
    m.run()
    o = oracle("value_noise", 7)
    s = m.summary()
    assert s["events"][0] == o.events and s["hash"][0] == o.hash
    with pytest.raises(ValueError):
        m.book_log_records(0)


@pytest.mark.parametrize("cfg,seed", [("rmsc03", 123456789), ("value_noise", 7)])
def test_gpu_fundamental_log_equals_reference(mx, cfg, seed, tmp_path):
    """SparseMeanRevertingOracle.f_log from the device stream (run + kernelStopping pass) equals
    the reference's; write_logs writes the run directory's frames"""
    import pandas as pd
    z = np.load(os.path.join(GOLDEN, "%s_%d_booklog.npz" % (cfg, seed)))
    m = mx.VecMarket(cfg, [seed], book_log=CAP, book_freq=0)  # the fixtures' -b 0 (rmsc03's own default)
    m.run()
    df = m.fundamental_log(0)
    assert np.array_equal(df.index.asi8 - pd.Timestamp(bl.SESSION_DATE).value, z["fund_time"])
    assert np.array_equal(df["FundamentalValue"].to_numpy(), z["fund_value"])
    m.finalize()  # idempotent: a second pass rewrites the same records
    assert m.fundamental_log(0).equals(df)
    paths = m.write_logs(0, str(tmp_path))
    sym = "ABM" if cfg == "rmsc03" else "JPM"
    assert sorted(os.path.basename(p) for p in paths) == sorted(
        ["summary_log.bz2", "fundamental_%s.bz2" % sym, "ORDERBOOK_%s_FULL.bz2" % sym])
    assert pd.read_pickle(os.path.join(str(tmp_path), "fundamental_%s.bz2" % sym), compression="bz2").equals(df)


def test_gpu_fundamental_records_equal_oracle(mx):
    seeds = [123456789, 7]
    m = mx.VecMarket("rmsc03", seeds, book_log=CAP)
    m.run()
    m.finalize()
    for i, sd in enumerate(seeds):
        o = oracle("rmsc03", sd)
        o.finish()
        r = m.book_log_records(i)
        ref = o.book_records()
        assert len(r) == len(ref)
        assert np.array_equal(r["t"], ref[:, 0]) and np.array_equal(r["price"], ref[:, 1])
        assert np.array_equal(r["qty"], ref[:, 2])


def test_gpu_write_logs_follows_the_config_book_freq(mx, tmp_path):
    """ExchangeAgent.kernelTerminating (ExchangeAgent.py:106-126): with book_freq None
    (random_fund_value, value_noise's default) no order-book file; the ticker names the files;
    a resampling frequency (rmsc01 "M", obi_rmsc02 "all") is not restated and says so (the
    reference's own pd.date_range(..., closed=) fails under pandas 2)"""
    import pandas as pd
    m = mx.VecMarket("value_noise", [7], book_log=CAP)
    m.run()
    paths = m.write_logs(0, str(tmp_path / "vn"))
    assert sorted(os.path.basename(p) for p in paths) == ["fundamental_JPM.bz2", "summary_log.bz2"]
    r = mx.VecMarket("random_fund_value", [7], book_log=1 << 20, symbol="IBM")
    r.run()
    paths = r.write_logs(0, str(tmp_path / "rfv"))
    assert sorted(os.path.basename(p) for p in paths) == ["fundamental_IBM.bz2", "summary_log.bz2"]
    assert len(pd.read_pickle(paths[1] if "fund" in paths[1] else paths[0], compression="bz2")) > 0
    q = mx.VecMarket("rmsc01", [7], book_log=CAP)
    with pytest.raises(NotImplementedError):
        q.write_logs(0, str(tmp_path / "r1"))


@pytest.mark.parametrize("tname", ["IBM_2003-01-14", "GOOG_2012-06-21"])
def test_gpu_replay_book_log_equals_reference(mx, tname, tmp_path):
    """config/marketreplay.py (book_freq 0) on the device's price ladder: the host replay of its
    book-update records (limit orders, cancellations, modifyOrder's head-replace) gives the
    reference's every book_log row and exchange event (digests; the first rows verbatim), and
    write_logs writes summary_log + ORDERBOOK_<sym>_FULL, with no fundamental file (oracle=None)"""
    import golden_util as gu
    import pandas as pd
    from mxabides import tape
    z = np.load(os.path.join(GOLDEN, "marketreplay_%s_1_booklog.npz" % tname))
    tp = tape.Tape.load(os.path.join(GOLDEN, "tape_%s.npz" % tname))
    m = mx.VecMarket("marketreplay_runner", [0, 0], tape=tp, book_log=CAP)
    m.run()
    s = m.summary()
    assert (s["status"] == 1).all(), s["err"]
    for e in range(2):
        rows = m.book_log_rows(e)
        assert np.array_equal(np.asarray(gu.book_row_digests(rows), dtype=np.uint64), z["row_digests"])
        assert np.array_equal(bl.strip_executions(rows)[:len(z["rows"])], z["rows"])
    ev = m.exchange_events(0)
    assert len(ev) == int(z["n_events"])
    mid = pd.Timestamp(tp.date).value
    assert gu.event_digest(zip((ev.index.asi8 - mid).tolist(), ev["EventType"], ev["Event"])) == int(z["ev_digest"])
    if tname.startswith("IBM"):  # the narrow frame of GOOG is 47 M cells: the same code, not rerun here
        paths = m.write_logs(0, str(tmp_path))
        assert sorted(os.path.basename(p) for p in paths) == ["ORDERBOOK_IBM_FULL.bz2", "summary_log.bz2"]
        back = pd.read_pickle(os.path.join(str(tmp_path), "ORDERBOOK_IBM_FULL.bz2"), compression="bz2")
        assert back.index.names == ["time", "quote"]
        assert back.index.get_level_values(0).nunique() == len({t for t, _, _, _, _ in bl.iter_rows(m.book_log_rows(0))})


@pytest.mark.parametrize("cfg", ["hist_fund_value", "hist_fund_diverse"])
def test_gpu_external_file_oracle_f_log_equals_reference(mx, cfg, tmp_path):
    """the ExternalFileOracle's f_log from the device (the value agents' observations, the
    kernelStopping pass) equals the reference's; write_logs writes fundamental_JPM"""
    import pandas as pd
    from golden_util import market_kw
    z = np.load(os.path.join(GOLDEN, "%s_7_flog.npz" % cfg))
    m = mx.VecMarket(cfg, [7], book_log=1 << 20, **market_kw(cfg))
    m.run()
    df = m.fundamental_log(0)
    assert np.array_equal(df.index.asi8 - pd.Timestamp(bl.SESSION_DATE).value, z["fund_time"])
    assert np.array_equal(df["FundamentalValue"].to_numpy(), z["fund_value"])
    paths = m.write_logs(0, str(tmp_path))
    assert sorted(os.path.basename(p) for p in paths) == ["fundamental_JPM.bz2", "summary_log.bz2"]
    assert pd.read_pickle(os.path.join(str(tmp_path), "fundamental_JPM.bz2"), compression="bz2").equals(df)
