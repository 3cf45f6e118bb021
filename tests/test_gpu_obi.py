"""GPU parity of config/obi_rmsc02.py (rmsc02's market with 89 ZI agents and 5
OrderBookImbalanceAgent trading the bid share of 10 levels of hourly market data) against the CPU
oracle: pop counts and per-pop trace hashes, the book, holdings and the summary log.  The
reference fixtures (seeds 7, 123456789 flat; 30, 107 with OBI trades) run through
test_gpu_parity.py (golden_util.FIXTURES)."""
import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def test_gpu_obi_rmsc02_batch_equals_oracle(mx):
    seeds = (np.arange(64, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket("obi_rmsc02", seeds)
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("obi_rmsc02", seeds.astype(np.uint32), threads=8)
    ok = s["status"] == 1
    assert ok.all(), (s["status"], s["err"])
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


def test_gpu_obi_rmsc02_chunked_launches_equal_oracle(mx):
    seeds = [123456789, 7, 42]
    m = mx.VecMarket("obi_rmsc02", seeds)
    m.run(chunk=997)
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("obi_rmsc02", np.array(seeds, dtype=np.uint32), threads=3)
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()


def test_gpu_obi_rmsc02_state_and_summary_equal_oracle(mx):
    seeds = [30, 107]
    m = mx.VecMarket("obi_rmsc02", seeds)
    m.run()
    for i, sd in enumerate(seeds):
        o = pyoracle.OracleEnv("obi_rmsc02", sd)
        o.run()
        assert m.book(i, 0) == o.book(0) and m.book(i, 1) == o.book(1)
        o.finish()
        rep = o.report()
        h, means = m.report(i)
        assert h == [l for l in rep if l.startswith("Final holdings")]
        assert means == [l for l in rep if not l.startswith("Final holdings")]
        assert m.summary_log(i) == o.summary_log()
