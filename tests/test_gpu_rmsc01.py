"""GPU parity of config/rmsc01.py (RMSC-1: MarketMakerAgent, ZI, HeuristicBeliefLearningAgent,
Momentum) against the CPU oracle: every env's pop count and per-pop trace hash, the book, the
agents' holdings and the summary log.  The reference fixtures of rmsc01 run through the generic
tests in test_gpu_parity.py (golden_util.FIXTURES); these cover more seeds, launch boundaries
(the order-history ring and the book's record indices saved across launches) and the HBL paths."""
import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def test_gpu_rmsc01_batch_equals_oracle(mx):
    seeds = (np.arange(64, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket("rmsc01", seeds)
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc01", seeds.astype(np.uint32), threads=8)
    ok = s["status"] == 1
    assert ok.all(), (s["status"], s["err"])
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


def test_gpu_rmsc01_chunked_launches_equal_oracle(mx):
    """many save/restore cycles: queue, book (incl. each resting order's history-record index),
    the LDS RNG windows and the HBL streams survive launch boundaries"""
    seeds = [123456789, 7, 42]
    m = mx.VecMarket("rmsc01", seeds)
    m.run(chunk=4999)
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc01", np.array(seeds, dtype=np.uint32), threads=3)
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()


def test_gpu_rmsc01_kernel_stopping_index_error(mx):
    """seed 123456789 ends in the reference's IndexError in ZeroIntelligenceAgent.kernelStopping
    (a ZI agent's holdings beyond its theta table): the device reports it for the same agent"""
    import mxabides
    m = mx.VecMarket("rmsc01", [123456789])
    m.run()
    with pytest.raises(mxabides.MxaError, match="agent 42.*IndexError"):
        m.summary_log(0)
    o = pyoracle.OracleEnv("rmsc01", 123456789)
    o.run()
    o.finish()
    assert o.error[0] == -10


def test_gpu_rmsc01_state_and_summary_equal_oracle(mx):
    seeds = [7, 99]
    m = mx.VecMarket("rmsc01", seeds)
    m.run()
    for i, sd in enumerate(seeds):
        o = pyoracle.OracleEnv("rmsc01", sd)
        o.run()
        assert m.book(i, 0) == o.book(0) and m.book(i, 1) == o.book(1)
        o.finish()
        rep = o.report()
        h, means = m.report(i)
        assert h == [l for l in rep if l.startswith("Final holdings")]
        assert means == [l for l in rep if not l.startswith("Final holdings")]
        assert m.summary_log(i) == o.summary_log()
