"""GPU parity of config/random_fund_value.py (rmsc03's agent classes at 5,101 agents: 5000 noise
agents waking once in 09:30-16:00, 100 value agents, the sparse mean-reverting oracle, a whole
09:30-16:00 session) and config/random_fund_diverse.py (the same plus a MarketMakerAgent and 25
momentum agents) against the CPU oracle: pop counts and per-pop trace hashes, the book, holdings
and the summary log.  Every agent keeps a wakeup pending, so the event queue holds ~5,100 events
(96 slots per lane: two groups per lane in LDS, six in HBM; 13-bit recipient field in the event
key); the reference fixtures (seeds 7, 123456789) run through test_gpu_parity.py
(golden_util.FIXTURES)."""
import numpy as np
import pytest

import pyoracle
from golden_util import market_kw

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


# hist_fund_*: the same markets on the ExternalFileOracle (config/hist_fund_value.py,
# hist_fund_diverse.py) with the fixtures' JPM mid-price series
CONFIGS = ["random_fund_value", "random_fund_diverse", "hist_fund_value", "hist_fund_diverse"]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_gpu_random_fund_batch_equals_oracle(mx, cfg):
    seeds = (np.arange(64, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch(cfg, seeds.astype(np.uint32), threads=8)
    assert (s["status"] == 1).all(), (s["status"], s["err"])
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg", CONFIGS)
def test_gpu_random_fund_chunked_launches_equal_oracle(mx, cfg):
    """997-pop launches: the 6,144-slot queue (payloads in HBM) and the 128-bit free-slot masks
    are saved and rebuilt ~100-200 times per env"""
    seeds = [123456789, 7, 42]
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run(chunk=997)
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch(cfg, np.array(seeds, dtype=np.uint32), threads=3)
    assert (s["status"] == 1).all(), (s["status"], s["err"])
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg", CONFIGS)
def test_gpu_random_fund_state_and_summary_equal_oracle(mx, cfg):
    seeds = [7, 1008]
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    for i, sd in enumerate(seeds):
        o = pyoracle.OracleEnv(cfg, sd)
        o.run()
        assert m.book(i, 0) == o.book(0) and m.book(i, 1) == o.book(1)
        o.finish()
        rep = o.report()
        h, means = m.report(i)
        assert h == [l for l in rep if l.startswith("Final holdings")]
        assert means == [l for l in rep if not l.startswith("Final holdings")]
        assert m.summary_log(i) == o.summary_log()
