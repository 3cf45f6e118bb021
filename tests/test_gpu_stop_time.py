"""Kernel.runner with a caller's stopTime on the device (mxa_set_stop_time / mxa_run_until):
bit-exact against reference runs with kernelStopTime replaced (golden_util.STOP_FIXTURES) and
against the oracle's ora_set_stop on batches."""
import numpy as np
import pytest

import pyoracle
from golden_util import STOP_FIXTURES, first_mismatch, load_named

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


@pytest.mark.parametrize("cfg,seed,stop,name", STOP_FIXTURES)
def test_gpu_stop_time_matches_reference(mx, cfg, seed, stop, name):
    d, ref, summ = load_named(name)
    m = mx.VecMarket(cfg, [seed], trace_cap=len(ref) + 1)
    ev = m.run_until(stop)
    s = m.summary()
    assert s["status"][0] == 1, "env error %d" % s["err"][0]
    assert int(ev[0]) == d["events"] and "%016x" % int(s["hash"][0]) == d["hash"]
    assert first_mismatch(m.trace(0), ref) == -1
    assert int(s["current_time"][0]) == d["final_time"]
    assert m.book(0, 0) == d["bids"] and m.book(0, 1) == d["asks"]
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"] and means == d["mean_lines"]
    got = m.summary_log(0)
    assert got == summ and all(type(a["Event"]) is type(b["Event"]) for a, b in zip(got, summ))


@pytest.mark.parametrize("cfg,n,stop", [("rmsc03", 64, 10 * 3600 * 10 ** 9 + 123),
                                        ("sparse_zi_100", 32, 13 * 3600 * 10 ** 9)])
def test_gpu_stop_time_batch_equals_oracle(mx, cfg, n, stop):
    """per env against the oracle; the override survives a reset and a chunked rerun; restoring
    the config's stop gives the ordinary run"""
    seeds = (np.arange(n, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket(cfg, seeds)
    m.set_stop_time(stop)
    m.run(chunk=3001)
    s = m.summary()
    for i, sd in enumerate(seeds[:8]):
        o = pyoracle.OracleEnv(cfg, int(sd))
        o.set_stop(stop)
        o.run()
        assert (int(s["events"][i]), int(s["hash"][i])) == (o.events, o.hash), i
    h1 = s["hash"].copy()
    m.reset()
    m.run()
    assert (m.summary()["hash"] == h1).all()
    m.set_stop_time(None)
    m.reset()
    m.run()
    ev, hs, _ = pyoracle.run_batch(cfg, seeds.astype(np.uint32), threads=8)
    s = m.summary()
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()
