"""config/rmsc03.py with its market-maker options per env (include/mxa.h mxa_create_params):
the sweep of the reference's only rmsc03 driver script (scripts/rmsc03.sh:5-13, 29-39: pov 0.05,
min order size 25, window 5, 50 ticks, wake-up "10S", seeds 30-35) against reference runs of the
script with those options (tests/golden/gen_fixtures.py "rmsc03%0.05,25,5,50,10S"), and a mixed
option grid at 4096 envs against the C oracle env by env."""
import json
import os

import numpy as np
import pytest

import pyoracle
from golden_util import first_mismatch, load_named
from mxabides import shard
from mxabides.configs import mm_params

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SCRIPT = dict(pov=0.05, min_order_size=25, window_size=5, num_ticks=50, wake_up_freq="10S")
SEEDS = list(range(30, 36))


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def mixed_grid(n, seed=1):
    """every option varied per env: pov 0.01-0.2, sizes 10-50, windows 1-10, 5-50 ticks (ladders of
    12-102 orders: one or two batched passes), wake-ups 1-60 s"""
    rs = np.random.RandomState(seed)
    return mm_params(n, pov=rs.choice([0.01, 0.05, 0.1, 0.2], n), min_order_size=rs.choice([10, 20, 25, 50], n),
                     window_size=rs.choice([1, 5, 10], n), num_ticks=rs.choice([5, 10, 20, 31, 50], n),
                     wake_up_freq=list(rs.choice([1, 5, 10, 60], n) * 10 ** 9))


@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_script_sweep_matches_reference(mx, seed):
    name = "rmsc03_mm_0.05_25_5_50_10S_%d" % seed
    d, ref, summ = load_named(name)
    m = mx.VecMarket("rmsc03", [seed], trace_cap=len(ref), mm_params=mm_params(1, **SCRIPT))
    m.run()
    s = m.summary()
    assert s["status"][0] == 1, "env error %d" % s["err"][0]
    assert first_mismatch(m.trace(0), ref) == -1
    assert int(s["events"][0]) == d["events"] and "%016x" % int(s["hash"][0]) == d["hash"]
    assert m.book(0, 0) == d["bids"] and m.book(0, 1) == d["asks"]
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"] and means == d["mean_lines"]
    got = m.summary_log(0)
    assert len(got) == len(summ)
    for a, b in zip(got, summ):
        assert a == b and type(a["Event"]) is type(b["Event"]), (a, b)


def test_gpu_script_sweep_is_one_batch(mx):
    """the six runs of the sweep as one handle, plus seeds the script never ran, against the oracle"""
    seeds = np.array(SEEDS + list(range(1000, 1058)), dtype=np.uint32)
    p = mm_params(len(seeds), **SCRIPT)
    m = mx.VecMarket("rmsc03", seeds, mm_params=p)
    m.run()
    s = m.summary()
    ev, hs, er, _ = pyoracle.run_batch_mm(seeds, p, 8)
    assert (er == 0).all() and (s["status"] == 1).all()
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()
    for i, seed in enumerate(SEEDS):
        with open(os.path.join(GOLD, "rmsc03_mm_0.05_25_5_50_10S_%d.json" % seed)) as f:
            assert int(s["events"][i]) == json.load(f)["events"]


def test_gpu_default_options_equal_rmsc03(mx):
    """the script's defaults through the parameterised instantiation give rmsc03's every result"""
    seeds = shard.env_seeds(0, 0, 1, 256)
    a = mx.VecMarket("rmsc03", seeds)
    b = mx.VecMarket("rmsc03", seeds, mm_params=mm_params(1))
    a.run()
    b.run()
    sa, sb = a.summary(), b.summary()
    for k in ("status", "events", "hash", "current_time", "order_counter", "last_trade"):
        assert (sa[k] == sb[k]).all(), k


@pytest.mark.timeout(600)
def test_gpu_mixed_options_bench_size_equal_oracle(mx):
    """4096 envs, every env its own options: events, hash and status equal the oracle's per env;
    then the same handle re-run with other options (mxa_set_mm_params + reset)"""
    n = 4096
    seeds = shard.env_seeds(0, 0, 1, n)
    m = mx.VecMarket("rmsc03", seeds, mm_params=mixed_grid(n, 1))
    for k, grid_seed in enumerate((1, 2)):
        p = mixed_grid(n, grid_seed)
        if k:
            m.set_mm_params(p)
            m.reset()
        m.run()
        s = m.summary()
        ev, hs, er, _ = pyoracle.run_batch_mm(seeds, p, min(16, os.cpu_count() or 1))
        assert (er == 0).all()
        bad = np.nonzero((s["status"] != 1) | (s["events"] != ev) | (s["hash"] != hs))[0]
        assert len(bad) == 0, [(int(i), int(s["err"][i]), p[i]) for i in bad[:10]]


def test_gpu_mm_order_size_beyond_int32_is_an_env_error(mx):
    """pov x transacted volume beyond the 32-bit order words: the env stops with error 29
    (ERR_ORDER_SIZE), never a wrapped order size; the reference's Python int has no
    bound, so this is a capacity error of the device, not a reference path.  rmsc03's exchange
    keeps 10 orders of history (stream_history), so the transacted volume the market maker sees
    stays in the hundreds: pov 1e9 outgrows int32 from 3 shares"""
    seeds = [30, 31, 32, 33]
    m = mx.VecMarket("rmsc03", seeds, mm_params=mm_params(len(seeds), pov=1e9))
    m.run()
    s = m.summary()
    assert (s["status"] == 2).all() and (s["err"] == 29).all(), (s["status"], s["err"])
