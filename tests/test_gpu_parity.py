"""GPU parity: libmxa's HIP kernels against the CPU oracle and the reference fixtures.

Every test goes through the C-ABI (include/mxa.h) via mxabides; the oracle is only the
checker.  Bar: bit-exact trace records / hashes / books / holdings (integer work); the
floating-point intermediates (oracle OU process, Bayesian estimates, latency model) are
only observable through the integers they round to, so they are bit-exact too.
"""
import json
import os

import numpy as np
import pytest

import pyoracle
from golden_util import market_kw, FIXTURES, first_mismatch, kat_lines, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import mxabides
    mxabides.load()
    return mxabides


def test_device_rng_matches_numpy_kats(mx, golden):
    import ctypes
    L = mx.load()
    kats = json.load(open(os.path.join(golden, "rng_kats.json")))
    for seed, d in kats.items():
        out = np.zeros(700, dtype=np.float64)
        assert L.mxa_rng_probe(0, int(seed), 0, 0.0, 0.0, 700, out.ctypes.data) == 0
        assert out.astype(np.int64).tolist() == d["u32"]
        out = np.zeros(300, dtype=np.float64)
        assert L.mxa_rng_probe(0, int(seed), 1, 0.0, 0.0, 300, out.ctypes.data) == 0
        assert out.tolist() == d["double"]
    # distributions against the oracle restatement (itself pinned to numpy above)
    for mode, a, b, fn in [(2, 20, 50, "randint"), (3, 1e5, 100.0, "normal"), (4, 1e12, 0, "exponential"),
                           (5, 21000.0, 1.3e7, "uniform")]:
        out = np.zeros(2000, dtype=np.float64)
        assert L.mxa_rng_probe(0, 424242, mode, a, b, 2000, out.ctypes.data) == 0
        r = pyoracle.RandomState(424242)
        ref = [getattr(r, fn)(*((a, b) if fn != "exponential" else (a,))) for _ in range(2000)]
        assert out.tolist() == [float(x) for x in ref]


def test_device_glibc_math(mx):
    import ctypes
    L = mx.load()
    libm = ctypes.CDLL("libm.so.6")
    rs = np.random.RandomState(5)
    n = 200_000
    cases = [(0, 1.0 - rs.rand(n), None), (0, 1 + (rs.rand(n) - 0.5) * 0.2, None),
             (1, -1.67e-12 * np.floor(rs.uniform(0, 2.4e13, n)), None),
             (2, np.full(n, 1 - 1.67e-15), np.floor(rs.uniform(0, 2.5e13, n))),
             (2, rs.uniform(0.05, 1, n), np.full(n, 3.0))]
    for mode, x, y in cases:
        x = np.ascontiguousarray(x)
        yy = np.ascontiguousarray(x if y is None else y)
        out = np.zeros(n)
        assert L.mxa_math_probe(0, mode, x.ctypes.data, yy.ctypes.data, out.ctypes.data, n) == 0
        # host reference through the very same libm the reference used
        fn = {0: libm.log, 1: libm.exp, 2: libm.pow}[mode]
        fn.restype = ctypes.c_double
        fn.argtypes = [ctypes.c_double] * (2 if mode == 2 else 1)
        idx = np.random.RandomState(mode).randint(0, n, 20000)
        ref = np.array([fn(x[i], yy[i]) if mode == 2 else fn(x[i]) for i in idx])
        assert (out[idx].view(np.uint64) == ref.view(np.uint64)).all()


@pytest.mark.parametrize("cfg,seed", FIXTURES)
def test_gpu_trace_matches_reference(mx, cfg, seed):
    d, ref = load(cfg, seed)
    m = mx.VecMarket(cfg, [seed], trace_cap=len(ref), **market_kw(cfg))
    m.run()
    s = m.summary()
    tr = m.trace(0)
    assert s["status"][0] == 1, "env error %d" % s["err"][0]
    assert first_mismatch(tr, ref) == -1
    assert int(s["events"][0]) == d["events"]
    assert "%016x" % int(s["hash"][0]) == d["hash"]
    assert m.book(0, 0) == d["bids"] and m.book(0, 1) == d["asks"]
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"]
    assert means == d["mean_lines"]
    assert int(s["order_counter"][0]) - 1 == d["order_id_counter"]


def test_gpu_sparse_zi_1000_known_answer(mx):
    holdings, means = kat_lines()
    m = mx.VecMarket("sparse_zi_1000", [123456789])
    m.run()
    s = m.summary()
    assert int(s["events"][0]) == 185200
    h, mm = m.report(0)
    assert sorted(h) == sorted(holdings) and mm == means


@pytest.mark.parametrize("cfg,n", [("rmsc03", 96), ("sparse_zi_100", 64), ("value_noise", 1024)])
def test_gpu_batch_equals_oracle(mx, cfg, n):
    seeds = (np.arange(n, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch(cfg, seeds.astype(np.uint32), threads=8)
    assert (s["status"] == 1).all()
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


def test_gpu_bench_workload_equals_oracle(mx):
    """the exact bench.py workload (rmsc03 x4096, seeds 123456789 + env) is bit-exact per env"""
    from mxabides import shard
    seeds = shard.env_seeds(0, 0, 1, 4096)
    m = mx.VecMarket("rmsc03", seeds)
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc03", seeds, threads=min(16, os.cpu_count() or 1))
    assert (s["status"] == 1).all()
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg,n", [("sparse_zi_1000", 1024), ("sparse_zi_100", 4096), ("value_noise", 4096)])
def test_gpu_config_bench_workload_equals_oracle(mx, cfg, n):
    """the exact `bench.py --config CFG --envs N` workloads (seeds 123456789 + env) are bit-exact
    per env: sparse_zi_1000 x1024 is BASELINE configs[2] at full size"""
    from mxabides import shard
    seeds = shard.env_seeds(0, 0, 1, n)
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch(cfg, seeds, threads=min(16, os.cpu_count() or 1))
    assert (s["status"] == 1).all()
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg,n", [("sparse_zi_1000", 8)])
def test_gpu_wide_config_equals_oracle(mx, cfg, n):
    seeds = (np.arange(n, dtype=np.int64) * 104729 + 3) & 0xFFFFFFFF
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch(cfg, seeds.astype(np.uint32), threads=8)
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg,seeds", [
    ("rmsc03", [3, 5, 123456789, 1008]),            # flat queue (3 slots per lane)
    ("sparse_zi_100", [3, 5, 123456789]),           # flat queue (8 slots per lane, select tree)
    ("value_noise", [3, 5, 123456789]),             # flat queue (6 slots per lane, select tree)
    ("sparse_zi_1000", [123456789, 5]),             # grouped queue: 3 groups of 12, payload in HBM
    ("random_fund_value", [123456789, 5]),          # two-tier queue: 2 LDS groups + 6 HBM groups of 12
    ("rmsc03_sbmm", [123456789, 7]),                # ladder deques in the record, MARKET_DATA subscription
    ("rmsc03_sbmm_poll", [123456789, 7]),
])
def test_gpu_chunked_launches_equal_single(mx, cfg, seeds):
    """many save/restore cycles of the queue (LDS) and the book (VGPRs): the reload refills the
    queue from the saved events and, in grouped mode, rebuilds the group minima from a
    non-empty queue"""
    a = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    a.run(chunk=1 << 30)
    b = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    b.run(chunk=977)
    sa, sb = a.summary(), b.summary()
    assert (sa["status"] == 1).all() and (sb["status"] == 1).all()
    assert (sa["hash"] == sb["hash"]).all() and (sa["events"] == sb["events"]).all()
    ev, hs, _ = pyoracle.run_batch(cfg, np.array(seeds, dtype=np.uint32), threads=4)
    assert (sb["events"] == ev).all() and (sb["hash"] == hs).all()


def test_gpu_launch_schedule_compacted_grid_equals_oracle(mx):
    """mxa_set_launch_schedule: a short first launch, then launches over the compacted list of
    running envs (one wave per listed env); envs that end early (seed 1008's stalled market
    maker and its like) leave the grid, and every env still equals the oracle"""
    seeds = ((np.arange(96, dtype=np.int64) * 7919 + 1008) & 0xFFFFFFFF).astype(np.uint32)
    m = mx.VecMarket("rmsc03", seeds)
    m.set_launch_schedule(3000)
    nl = m.run(chunk=40000)
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc03", seeds, threads=8)
    assert (s["status"] == 1).all()
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()
    assert 2 <= nl <= 2 + -(-(int(ev.max()) - 3000) // 40000)
    m.set_launch_schedule(0)
    m.reset()
    assert m.run(chunk=1 << 22) == 1
    assert (m.summary()["hash"] == hs).all()


def test_gpu_reset_reproduces(mx):
    m = mx.VecMarket("rmsc03", [17, 18])
    m.run()
    h1 = m.summary()["hash"].copy()
    m.reset()
    m.run()
    assert (m.summary()["hash"] == h1).all()


@pytest.mark.parametrize("n", [1, 257])
def test_gpu_odd_env_counts_equal_oracle(mx, n):
    """a single env and a batch that fills no CU evenly (grid = n_envs, one wave per env)"""
    seeds = (np.arange(n, dtype=np.int64) * 15485863 + 99) & 0xFFFFFFFF
    m = mx.VecMarket("rmsc03", seeds)
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc03", seeds.astype(np.uint32), threads=8)
    assert (s["status"] == 1).all()
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()


def test_gpu_launch_budget_then_resume(mx):
    """mxa_run with a launch cap stops mid-episode; later launches finish it bit-exactly"""
    seeds = [123456789, 7]
    m = mx.VecMarket("rmsc03", seeds)
    m.run(chunk=5000, max_launches=3)
    s = m.summary()
    assert (s["status"] == 0).all() and (s["events"] == 15000).all()
    m.run()
    s = m.summary()
    ev, hs, _ = pyoracle.run_batch("rmsc03", np.array(seeds, dtype=np.uint32), threads=2)
    assert (s["events"] == ev).all() and (s["hash"] == hs).all()


@pytest.mark.parametrize("cfg,seed", FIXTURES)
def test_gpu_summary_log_matches_reference(mx, cfg, seed, tmp_path):
    """mxa_finalize (Kernel.runner's kernelStopping pass) + the host summary log equal the
    reference's Kernel.summaryLog; the bz2 pickle round-trips as cli/stats.py reads it"""
    import pandas as pd
    with open(os.path.join(os.path.dirname(__file__), "golden", "%s_%d_summary.json" % (cfg, seed))) as f:
        ref = json.load(f)
    m = mx.VecMarket(cfg, [seed], **market_kw(cfg))
    m.run()
    got = m.summary_log(0)
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a == b and type(a["Event"]) is type(b["Event"]), (a, b)
    m.finalize()  # idempotent: the pass does not save the oracle's advance
    assert m.summary_log(0) == got
    df = pd.read_pickle(m.write_summary_log(0, str(tmp_path)), compression="bz2")
    assert list(df.columns) == ["AgentID", "AgentStrategy", "EventType", "Event"] and len(df) == len(ref)


@pytest.mark.parametrize("cfg,n", [("rmsc03", 64), ("sparse_zi_100", 16), ("value_noise", 64)])
def test_gpu_summary_log_batch_equals_oracle(mx, cfg, n):
    seeds = (np.arange(n, dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
    m = mx.VecMarket(cfg, seeds, **market_kw(cfg))
    m.run()
    m.finalize()
    for i, s in enumerate(seeds):
        o = pyoracle.OracleEnv(cfg, int(s))
        o.run()
        o.finish()
        ref = o.summary_log()
        got = m.summary_log(i)
        assert got == ref, (cfg, int(s))


def test_gpu_sbmm_unbound_mid_matches_reference(mx):
    """rmsc03 + SpreadBasedMarketMakerAgent (polling), seed 123456798: the reference's run ends in
    the agent's UnboundLocalError after 649 pops; the device stops at the same pop with env error
    28 (ERR_SB_MID) and the same trace"""
    d, ref = load("rmsc03_sbmm_poll", 123456798)
    m = mx.VecMarket("rmsc03_sbmm_poll", [123456798], trace_cap=len(ref) + 10)
    m.run()
    s = m.summary()
    assert int(s["status"][0]) == 2 and int(s["err"][0]) == 28
    assert int(s["events"][0]) == d["events"] == 649
    tr = m.trace(0)
    assert first_mismatch(tr, ref) == -1 and len(tr) == len(ref)
