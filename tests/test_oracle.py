"""The CPU parity oracle is pinned against the reference's own outputs:
golden traces captured from the reference (tests/golden/gen_fixtures.py) and the
reference's known-answer file tests/sparse_zi_1000.txt."""
import json
import os

import numpy as np
import pytest

import pyoracle
from golden_util import FIXTURES, GOLDEN, first_mismatch, kat_lines, load


@pytest.mark.parametrize("cfg,seed", FIXTURES)
def test_oracle_matches_reference_fixture(cfg, seed):
    d, ref = load(cfg, seed)
    e = pyoracle.OracleEnv(cfg, seed, trace_cap=len(ref))
    e.run()
    assert e.error[0] == 0
    tr = e.trace()
    assert first_mismatch(tr, ref) == -1 or len(tr) == len(ref) and first_mismatch(tr, ref) == -1
    assert e.events == d["events"]
    assert "%016x" % e.hash == d["hash"]
    e.finish()
    rep = e.report()
    assert [l for l in rep if l.startswith("Final holdings")] == d["final_holdings_lines"]
    assert [l for l in rep if not l.startswith("Final holdings")] == d["mean_lines"]
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert e.order_counter - 1 == d["order_id_counter"]
    assert e.last_trade == d["last_trade"]


def test_oracle_sparse_zi_1000_known_answer():
    """tests/sparse_zi_1000.txt of the reference: 1000 holdings lines, 7 means, 185200 msgs."""
    holdings, means = kat_lines()
    e = pyoracle.OracleEnv("sparse_zi_1000", 123456789)
    e.run()
    assert e.events == 185200
    e.finish()
    rep = e.report()
    assert sorted(l for l in rep if l.startswith("Final holdings")) == sorted(holdings)
    assert [l for l in rep if not l.startswith("Final holdings")] == means


def test_oracle_rng_known_answers(golden):
    kats = json.load(open(os.path.join(golden, "rng_kats.json")))
    for seed, d in kats.items():
        r = pyoracle.RandomState(int(seed))
        assert [r.u32() for _ in range(len(d["u32"]))] == d["u32"]
        r = pyoracle.RandomState(int(seed))
        assert [r.rand() for _ in range(len(d["double"]))] == d["double"]
        r = pyoracle.RandomState(int(seed))
        for name, a, b, v in d["mixed"]:
            if name == "randint":
                assert r.randint(a, b) == v
            elif name == "normal":
                assert r.normal(a, b) == v
            elif name == "exponential":
                assert r.exponential(a) == v
            elif name == "uniform":
                assert r.uniform(a, b) == v
            else:
                assert r.rand() == v


def test_oracle_batch_runner_deterministic():
    seeds = np.arange(1, 9, dtype=np.uint32)
    ev1, h1, _ = pyoracle.run_batch("rmsc03", seeds, threads=4)
    ev2, h2, _ = pyoracle.run_batch("rmsc03", seeds[::-1].copy(), threads=2)
    assert (ev1 == ev2[::-1]).all() and (h1 == h2[::-1]).all()
    for i, s in enumerate(seeds[:2]):
        e = pyoracle.OracleEnv("rmsc03", int(s))
        e.run()
        assert e.events == ev1[i] and e.hash == h1[i]


@pytest.mark.parametrize("cfg,seed", FIXTURES)
def test_oracle_summary_log_matches_reference(cfg, seed):
    """Kernel.summaryLog (what writeSummaryLog pickles): STARTING_CASH, FINAL_CASH_POSITION,
    ENDING_CASH and the agents' FINAL_VALUATION, int/float types included"""
    with open(os.path.join(os.path.dirname(__file__), "golden", "%s_%d_summary.json" % (cfg, seed))) as f:
        ref = json.load(f)
    e = pyoracle.OracleEnv(cfg, seed)
    e.run()
    e.finish()
    got = e.summary_log()
    assert e.error[0] == 0
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a == b and type(a["Event"]) is type(b["Event"]), (a, b)


def test_oracle_rmsc01_kernel_stopping_index_error():
    """rmsc01 seed 123456789: the reference's own run ends in an IndexError inside
    ZeroIntelligenceAgent.kernelStopping (agent 42's holdings index past its theta table); the
    fixture holds the trace, the book and the stdout / summary rows written before the crash"""
    d, ref = load("rmsc01", 123456789)
    assert d["stop_error"].startswith("IndexError")
    e = pyoracle.OracleEnv("rmsc01", 123456789, trace_cap=len(ref))
    e.run()
    assert e.error[0] == 0 and first_mismatch(e.trace(), ref) == -1
    assert e.events == d["events"] and "%016x" % e.hash == d["hash"]
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    e.finish()
    assert e.error[0] == -10
    rep = [l for l in e.report() if l.startswith("Final holdings")]
    assert rep[:len(d["final_holdings_lines"])] == d["final_holdings_lines"]
    with open(os.path.join(GOLDEN, "rmsc01_123456789_summary.json")) as f:
        summ = json.load(f)
    assert e.summary_log()[:len(summ)] == summ


def test_oracle_sbmm_unbound_mid_matches_reference():
    """rmsc03 + SpreadBasedMarketMakerAgent (polling), seed 123456798: the agent's first
    QUERY_SPREAD reply has an empty side and no last mid, so receiveMessage reads an unbound `mid`
    (SpreadBasedMarketMakerAgent.py:100-111) and the reference's run ends in UnboundLocalError
    after 649 pops; the oracle stops at the same pop with error -18"""
    d, ref = load("rmsc03_sbmm_poll", 123456798)
    assert d["stop_error"].startswith("UnboundLocalError")
    e = pyoracle.OracleEnv("rmsc03_sbmm_poll", 123456798, trace_cap=len(ref) + 10)
    e.run()
    assert e.error[0] == -18
    assert e.events == d["events"] == 649
    assert first_mismatch(e.trace(), ref) == -1 and len(e.trace()) == len(ref)
