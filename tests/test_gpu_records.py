"""mxa_write_records (include/mxa.h): the per-env episode record bench.py all-gathers across ranks
 agrees with the handle's own readers: summary counters, the env seed, and the
cash / holdings / mark-to-market gain summed over the trading agents (TradingAgent.markToMarket,
TradingAgent.py:609-633) or the execution agent's own for a GymKernel handle."""
import json
import os

import numpy as np
import pytest
import torch

from mxabides import shard

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _check(rec, s, seeds):
    assert (rec[:, shard.R_EVENTS] == s["events"]).all()
    assert (rec[:, shard.R_HASH].view(np.uint64) == s["hash"]).all()
    assert (rec[:, shard.R_STATUS] == s["status"]).all()
    assert (rec[:, shard.R_TIME] == s["current_time"]).all()
    assert (rec[:, shard.R_SEED] == np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF).all()


def test_records_kernel_runner_config():
    import mxabides
    seeds = [123456789, 7, 1008, 99]  # the first three are reference fixtures
    m = mxabides.VecMarket("rmsc03", seeds)
    m.run()
    out = torch.zeros((len(seeds), shard.RECORD_WORDS), dtype=torch.int64, device="cuda")
    m.write_records(out.data_ptr())
    torch.cuda.synchronize()
    rec = out.cpu().numpy()
    s = m.summary()
    _check(rec, s, seeds)
    assert (rec[:, shard.R_LAST] == s["last_trade"]).all() and (rec[:, shard.R_OCNT] == s["order_counter"]).all()
    for e in range(len(seeds)):
        ag = m.agents(e)[1:]
        assert rec[e, shard.R_CASH] == sum(a["cash"] for a in ag)
        assert rec[e, shard.R_HOLD] == sum(a["shares"] for a in ag) == 0  # every trade has two sides
        gain = sum(a["cash"] + (a["last_trade"] * a["shares"] if a["shares"] else 0) - a["starting_cash"] for a in ag)
        assert rec[e, shard.R_GAIN] == gain
    # the reference's own Kernel.summaryLog of the fixture seeds (tests/golden/rmsc03_<seed>_summary.json):
    # cash = sum of FINAL_CASH_POSITION, gain = sum of ENDING_CASH - STARTING_CASH (TradingAgent.py:101, 118-123)
    for e, seed in enumerate(seeds[:3]):
        with open(os.path.join(GOLD, "rmsc03_%d_summary.json" % seed)) as f:
            rows = json.load(f)
        ev = {(r["AgentID"], r["EventType"]): r["Event"] for r in rows}
        ids = sorted({r["AgentID"] for r in rows})
        assert rec[e, shard.R_CASH] == sum(ev[(a, "FINAL_CASH_POSITION")] for a in ids), seed
        assert rec[e, shard.R_GAIN] == sum(ev[(a, "ENDING_CASH")] - ev[(a, "STARTING_CASH")] for a in ids), seed


def test_records_gym_handle():
    from mxabides.gym import VecABIDESEnv
    seeds = [123456789, 2024]
    v = VecABIDESEnv(seeds=seeds)
    rs = np.random.RandomState(3)
    for _ in range(27):
        a = rs.uniform(0, 1, (2, 3))
        a[:, 0] *= 0.05
        v.step(a)
    out = torch.zeros((2, shard.RECORD_WORDS), dtype=torch.int64, device="cuda")
    v.write_records(out.data_ptr())
    torch.cuda.synchronize()
    rec = out.cpu().numpy()
    _check(rec, v.summary(), seeds)
    for e in range(2):
        cash, shares, _ = v.agents(e)[v.n_agents - 1]  # DummyRLExecutionAgent (id 64)
        assert rec[e, shard.R_CASH] == cash and rec[e, shard.R_HOLD] == shares


@pytest.mark.parametrize("cfg,seed", [("rmsc03", 123456789), ("sparse_zi_100", 123456789), ("value_noise", 7),
                                      ("sparse_zi_1000", 123456789), ("random_fund_value", 7)])
def test_counters_agree_with_the_trace(cfg, seed):
    """the event-class counters of an instrumented run (mxa_read_counters, the algorithmic-byte
    count of bench.py) equal the per-kind histogram of the env's full parity trace, whose records
    are the reference's (test_gpu_parity)"""
    import mxabides
    from mxabides import counters as mc
    m = mxabides.VecMarket(cfg, [seed], trace_cap=400000)
    m.run()
    c = m.counters()[0]
    tr = m.trace(0)
    s = m.summary()
    assert len(tr) == s["events"][0] == c[mc.C_POPS]
    hist = np.bincount(tr[:, 3], minlength=26)
    assert (c[:25] == hist[:25]).all(), (c[:25], hist[:25])
    # every pop but a requeue consumes an event: the initial wakeups (one per agent) plus the run's pushes
    assert c[mc.C_PUSH] + m.n_agents >= c[mc.C_POPS] - c[mc.C_REQUEUE] and c[mc.C_RNG] > 0
    bpe, parts, units = mc.bytes_per_event(m.counters())
    assert 100 < bpe < 600 and 0 < units["record_round_trips"] <= 1
    # every agent record's stream position is a real one: an event that ran on a record it never
    # loaded (the round-4 early record fetch once did, for the exchange) stores a zeroed position
    assert 0 <= units["rng_words"] < 50, units


def test_counters_off_without_instrumentation():
    import mxabides
    m = mxabides.VecMarket("rmsc03", [7, 8])
    m.set_parity_hash(False)
    m.run()
    c = m.counters()
    assert (c[:, :26] == 0).all() and (c[:, 28] > 0).all()
