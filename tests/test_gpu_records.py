"""mxa_write_records (include/mxa.h): the per-env episode record bench.py all-gathers across ranks
 agrees with the handle's own readers: summary counters, the env seed, and the
cash / holdings / mark-to-market gain summed over the trading agents (TradingAgent.markToMarket,
TradingAgent.py:609-633) or the execution agent's own for a GymKernel handle."""
import numpy as np
import pytest
import torch

from mxabides import shard

pytestmark = pytest.mark.gpu


def _check(rec, s, seeds):
    assert (rec[:, shard.R_EVENTS] == s["events"]).all()
    assert (rec[:, shard.R_HASH].view(np.uint64) == s["hash"]).all()
    assert (rec[:, shard.R_STATUS] == s["status"]).all()
    assert (rec[:, shard.R_TIME] == s["current_time"]).all()
    assert (rec[:, shard.R_SEED] == np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF).all()


def test_records_kernel_runner_config():
    import mxabides
    seeds = [123456789, 7, 1008, 99]
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
