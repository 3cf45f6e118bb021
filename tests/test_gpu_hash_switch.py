"""The per-pop parity hash is test instrumentation (the reference computes nothing like it).
bench.py times the market step with it off, so these tests prove that switching it off changes
nothing but the hash field: the whole HBM block of every env (agent records, open orders, RNG
streams, queue, book, trade history) is byte-identical to the hash-on run except the 8-byte
hash, for the bench workload's seeds, and the GymKernel composition steps to the same
observations."""
import numpy as np
import pytest

import mxabides
from mxabides import shard
from mxabides.gym import VecABIDESEnv

pytestmark = pytest.mark.gpu
HASH_OFF = 16  # EnvHdr.hash (include/mxa.h layout: cur, pops, hash, ...)
KC_OFF, KC_END = 368, 368 + 28 * 4  # EnvHdr.kc: the event-class counters instrumented runs keep



def _blocks(m, envs):
    """env blocks with the hash field and the event-class counters (mxa_read_counters) zeroed:
    the only two places where the instrumented and the plain run may differ.  (Empty saved-queue
    slots carry no payload words: save() writes zeros there, so stale LDS contents cannot leak
    into the env block.)"""
    n = m.env_bytes
    out = []
    for e in envs:
        b = m.raw(int(e), 0, n)
        b[HASH_OFF:HASH_OFF + 8] = 0
        b[KC_OFF:KC_END] = 0
        out.append(b)
    return out


@pytest.mark.parametrize("config,n", [("rmsc03", 512), ("sparse_zi_100", 128), ("value_noise", 128)])
def test_hash_off_leaves_every_env_block_identical(config, n):
    seeds = shard.env_seeds(0, 0, 1, n)
    on = mxabides.VecMarket(config, seeds)
    on.run()
    off = mxabides.VecMarket(config, seeds)
    off.set_parity_hash(False)
    off.run()
    s_on, s_off = on.summary(), off.summary()
    for k in ("events", "status", "current_time", "order_counter"):
        assert (s_on[k] == s_off[k]).all(), k
    assert (s_off["hash"] != s_on["hash"]).all()  # the hash really was not computed
    envs = np.arange(n)
    lay = on.layout()
    for e, a, b in zip(envs, _blocks(on, envs), _blocks(off, envs)):
        if not np.array_equal(a, b):
            d = np.nonzero(a != b)[0]
            sec = max((o, k) for k, o in lay.items() if 0 < o <= d[0]) if d[0] >= 512 else (0, "header")
            raise AssertionError("%s env %d: %d bytes differ, first at %d (%s), last at %d: %s vs %s" % (
                config, e, len(d), d[0], sec[1], d[-1], a[d[:8]].tolist(), b[d[:8]].tolist()))


def test_hash_off_bench_workload_summaries_identical():
    seeds = shard.env_seeds(0, 0, 1, 4096)
    on = mxabides.VecMarket("rmsc03", seeds)
    on.run()
    off = mxabides.VecMarket("rmsc03", seeds)
    off.set_parity_hash(False)
    off.run()
    s_on, s_off = on.summary(), off.summary()
    for k in ("events", "status", "current_time", "order_counter"):
        assert (s_on[k] == s_off[k]).all(), k
    for e in range(0, 4096, 97):
        assert on.agents(e) == off.agents(e), e
        assert on.book(e, 0) == off.book(e, 0) and on.book(e, 1) == off.book(e, 1), e


def test_hash_off_gym_steps_identical():
    seeds = [123456789, 2024, 7, 123, 99991, 31337]
    a, b = VecABIDESEnv(seeds=seeds), VecABIDESEnv(seeds=seeds)
    b.set_parity_hash(False)
    rs = np.random.RandomState(5)
    for _ in range(27):
        act = rs.uniform(0, 1, (len(seeds), 3))
        act[:, 0] *= 0.05
        oa, da, va, ea = a.step(act)
        ob, db, vb, eb = b.step(act)
        assert np.array_equal(oa, ob) and (da == db).all() and (va == vb).all() and (ea == eb).all()
    sa, sb = a.summary(), b.summary()
    assert (sa["events"] == sb["events"]).all()
    for e in range(len(seeds)):
        assert a.agents(e) == b.agents(e) and a.book(e, 0) == b.book(e, 0)
