"""GPU parity of runtime compositions (include/mxa.h mxa_create_config): each
composition's specialised engine (prebuilt by __graft_entry__.build(); these tests never compile)
against reference runs of the same agent list (tests/golden/gen_config_fixtures.py) and against
the oracle over a batch of seeds.  A base script's own composition runs exactly as the built-in
configuration does."""
import numpy as np
import pytest

import pyoracle
from golden_util import COMPOSITION_FIXTURES, composition_names, first_mismatch, load_composition

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    import mxabides
    mxabides.load()
    from mxabides import composition
    return composition


def _composition(C, name):
    seed = next(s for n, s in COMPOSITION_FIXTURES if n == name)
    return C.from_dict(load_composition(name, seed)[0]["composition"])


@pytest.mark.parametrize("base", ["rmsc03", "sparse_zi_100"])
def test_gpu_base_composition_equals_builtin(C, base):
    """mxa_create_config(mxa_config_defaults(base)) is the built-in configuration, env by env"""
    import mxabides
    seeds = (np.arange(64, dtype=np.int64) * 104729 + 5) & 0xFFFFFFFF
    a = mxabides.VecMarket(C.defaults(base), seeds)
    b = mxabides.VecMarket(base, seeds)
    a.run()
    b.run()
    sa, sb = a.summary(), b.summary()
    assert (sa["status"] == 1).all()
    for k in ("events", "hash", "current_time", "order_counter", "last_trade"):
        assert (sa[k] == sb[k]).all(), k
    assert a.n_agents == b.n_agents


@pytest.mark.parametrize("name,seed", COMPOSITION_FIXTURES)
def test_gpu_composition_matches_reference(C, name, seed):
    import mxabides
    d, ref, summ = load_composition(name, seed)
    m = mxabides.VecMarket(C.from_dict(d["composition"]), [seed], trace_cap=len(ref))
    m.run()
    s = m.summary()
    assert s["status"][0] == 1, "env error %d" % s["err"][0]
    assert first_mismatch(m.trace(0), ref) == -1
    assert int(s["events"][0]) == d["events"]
    assert "%016x" % int(s["hash"][0]) == d["hash"]
    assert m.book(0, 0) == d["bids"] and m.book(0, 1) == d["asks"]
    assert int(s["order_counter"][0]) - 1 == d["order_id_counter"]
    holdings, means = m.report(0)
    assert holdings == d["final_holdings_lines"]
    assert means == d["mean_lines"]


@pytest.mark.parametrize("name", composition_names())
def test_gpu_composition_batch_equals_oracle(C, name):
    """256 seeds per composition, each env bit-exact with the oracle (events, FNV hash, errors)"""
    import mxabides
    cfg = _composition(C, name)
    seeds = (np.arange(256, dtype=np.int64) * 7919 + 3) & 0xFFFFFFFF
    m = mxabides.VecMarket(cfg, seeds)
    m.run()
    s = m.summary()
    ev, hs, er, _ = pyoracle.run_batch_config(cfg, seeds.astype(np.uint32), threads=16)
    assert (er == 0).all() and (s["status"] == 1).all()
    assert (s["events"] == ev).all()
    assert (s["hash"] == hs).all()


@pytest.mark.parametrize("name", ["rmsc03_alt", "sparse_zi_alt"])
def test_gpu_composition_chunked_launches_and_exchange_log(C, name, tmp_path):
    """a composition's handle is an ordinary Kernel.runner handle: 997-pop launches equal one
    launch, and its book-update stream with the exchange log on is the oracle's record for record;
    the written run directory names the agents as the base script does"""
    import mxabides
    cfg = _composition(C, name)
    seeds = [123456789, 7, 99]
    one = mxabides.VecMarket(cfg, seeds, book_log=1 << 20, exchange_log=True)
    one.run()
    many = mxabides.VecMarket(cfg, seeds)
    many.run(chunk=997)
    s1, s2 = one.summary(), many.summary()
    for k in ("events", "hash", "current_time", "order_counter", "status"):
        assert (s1[k] == s2[k]).all(), k
    for i, sd in enumerate(seeds):
        o = pyoracle.OracleEnv(cfg, sd)
        o.set_book_log()
        o.set_exchange_log()
        o.run()
        a = o.book_records()
        d = one.book_log_records(i)
        assert len(d) == len(a)
        assert (d["t"] == a[:, 0]).all() and (d["price"] == a[:, 1]).all() and (d["qty"] == a[:, 2]).all()
    one.write_logs(0, str(tmp_path))
    names, types = C.agent_names(cfg), C.agent_type_names(cfg)
    assert (tmp_path / ("%s.bz2" % names[0].replace(" ", ""))).exists()  # the exchange's own log
    assert (tmp_path / "summary_log.bz2").exists()
    rows = one.summary_log(0)
    assert rows and all(r["AgentStrategy"] == types[r["AgentID"]] for r in rows)
