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
