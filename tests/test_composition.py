"""Runtime compositions (include/mxa.h mxa_config) on the CPU: the oracle against
reference runs of compositions built from the reference's classes (tests/golden/gen_config_fixtures.py),
the device's and the oracle's base-script defaults against each other, and the C-ABI's checks.
No GPU: mxa_config_defaults / _key / _info / the validation are host functions."""
import ctypes

import numpy as np
import pytest

import pyoracle
from golden_util import COMPOSITION_FIXTURES, first_mismatch, load_composition


@pytest.fixture(scope="module")
def C():
    from mxabides import composition
    return composition


@pytest.mark.parametrize("base", ["rmsc03", "value_noise", "sparse_zi_100", "sparse_zi_1000"])
def test_device_and_oracle_defaults_agree(C, base):
    """mxa_config_defaults (mxa_config.h config_defaults, from the device's constexpr parameters)
    and ora_config_defaults restate the same script: the same bytes"""
    assert ctypes.sizeof(C.MarketConfig) == ctypes.sizeof(pyoracle.OraConfig)
    assert bytes(C.defaults(base)) == bytes(pyoracle.config_defaults(base))


def test_exchange_log_orders_agree_for_every_config():
    """the device's ExchangeAgent log_orders (mxa_config_info) and the oracle's list agree for every
    configuration (rmsc03_rl disagreed)"""
    from mxabides import _lib
    L = _lib.load()
    names = dict(_lib.CONFIG_IDS)
    names.update({"rmsc03_rl": _lib.MXA_RMSC03_RL, "marketreplay": _lib.MXA_MARKETREPLAY})
    for name, cid in names.items():
        out = np.zeros(8, dtype=np.int64)
        assert L.mxa_config_info(cid, out.ctypes.data) == 0
        if name == "marketreplay_twap_e":
            name = "marketreplay_twap"
        assert out[1] == pyoracle.config_log_orders(name), name


@pytest.mark.parametrize("name,seed", COMPOSITION_FIXTURES)
def test_oracle_composition_matches_reference(C, name, seed):
    d, ref, summ = load_composition(name, seed)
    cfg = C.from_dict(d["composition"])
    assert bytes(cfg) == bytes(pyoracle.as_config(cfg))
    e = pyoracle.OracleEnv(cfg, seed, trace_cap=len(ref))
    e.run()
    assert e.error[0] == 0, e.error
    assert first_mismatch(e.trace(), ref) == -1
    assert e.events == d["events"]
    assert "%016x" % e.hash == d["hash"]
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    assert e.order_counter - 1 == d["order_id_counter"]
    assert e.last_trade == d["last_trade"]
    e.finish()
    rep = e.report()
    assert [l for l in rep if l.startswith("Final holdings")] == d["final_holdings_lines"]
    assert [l for l in rep if not l.startswith("Final holdings")] == d["mean_lines"]


def test_composition_names_follow_the_scripts(C):
    """agent names of a composition as its base script names them (reports, EXCHANGE_AGENT.bz2)"""
    d, _, _ = load_composition("sparse_zi_alt", 7)
    cfg = C.from_dict(d["composition"])
    names = C.agent_names(cfg)
    assert len(names) == cfg.n_agents == 61
    assert names[1] == "ZI Agent 1 Type 1 [0 <= R <= 100, eta=1]"
    assert names[21] == "ZI Agent 21 Type 2 [100 <= R <= 400, eta=0.9]"
    assert names[41] == "ZI Agent 41 Type 3 [0 <= R <= 1500, eta=0.75]"
    c = C.make("rmsc03", n_noise=3, n_value=2, n_momentum=1)
    assert C.agent_names(c) == ["EXCHANGE_AGENT", "NoiseAgent 1", "NoiseAgent 2", "NoiseAgent 3", "Value Agent 4",
                                "Value Agent 5", "POV_MARKET_MAKER_AGENT_6", "MOMENTUM_AGENT_7"]


def test_key_ignores_the_date_only(C):
    a = C.defaults("rmsc03")
    b = C.defaults("rmsc03")
    b.date_ns += 86400 * 10**9
    assert C.key(a) == C.key(b)
    b.n_noise += 1
    assert C.key(a) != C.key(b)


@pytest.mark.parametrize("change,msg", [
    (dict(n_mm=2), "at most one POVMarketMakerAgent"),
    (dict(n_noise=-1), "negative count"),
    (dict(n_noise=9000), "8191 agents"),
    (dict(mkt_close_ns=0), "session"),
    (dict(zi_table=[(5, 0, 100, 1)]), "ZI groups belong"),
    (dict(mom_min_size=10, mom_max_size=10), "momentum options"),
    (dict(mm={"mm_num_ticks": 61}), "market maker options"),
    (dict(base=3), "base must be"),
])
def test_invalid_compositions_are_refused_before_any_compile(C, change, msg):
    from mxabides import _lib
    c = C.make("rmsc03", **{k: v for k, v in change.items() if k not in ("zi_table", "mm")},
               zi_table=change.get("zi_table"), mm=change.get("mm"))
    with pytest.raises(_lib.MxaError, match=msg):
        C.compile(c, cache_dir="/nonexistent/never/written")


def test_zi_composition_bounds(C):
    from mxabides import _lib
    c = C.make("sparse_zi_100", zi_q_max=11)
    with pytest.raises(_lib.MxaError, match="zi_q_max"):
        C.compile(c, cache_dir="/nonexistent/never/written")
    c = C.make("sparse_zi_100", n_noise=1)
    with pytest.raises(_lib.MxaError, match="ZI agents only"):
        C.compile(c, cache_dir="/nonexistent/never/written")


def test_test_compositions_are_prebuilt():
    """__graft_entry__.build() compiled every composition the GPU tests run (they never compile)"""
    import os

    import __graft_entry__ as g
    from mxabides import composition as C
    for c in g.compositions():
        path = os.path.join(os.path.dirname(C._lib.LIB_PATH), "custom", "libmxa_cfg_%s.so" % C.key(c))
        assert os.path.exists(path), path
