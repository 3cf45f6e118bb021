#!/usr/bin/env python3
"""Golden fixtures of runtime compositions (include/mxa.h mxa_config).

CONTAINER-ONLY TEST INFRASTRUCTURE (see gen_fixtures.py).  Each composition is an agent list
built from the reference's own classes the way its base script builds its own list, with other
counts and parameters, and run by the reference's Kernel.runner:
  * base rmsc03:        config/rmsc03.py:55-235 (oracle symbol dict, exchange, NoiseAgent with
                        util.get_wake_time, ValueAgent, POVMarketMakerAgent, MomentumAgent, the
                        kernel; zero latency, noise [0.0]);
  * base value_noise:   config/value_noise.py:80-290 (the kernel before the agents, NoiseAgent
                        waking at open + rand() * (close - open), ValueAgent with its default cash,
                        the symmetric latency matrix, 6-way noise);
  * base sparse_zi_100: config/sparse_zi_100.py:140-334 (latency RandomState, the ZI strategy
                        table, the cubic LatencyModel); sparse_zi_1000: its matrix latency.
Every global draw happens in the script's order, keyword arguments in the script's order (their
evaluation order is the draw order).  The recording (trace, hash, final state, summary log) is
gen_fixtures.run_config's.  The composition's every field is stored in the fixture JSON, so a
test builds the same MarketConfig from the fixture alone.

Usage: python tests/golden/gen_config_fixtures.py [NAME ...]   (default: all of COMPOSITIONS)
       python tests/golden/gen_config_fixtures.py run NAME SEED OUT [--full]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)

# name -> (base, overrides of the base script's values, seeds, full trace?)
COMPOSITIONS = {
    # BASELINE's "~100 background agents": rmsc03 with 100 noise and 20 value agents
    "rmsc03_n100_v20": ("rmsc03", {"n_noise": 100, "n_value": 20}, [123456789, 7], True),
    # rmsc03's classes with other parameters and session: a 10-tick market maker at pov 0.1 every
    # 2 s, 5 momentum agents (1-20 shares, 30 s), value agents with another arrival rate and r_bar
    # belief, market 09:30-10:00, kernel to 10:01
    "rmsc03_alt": ("rmsc03", {"n_noise": 80, "n_value": 15, "n_momentum": 5, "mom_min_size": 1, "mom_max_size": 20,
                              "mom_wake_up_freq_ns": 30 * 10**9, "mkt_close_ns": 10 * 3600 * 10**9,
                              "kernel_stop_ns": 10 * 3600 * 10**9 + 60 * 10**9, "value_lambda_a": 1e-10,
                              "value_sigma_n": 5e3, "r_bar": 1.2e5, "value_r_bar": 1.2e5,
                              "mm": {"mm_pov": 0.1, "mm_min_order_size": 30, "mm_window_size": 3,
                                     "mm_num_ticks": 10, "mm_wake_up_freq_ns": 2 * 10**9}},
                   [123456789, 11], False),
    # sparse_zi_100 with another strategy table (60 agents, four groups) and q_max 6
    "sparse_zi_alt": ("sparse_zi_100", {"zi_table": [(20, 0, 100, 1), (20, 100, 400, 0.9), (10, 0, 1500, 0.75),
                                                     (10, 300, 600, 1)], "zi_q_max": 6},
                      [123456789, 7], True),
    # sparse_zi_1000's matrix latency at 200 agents (two groups)
    "sparse_zi_matrix_200": ("sparse_zi_1000", {"zi_table": [(120, 0, 500, 1), (79, 100, 1000, 0.8)]},
                             [123456789], False),
    # value_noise with 60 noise and 30 value agents, market 09:30-10:00, 0.5 s compute delays
    "value_noise_alt": ("value_noise", {"n_noise": 60, "n_value": 30, "mkt_close_ns": 10 * 3600 * 10**9,
                                        "default_computation_delay_ns": 500000000},
                        [123456789, 7], True),
}


def full_composition(base, over):
    """the base script's composition (oracle/pyoracle.config_defaults, pinned against the device's
    mxa_config_defaults by tests/test_composition.py) with the overrides, as a plain dict"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    c = pyoracle.config_defaults(base)
    d = {}
    for k, _ in c._fields_:
        v = getattr(c, k)
        if k == "mm":
            d[k] = {n: getattr(v, n) for n, _ in v._fields_}
        elif k in ("zi_count", "zi_r_min", "zi_r_max", "zi_eta"):
            d[k] = list(v)
        else:
            d[k] = v
    for k, v in over.items():
        if k == "zi_table":
            d["n_zi_groups"] = len(v)
            d["zi_count"] = [int(r[0]) for r in v] + [0] * (8 - len(v))
            d["zi_r_min"] = [int(r[1]) for r in v] + [0] * (8 - len(v))
            d["zi_r_max"] = [int(r[2]) for r in v] + [0] * (8 - len(v))
            d["zi_eta"] = [float(r[3]) for r in v] + [0.0] * (8 - len(v))
            d["zi_table_literal"] = [list(r) for r in v]  # the script's tuples (ints stay ints)
        elif k == "mm":
            d["mm"].update(v)
        else:
            d[k] = v
    d["base_name"] = base
    return d


def _freq(ns):
    """a pandas frequency string for ns, as the scripts write theirs ("1S", "20s")"""
    return "%ds" % (ns // 10**9) if ns % 10**9 == 0 else "%dns" % ns


def script(c, seed):
    """the composition's config script body: builds the agents and calls Kernel.runner"""
    import pandas as pd
    from agent.ExchangeAgent import ExchangeAgent
    from Kernel import Kernel
    from util import util
    from util.oracle.SparseMeanRevertingOracle import SparseMeanRevertingOracle
    from util.order import LimitOrder

    np.random.seed(seed)
    util.silent_mode = True
    LimitOrder.silent_mode = True
    midnight = pd.Timestamp(int(c["date_ns"]), unit="ns")
    T = lambda ns: midnight + pd.to_timedelta(int(ns), unit="ns")  # noqa: E731
    rs = lambda: np.random.RandomState(seed=np.random.randint(low=0, high=2 ** 32, dtype="uint64"))  # noqa: E731
    base = c["base_name"]
    mkt_open, mkt_close = T(c["mkt_open_ns"]), T(c["mkt_close_ns"])

    def sym_dict(agent_kappa):
        return {"r_bar": c["r_bar"], "kappa": c["kappa"], "agent_kappa": agent_kappa, "sigma_s": 0,
                "fund_vol": c["fund_vol"], "megashock_lambda_a": c["megashock_lambda_a"],
                "megashock_mean": c["megashock_mean"], "megashock_var": c["megashock_var"], "random_state": rs()}

    if base == "rmsc03":  # config/rmsc03.py:55-235
        from agent.examples.MomentumAgent import MomentumAgent
        from agent.market_makers.POVMarketMakerAgent import POVMarketMakerAgent
        from agent.NoiseAgent import NoiseAgent
        from agent.ValueAgent import ValueAgent
        symbol = "ABM"
        symbols = {symbol: sym_dict(c["value_kappa"])}
        oracle = SparseMeanRevertingOracle(mkt_open, mkt_close, symbols)
        agents = [ExchangeAgent(id=0, name="EXCHANGE_AGENT", type="ExchangeAgent", mkt_open=mkt_open,
                                mkt_close=mkt_close, symbols=[symbol], log_orders=bool(c["log_orders"]),
                                pipeline_delay=0, computation_delay=0, stream_history=10, book_freq=0,
                                wide_book=False, random_state=rs())]
        n = 1
        noise_open, noise_close = T(c["noise_wake_open_ns"]), T(c["noise_wake_close_ns"])
        agents += [NoiseAgent(id=j, name="NoiseAgent {}".format(j), type="NoiseAgent", symbol=symbol,
                              starting_cash=c["starting_cash"], wakeup_time=util.get_wake_time(noise_open, noise_close),
                              log_orders=False, random_state=rs()) for j in range(n, n + c["n_noise"])]
        n += c["n_noise"]
        agents += [ValueAgent(id=j, name="Value Agent {}".format(j), type="ValueAgent", symbol=symbol,
                              starting_cash=c["value_starting_cash"], sigma_n=c["value_sigma_n"],
                              r_bar=c["value_r_bar"], kappa=c["value_kappa"], sigma_s=c["value_sigma_s"],
                              lambda_a=c["value_lambda_a"], random_state=rs()) for j in range(n, n + c["n_value"])]
        n += c["n_value"]
        m = c["mm"]
        agents += [POVMarketMakerAgent(id=j, name="POV_MARKET_MAKER_AGENT_{}".format(j), type="POVMarketMakerAgent",
                                       symbol=symbol, starting_cash=c["starting_cash"], pov=m["mm_pov"],
                                       min_order_size=m["mm_min_order_size"], window_size=m["mm_window_size"],
                                       num_ticks=m["mm_num_ticks"], wake_up_freq=_freq(m["mm_wake_up_freq_ns"]),
                                       log_orders=False, random_state=rs()) for j in range(n, n + c["n_mm"])]
        n += c["n_mm"]
        agents += [MomentumAgent(id=j, name="MOMENTUM_AGENT_{}".format(j), type="MomentumAgent", symbol=symbol,
                                 starting_cash=c["starting_cash"], min_size=c["mom_min_size"],
                                 max_size=c["mom_max_size"], wake_up_freq=_freq(c["mom_wake_up_freq_ns"]),
                                 log_orders=False, random_state=rs()) for j in range(n, n + c["n_momentum"])]
        n += c["n_momentum"]
        kernel = Kernel("Market Replay Kernel", random_state=rs())
        kernel.runner(agents=agents, startTime=T(c["kernel_start_ns"]), stopTime=T(c["kernel_stop_ns"]),
                      agentLatency=np.zeros((n, n)), latencyNoise=[0.0],
                      defaultComputationDelay=c["default_computation_delay_ns"], defaultLatency=0, oracle=oracle,
                      log_dir=None)
        return
    symbol = "JPM"
    if base == "value_noise":  # config/value_noise.py:80-290
        from agent.NoiseAgent import NoiseAgent
        from agent.ValueAgent import ValueAgent
        symbols = {symbol: sym_dict(c["value_kappa"])}
        kernel = Kernel("Base Kernel", random_state=rs())
        oracle = SparseMeanRevertingOracle(mkt_open, mkt_close, symbols)
        log_orders = bool(c["log_orders"])
        agents = [ExchangeAgent(0, "Exchange Agent 0", "ExchangeAgent", mkt_open, mkt_close, [symbol],
                                log_orders=log_orders, book_freq=None, pipeline_delay=0, computation_delay=0,
                                stream_history=10, random_state=rs())]
        n = 1
        agents += [NoiseAgent(j, "NoiseAgent {}".format(j), "NoiseAgent", random_state=rs(), log_orders=log_orders,
                              symbol=symbol, starting_cash=c["starting_cash"],
                              wakeup_time=mkt_open + np.random.rand() * (mkt_close - mkt_open))
                   for j in range(n, n + c["n_noise"])]
        n += c["n_noise"]
        # the script leaves ValueAgent's starting_cash at its default (100000, value_starting_cash)
        assert c["value_starting_cash"] == 100000
        agents += [ValueAgent(j, "Value Agent {}".format(j), "ValueAgent {}".format(j), random_state=rs(),
                              log_orders=log_orders, symbol=symbol, sigma_n=c["value_sigma_n"],
                              r_bar=c["value_r_bar"], kappa=c["value_kappa"], sigma_s=c["value_sigma_s"],
                              lambda_a=c["value_lambda_a"]) for j in range(n, n + c["n_value"])]
        n += c["n_value"]
        latency = np.random.uniform(low=c["lat_low"], high=c["lat_high"], size=(n, n))
        for i in range(n):  # the script's symmetric fill (no ZeroIntelligenceAgent pairs here)
            for j in range(n):
                if i > j:
                    latency[i, j] = latency[j, i]
                elif i == j:
                    latency[i, j] = 20000
        kernel.runner(agents=agents, startTime=T(c["kernel_start_ns"]), stopTime=T(c["kernel_stop_ns"]),
                      agentLatency=latency, latencyNoise=[0.25, 0.25, 0.20, 0.15, 0.10, 0.05],
                      defaultComputationDelay=c["default_computation_delay_ns"], oracle=oracle, log_dir=None)
        return
    # config/sparse_zi_100.py:140-334 (sparse_zi_1000.py: no latency RandomState, the matrix)
    from agent.ZeroIntelligenceAgent import ZeroIntelligenceAgent
    big = base == "sparse_zi_1000"
    symbols = {symbol: sym_dict(c["zi_kappa"])}
    kernel = Kernel("Base Kernel", random_state=rs())
    if not big:
        latency_rstate = np.random.RandomState(seed=np.random.randint(low=0, high=2 ** 32))
    oracle = SparseMeanRevertingOracle(mkt_open, mkt_close, symbols)
    agents = [ExchangeAgent(0, "Exchange Agent 0", "ExchangeAgent", mkt_open, mkt_close, [symbol],
                            log_orders=bool(c["log_orders"]), book_freq=None, pipeline_delay=0, computation_delay=0,
                            stream_history=10, random_state=rs())]
    agent_types = ["ExchangeAgent"]
    n = 1
    for i, x in enumerate(c["zi_table_literal"]):
        strat_name = "Type {} [{} <= R <= {}, eta={}]".format(i + 1, x[1], x[2], x[3])
        agents += [ZeroIntelligenceAgent(j, "ZI Agent {} {}".format(j, strat_name),
                                         "ZeroIntelligenceAgent {}".format(strat_name), random_state=rs(),
                                         log_orders=False, symbol=symbol, starting_cash=c["starting_cash"],
                                         sigma_n=c["zi_sigma_n"], r_bar=c["zi_r_bar"], kappa=c["zi_kappa"],
                                         sigma_s=c["zi_sigma_s"], q_max=c["zi_q_max"], sigma_pv=c["zi_sigma_pv"],
                                         R_min=x[1], R_max=x[2], eta=x[3], lambda_a=c["zi_lambda_a"])
                   for j in range(n, n + x[0])]
        agent_types += ["ZeroIntelligenceAgent {}".format(strat_name)] * x[0]
        n += x[0]
    if not big:
        from model.LatencyModel import LatencyModel
        model_args = {"connected": True,
                      "min_latency": np.random.uniform(low=c["lat_low"], high=c["lat_high"], size=(n, n)),
                      "jitter": 0.3, "jitter_clip": 0.05, "jitter_unit": 5}
        latency_model = LatencyModel(latency_model="cubic", random_state=latency_rstate, kwargs=model_args)
        kernel.runner(agents=agents, startTime=T(c["kernel_start_ns"]), stopTime=T(c["kernel_stop_ns"]),
                      agentLatencyModel=latency_model, agentLatency=None, latencyNoise=None,
                      defaultComputationDelay=c["default_computation_delay_ns"], oracle=oracle, log_dir=None)
        return
    latency = np.random.uniform(low=c["lat_low"], high=c["lat_high"], size=(n, n))
    for i in range(n):
        for j in range(n):
            if i > j:
                latency[i, j] = latency[j, i]
            elif i == j:
                latency[i, j] = 20000
    kernel.runner(agents=agents, startTime=T(c["kernel_start_ns"]), stopTime=T(c["kernel_stop_ns"]),
                  agentLatency=latency, latencyNoise=[0.25, 0.25, 0.20, 0.15, 0.10, 0.05],
                  defaultComputationDelay=c["default_computation_delay_ns"], oracle=oracle, log_dir=None)


def run_one(name, seed, out, full):
    import gen_fixtures as G
    base, over, _, _ = COMPOSITIONS[name]
    c = full_composition(base, over)
    date = str(np.datetime64(int(c["date_ns"]), "ns").astype("datetime64[D]"))
    G.run_config(name, seed, out, full, composition={"date": date, "script": lambda: script(c, seed)})
    with open(out + ".json") as f:  # the fixture carries its composition
        final = json.load(f)
    final["composition"] = c
    with open(out + ".json", "w") as f:
        json.dump(final, f, indent=0)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run_one(sys.argv[2], int(sys.argv[3]), sys.argv[4], "--full" in sys.argv)
        return
    names = sys.argv[1:] or list(COMPOSITIONS)
    procs = []
    for name in names:
        for seed in COMPOSITIONS[name][2]:
            out = os.path.join(HERE, "cfg_%s_%d" % (name, seed))
            cmd = [sys.executable, os.path.abspath(__file__), "run", name, str(seed), out] + \
                (["--full"] if COMPOSITIONS[name][3] else [])
            procs.append((name, seed, subprocess.Popen(cmd, cwd=tempfile.mkdtemp(prefix="gc_"),
                                                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))))
    for name, seed, p in procs:
        print(name, seed, "rc", p.wait())


if __name__ == "__main__":
    main()
