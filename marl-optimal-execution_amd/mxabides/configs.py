"""Agent naming of the reference configs (used for the reference-format stdout report).

config/rmsc03.py:95-197, config/sparse_zi_100.py:177-256, config/sparse_zi_1000.py,
config/value_noise.py:98-161 (every ValueAgent gets its own type string "ValueAgent {id}"),
config/rmsc01.py:75-211 and config/rmsc02.py (the same agents), config/obi_rmsc02.py,
config/random_fund_value.py:113-153, config/random_fund_diverse.py:116-198,
config/hist_fund_value.py:84-148, config/hist_fund_diverse.py:86-190 (the same agents).
"""
import numpy as np

ZI_GROUPS = [(0, 250, "1"), (0, 500, "1"), (0, 1000, "0.8"), (0, 1000, "1"), (0, 2000, "0.8"), (250, 500, "0.8"),
             (250, 500, "1")]
ZI_COUNTS = {"sparse_zi_100": [15, 15, 14, 14, 14, 14, 14], "sparse_zi_1000": [143] * 6 + [142]}


# configs whose script takes the ticker from -t/--ticker (config/rmsc03.py:31, random_fund_*.py,
# hist_fund_*.py); the default is the one the fixtures and the bench use
TICKER_CONFIGS = ("rmsc03", "rmsc03_sbmm", "rmsc03_sbmm_poll", "random_fund_value", "random_fund_diverse", "hist_fund_value", "hist_fund_diverse",
                  "marketreplay_runner", "marketreplay_twap", "marketreplay_twap_e")
HIST_CONFIGS = ("hist_fund_value", "hist_fund_diverse")
# config/marketreplay.py (a LOBSTER tape, no oracle) and config/execution/marketreplay/
# execution_marketreplay.py (the same plus TWAP_EXECUTION_AGENT; _e: its -e flag, the agent trades)
REPLAY_CONFIGS = ("marketreplay_runner", "marketreplay_twap", "marketreplay_twap_e")


def symbol_of(config, symbol=None, tape=None):
    """the ticker of a configuration's outputs: the caller's -t for the configs that take one; a
    replay config's default is its tape's ticker (a replay has no default of its own)"""
    if symbol is not None:
        if config not in TICKER_CONFIGS:
            raise ValueError("%s has a fixed symbol (JPM); only %s take -t/--ticker" % (config, TICKER_CONFIGS))
        return symbol
    if config in HIST_CONFIGS:
        return "JPM"
    if config in REPLAY_CONFIGS:
        sym = getattr(tape, "symbol", None)
        if not sym:
            raise ValueError("%s: the tape carries no ticker; pass symbol=" % config)
        return sym
    return "ABM" if config in TICKER_CONFIGS else "JPM"


# ExchangeAgent(book_freq=...) of each config script: 0 archives every snapshot
# (ORDERBOOK_<sym>_FULL), None archives nothing, a pandas frequency resamples
# (ExchangeAgent.py:389-469; value_noise / sparse_zi_* take -b, default None)
BOOK_FREQ = {"rmsc03": 0, "rmsc03_sbmm": 0, "rmsc03_sbmm_poll": 0, "rmsc02": 0, "rmsc01": "M", "obi_rmsc02": "all", "random_fund_value": None,
             "random_fund_diverse": None, "hist_fund_value": None, "hist_fund_diverse": None, "value_noise": None,
             "sparse_zi_100": None, "sparse_zi_1000": None, "marketreplay_runner": 0,
             "marketreplay_twap": 0, "marketreplay_twap_e": 0}


def agent_names(config):
    if config == "marketreplay_runner":  # config/marketreplay.py:66-110
        return ["EXCHANGE_AGENT", "MARKET_REPLAY_AGENT"]
    if config in ("marketreplay_twap", "marketreplay_twap_e"):  # execution_marketreplay.py:66-140
        return ["EXCHANGE_AGENT", "MARKET_REPLAY_AGENT", "TWAP_EXECUTION_AGENT"]
    if config == "obi_rmsc02":
        return (["EXCHANGE_AGENT", "MARKET_MAKER_AGENT_1"] + ["ZI_AGENT_%d" % j for j in range(2, 91)] +
                ["OBI_AGENT_%d" % j for j in range(91, 96)] + ["MOMENTUM_AGENT_%d" % j for j in range(96, 101)])
    if config in ("rmsc01", "rmsc02"):
        return (["EXCHANGE_AGENT", "MARKET_MAKER_AGENT_1"] + ["ZI_AGENT_%d" % j for j in range(2, 52)] +
                ["HBL_AGENT_%d" % j for j in range(52, 77)] + ["MOMENTUM_AGENT_%d" % j for j in range(77, 101)])
    if config == "value_noise":
        return (["Exchange Agent 0"] + ["NoiseAgent %d" % j for j in range(1, 101)] +
                ["Value Agent %d" % j for j in range(101, 151)])
    if config in ("random_fund_value", "random_fund_diverse", "hist_fund_value", "hist_fund_diverse"):
        extra = ["MARKET_MAKER_AGENT_5101"] + ["MOMENTUM_AGENT_%d" % j for j in range(5102, 5127)]
        return (["EXCHANGE_AGENT"] + ["NoiseAgent %d" % j for j in range(1, 5001)] +
                ["Value Agent %d" % j for j in range(5001, 5101)] + (extra if config.endswith("diverse") else []))
    if config in ("rmsc03", "rmsc03_sbmm", "rmsc03_sbmm_poll"):
        mm = "POV_MARKET_MAKER_AGENT_61" if config == "rmsc03" else "SPREAD_BASED_MARKET_MAKER_AGENT_61"
        return (["EXCHANGE_AGENT"] + ["NoiseAgent %d" % j for j in range(1, 51)] +
                ["Value Agent %d" % j for j in range(51, 61)] + [mm] +
                ["MOMENTUM_AGENT_%d" % j for j in (62, 63)])
    names, a = ["Exchange Agent 0"], 1
    for g, cnt in enumerate(ZI_COUNTS[config]):
        lo, hi, eta = ZI_GROUPS[g]
        for _ in range(cnt):
            names.append("ZI Agent %d Type %d [%d <= R <= %d, eta=%s]" % (a, g + 1, lo, hi, eta))
            a += 1
    return names


def agent_type_names(config):
    if config == "marketreplay_runner":
        return ["ExchangeAgent", "MarketReplayAgent"]
    if config in ("marketreplay_twap", "marketreplay_twap_e"):
        return ["ExchangeAgent", "MarketReplayAgent", "ExecutionAgent"]
    if config == "obi_rmsc02":
        return (["ExchangeAgent", "MarketMakerAgent"] + ["ZeroIntelligenceAgent"] * 89 +
                ["OrderBookImbalanceAgent"] * 5 + ["MomentumAgent"] * 5)
    if config in ("rmsc01", "rmsc02"):
        return (["ExchangeAgent", "MarketMakerAgent"] + ["ZeroIntelligenceAgent"] * 50 +
                ["HeuristicBeliefLearningAgent"] * 25 + ["MomentumAgent"] * 24)
    if config == "value_noise":
        return ["ExchangeAgent"] + ["NoiseAgent"] * 100 + ["ValueAgent %d" % j for j in range(101, 151)]
    if config in ("random_fund_value", "random_fund_diverse", "hist_fund_value", "hist_fund_diverse"):
        extra = ["MarketMakerAgent"] + ["MomentumAgent"] * 25 if config.endswith("diverse") else []
        return ["ExchangeAgent"] + ["NoiseAgent"] * 5000 + ["ValueAgent"] * 100 + extra
    if config in ("rmsc03", "rmsc03_sbmm", "rmsc03_sbmm_poll"):
        mm = "POVMarketMakerAgent" if config == "rmsc03" else "SpreadBasedMarketMakerAgent"
        return ["ExchangeAgent"] + ["NoiseAgent"] * 50 + ["ValueAgent"] * 10 + [mm] + ["MomentumAgent"] * 2
    out = ["ExchangeAgent"]
    for g, cnt in enumerate(ZI_COUNTS[config]):
        lo, hi, eta = ZI_GROUPS[g]
        out += ["ZeroIntelligenceAgent Type %d [%d <= R <= %d, eta=%s]" % (g + 1, lo, hi, eta)] * cnt
    return out


# include/mxa.h mxa_mm_params: config/rmsc03.py's market-maker options (config/rmsc03.py:39-43)
MM_PARAMS_DTYPE = np.dtype([("mm_pov", "<f8"), ("mm_min_order_size", "<i4"), ("mm_window_size", "<i4"),
                            ("mm_num_ticks", "<i4"), ("pad", "<i4"), ("mm_wake_up_freq_ns", "<i8")])
MM_DEFAULTS = {"pov": 0.05, "min_order_size": 20, "window_size": 5, "num_ticks": 20, "wake_up_freq": "1S"}


def _timedelta_ns(x):
    """pd.Timedelta(wake_up_freq).value, as getWakeFrequency and the transacted-volume lookback
    read the option (POVMarketMakerAgent.py:203-206, OrderBook.py:400-436)"""
    if isinstance(x, str):
        import pandas as pd
        return int(pd.Timedelta(x).value)
    return int(x)


def mm_params(n=1, pov=0.05, min_order_size=20, window_size=5, num_ticks=20, wake_up_freq="1S"):
    """[n] MM_PARAMS_DTYPE records of `python abides.py -c rmsc03 --mm-pov POV --mm-min-order-size
    MIN_ORDER_SIZE --mm-window-size WINDOW_SIZE --mm-num-ticks NUM_TICKS --mm-wake-up-freq
    WAKE_UP_FREQ`; each option a scalar or one value per env (a parameter sweep in one batch,
    scripts/rmsc03.sh).  wake_up_freq: a pandas frequency string ("10S") or ns."""
    out = np.zeros(n, dtype=MM_PARAMS_DTYPE)
    out["mm_pov"] = pov
    out["mm_min_order_size"] = min_order_size
    out["mm_window_size"] = window_size
    out["mm_num_ticks"] = num_ticks
    wf = wake_up_freq if isinstance(wake_up_freq, (list, tuple, np.ndarray)) else [wake_up_freq] * n
    if len(wf) != n:
        raise ValueError("wake_up_freq: one value or one per env")
    out["mm_wake_up_freq_ns"] = [_timedelta_ns(x) for x in wf]
    return out
