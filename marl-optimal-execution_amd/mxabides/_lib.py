"""ctypes binding of libmxa (include/mxa.h).

The product path is the HIP library only: if lib/libmxa.so is missing or cannot be
loaded this module raises — there is deliberately no CPU fallback.
"""
import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MXA_LIB") or os.path.join(PKG_ROOT, "lib", "libmxa.so")

MXA_RMSC03, MXA_SPARSE_ZI_100, MXA_SPARSE_ZI_1000, MXA_MARKETREPLAY, MXA_RMSC03_RL, MXA_VALUE_NOISE = 0, 1, 2, 3, 4, 5
MXA_RMSC01 = 6
MXA_RMSC02 = 7
MXA_OBI_RMSC02 = 8
MXA_RANDOM_FUND_VALUE = 9
MXA_RANDOM_FUND_DIVERSE = 10
MXA_HIST_FUND_VALUE = 11
MXA_HIST_FUND_DIVERSE = 12
MXA_MARKETREPLAY_RUNNER = 13
MXA_MARKETREPLAY_TWAP = 14
MXA_RMSC03_SBMM = 15
MXA_RMSC03_SBMM_POLL = 16
MXA_RMSC03_MM = 17  # config/rmsc03.py with per-env --mm-* options (mxa_create_params)
CONFIG_IDS = {"rmsc03": MXA_RMSC03, "sparse_zi_100": MXA_SPARSE_ZI_100, "sparse_zi_1000": MXA_SPARSE_ZI_1000,
              "value_noise": MXA_VALUE_NOISE, "rmsc01": MXA_RMSC01, "rmsc02": MXA_RMSC02,
              "obi_rmsc02": MXA_OBI_RMSC02, "random_fund_value": MXA_RANDOM_FUND_VALUE,
              "random_fund_diverse": MXA_RANDOM_FUND_DIVERSE, "hist_fund_value": MXA_HIST_FUND_VALUE,
              "hist_fund_diverse": MXA_HIST_FUND_DIVERSE,
              # config/marketreplay.py (Kernel.runner; ABIDESEnv's GymKernel replay is mxabides.gym)
              "marketreplay_runner": MXA_MARKETREPLAY_RUNNER,
              # config/execution/marketreplay/execution_marketreplay.py (TWAP agent passive / -e)
              "marketreplay_twap": MXA_MARKETREPLAY_TWAP, "marketreplay_twap_e": MXA_MARKETREPLAY_TWAP,
              # rmsc03 with a SpreadBasedMarketMakerAgent in the market maker's slot (subscribe / polling)
              "rmsc03_sbmm": MXA_RMSC03_SBMM, "rmsc03_sbmm_poll": MXA_RMSC03_SBMM_POLL}
ENV_RUNNING, ENV_DONE, ENV_ERROR = 0, 1, 2
ERR_NAMES = {0: "none", 1: "event queue capacity", 2: "order book capacity", 3: "open-order list capacity",
             4: "transaction history capacity", 5: "get_transacted_volume without transactions (pandas error)",
             6: "setWakeup in the past", 7: "ZI theta index (IndexError)", 8: "bad config",
             9: "RNG look-ahead overrun", 10: "price outside the replay ladder", 11: "book entry pool capacity",
             12: "agent order-id capacity", 13: "MarketReplayAgent KeyError (no tape group at wake time)",
             14: "get_observation/get_reward on missing or None data", 15: "kernelStopping with trade on (TypeError)",
             16: "modify changing price or side",
             17: "HBL order stream outside the history window / device ring (MXA_OH_CAP)",
             18: "HBL streamed price range beyond the device histogram (MXA_HBL_RANGE)",
             19: "limit price the reference would carry as a python float (not restated)",
             20: "book-update log full (raise the book_log capacity)",
             21: "market data published before the book's first change (the reference's TypeError)",
             22: "more market-data subscriptions than the device table",
             23: "cancelled a market-data subscription that does not exist (KeyError)",
             24: "two MARKET_DATA messages in flight to one agent (subscription freq below the latency)",
             25: "ExecutionAgent.placeOrders: schedule[Interval(t, t + 30 s)] of a 60 s TWAP schedule (KeyError)",
             26: "ExecutionAgent.placeOrders: (bid + ask) / 2 with a None side (TypeError)",
             27: "ExecutionAgent.placeOrders: placeMarketOrder at horizon[-2] (not restated)",
             28: "SpreadBasedMarketMakerAgent: mid unbound (UnboundLocalError)",
             29: "order quantity beyond the device's 32-bit order words (POVMarketMakerAgent pov x volume)"}


class EnvSummary(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("err", ctypes.c_int32), ("events", ctypes.c_int64),
                ("hash", ctypes.c_uint64), ("current_time", ctypes.c_int64), ("order_counter", ctypes.c_int64),
                ("last_trade", ctypes.c_int64), ("max_queue", ctypes.c_int32), ("max_book", ctypes.c_int32)]


class AgentState(ctypes.Structure):
    _fields_ = [("cash", ctypes.c_int64), ("shares", ctypes.c_int64), ("n_open", ctypes.c_int64),
                ("last_trade", ctypes.c_int64), ("type", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("starting_cash", ctypes.c_int64)]


class AgentFinal(ctypes.Structure):  # mxa_agent_final
    _fields_ = [("final_fundamental", ctypes.c_int64), ("valuation_int", ctypes.c_int64), ("valuation", ctypes.c_double),
                ("kind", ctypes.c_int32), ("err", ctypes.c_int32)]


EXPORTS = ["mxa_create", "mxa_reset", "mxa_launch", "mxa_sync", "mxa_run", "mxa_read_summary", "mxa_read_agents",
           "mxa_read_book", "mxa_read_trace", "mxa_n_agents", "mxa_n_envs", "mxa_env_bytes", "mxa_set_stream",
           "mxa_last_kernel_ms", "mxa_last_error", "mxa_destroy", "mxa_rng_probe", "mxa_math_probe",
           "mxa_set_seeds", "mxa_write_results", "mxa_read_raw", "mxa_layout", "mxa_create_replay", "mxa_step",
           "mxa_step_device", "mxa_finalize", "mxa_read_final", "mxa_write_rl_state", "mxa_set_parity_hash",
           "mxa_build_id", "mxa_set_book_log", "mxa_read_book_log", "mxa_write_records", "mxa_set_id_persistence",
           "mxa_read_counters", "mxa_create_hist", "mxa_create_replay_runner",
           "mxa_set_stop_time", "mxa_run_until", "mxa_create_replay_twap", "mxa_create_params", "mxa_set_mm_params",
           "mxa_mm_defaults", "mxa_resident_envs", "mxa_set_exchange_log", "mxa_config_defaults",
           "mxa_config_compile", "mxa_config_key", "mxa_create_config", "mxa_config_info",
           "mxa_step_many", "mxa_set_launch_schedule"]
COUNTER_WORDS = 34  # include/mxa.h MXA_COUNTER_WORDS
RECORD_WORDS = 12  # include/mxa.h MXA_RECORD_WORDS

_lib = None


class MxaError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MxaError("libmxa.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, U32, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double
    L.mxa_create.argtypes = [I32, I32, P, I32, I32, ctypes.POINTER(P)]
    L.mxa_reset.argtypes = [P, P]
    L.mxa_launch.argtypes = [P, I64]
    L.mxa_sync.argtypes = [P]
    L.mxa_run.argtypes = [P, I64, I32, ctypes.POINTER(I32)]
    L.mxa_read_summary.argtypes = [P, P]
    L.mxa_read_agents.argtypes = [P, I32, P, I32]
    L.mxa_read_book.argtypes = [P, I32, I32, P, I32]
    L.mxa_read_trace.argtypes = [P, I32, P, I64, ctypes.POINTER(I64)]
    L.mxa_n_agents.argtypes = [P]
    L.mxa_n_envs.argtypes = [P]
    L.mxa_env_bytes.argtypes = [P]
    L.mxa_env_bytes.restype = I64
    L.mxa_set_stream.argtypes = [P, P]
    L.mxa_last_kernel_ms.argtypes = [P]
    L.mxa_last_kernel_ms.restype = D
    L.mxa_last_error.argtypes = [P]
    L.mxa_last_error.restype = ctypes.c_char_p
    L.mxa_destroy.argtypes = [P]
    L.mxa_destroy.restype = None
    L.mxa_set_seeds.argtypes = [P, P]
    L.mxa_read_raw.argtypes = [P, I32, I64, I64, P]
    L.mxa_layout.argtypes = [P, P]
    L.mxa_write_results.argtypes = [P, P]
    for name, args in (("mxa_write_records", [P, P]), ("mxa_set_id_persistence", [P, I32]),
                       ("mxa_read_counters", [P, P]),
                       ("mxa_create_hist", [I32, I32, P, I32, I32, P, P, I32, ctypes.POINTER(P)]),
                       ("mxa_create_replay_runner", [P, P, P, P, P, I32, I32, I32, I32, ctypes.POINTER(P)]),
                       ("mxa_set_stop_time", [P, I64]), ("mxa_run_until", [P, I64, P]),
                       ("mxa_create_replay_twap", [P, P, P, P, P, I32, I32, I32, I32, I32, ctypes.POINTER(P)]),
                       ("mxa_create_params", [I32, I32, P, P, I32, I32, ctypes.POINTER(P)]),
                       ("mxa_set_mm_params", [P, P]), ("mxa_resident_envs", [P]),
                       ("mxa_set_exchange_log", [P, I32]), ("mxa_set_launch_schedule", [P, I64]),
                       ("mxa_config_defaults", [I32, P]), ("mxa_config_compile", [P, ctypes.c_char_p, P, I32]),
                       ("mxa_config_key", [P, P]), ("mxa_config_info", [I32, P]),
                       ("mxa_create_config", [P, I32, P, I32, I32, ctypes.c_char_p, ctypes.POINTER(P)])):
        if hasattr(L, name):  # (older single-configuration A/B builds lack them; libmxa.so has all)
            getattr(L, name).argtypes = args
    L.mxa_write_rl_state.argtypes = [P, P]
    L.mxa_set_parity_hash.argtypes = [P, I32]
    L.mxa_rng_probe.argtypes = [I32, U32, I32, D, D, I32, P]
    L.mxa_math_probe.argtypes = [I32, I32, P, P, P, I64]
    L.mxa_create_replay.argtypes = [P, P, P, P, P, I32, I32, I32, I32, ctypes.POINTER(P)]
    L.mxa_step.argtypes = [P, P, P, P]
    L.mxa_step_device.argtypes = [P, P, P, P]
    if hasattr(L, "mxa_step_many"):  # (A/B builds of earlier sources lack it; tests check the exports)
        L.mxa_step_many.argtypes = [P, I32, P, P, P]
    L.mxa_finalize.argtypes = [P]
    L.mxa_read_final.argtypes = [P, I32, P, I32]
    if hasattr(L, "mxa_set_book_log"):
        L.mxa_set_book_log.argtypes = [P, I32]
        L.mxa_read_book_log.argtypes = [P, I32, P, I64, ctypes.POINTER(I64)]
    if hasattr(L, "mxa_build_id"):  # (absent from libraries built before it existed: A/B runs)
        L.mxa_build_id.argtypes = []
        L.mxa_build_id.restype = ctypes.c_char_p
    _lib = L
    return L


def build_id():
    """the kernel-source hash libmxa was built with (build_lib.build_id)"""
    L = load()
    return L.mxa_build_id().decode() if hasattr(L, "mxa_build_id") else "unknown"
