"""ctypes binding of the CPU parity oracle (oracle/abides_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product package.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libabides_oracle.so")
# the ExternalFileOracle series of the hist_fund_* fixtures (tests/golden/gen_fixtures.py fund_series)
DEFAULT_FUND = os.path.join(os.path.dirname(HERE), "tests", "golden", "fund_JPM_20190628.npz")
HIST_CONFIGS = ("hist_fund_value", "hist_fund_diverse")
_lib = None
_fund_set = False


def _ensure_fundamental(config):
    """hist_fund_* envs read the process-wide series: the fixtures' one unless set_fundamental ran"""
    global _fund_set
    if config in HIST_CONFIGS and not _fund_set:
        z = np.load(DEFAULT_FUND, allow_pickle=False)
        _set_arrays(z["t"], z["v"])


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, U64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int
        L.ora_create.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(P)]
        L.ora_run.argtypes = [P, I64]
        L.ora_run.restype = I64
        L.ora_finish.argtypes = [P]
        L.ora_done.argtypes = [P]
        L.ora_error.argtypes = [P]
        L.ora_error_str.argtypes = [P]
        L.ora_error_str.restype = ctypes.c_char_p
        L.ora_hash.argtypes = [P]
        L.ora_hash.restype = U64
        L.ora_events.argtypes = [P]
        L.ora_events.restype = I64
        L.ora_current_time.argtypes = [P]
        L.ora_current_time.restype = I64
        L.ora_set_trace.argtypes = [P, ctypes.c_void_p, I64]
        L.ora_trace_len.argtypes = [P]
        L.ora_trace_len.restype = I64
        L.ora_n_agents.argtypes = [P]
        L.ora_agent_state.argtypes = [P, I32, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I64)]
        L.ora_book.argtypes = [P, I32, ctypes.c_void_p, I64]
        L.ora_book.restype = I64
        L.ora_order_counter.argtypes = [P]
        L.ora_order_counter.restype = I64
        L.ora_last_trade.argtypes = [P]
        L.ora_last_trade.restype = I64
        L.ora_report.argtypes = [P, ctypes.c_char_p, I64]
        L.ora_report.restype = I64
        L.ora_destroy.argtypes = [P]
        L.ora_create_mr.argtypes = [ctypes.c_void_p] * 5 + [I32, ctypes.POINTER(P)]
        L.ora_gym_step.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(I32), ctypes.POINTER(I32)]
        L.ora_rl_state.argtypes = [P, ctypes.c_void_p]
        L.ora_run_batch.argtypes = [ctypes.c_char_p, ctypes.c_void_p, I32, I32, I64, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        L.ora_run_batch_err.argtypes = [ctypes.c_char_p, ctypes.c_void_p, I32, I32, I64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        L.ora_rs_new.argtypes = [ctypes.c_uint32]
        L.ora_rs_new.restype = P
        L.ora_rs_free.argtypes = [P]
        L.ora_rs_u32.argtypes = [P]
        L.ora_rs_u32.restype = ctypes.c_uint32
        L.ora_rs_double.argtypes = [P]
        L.ora_rs_double.restype = ctypes.c_double
        L.ora_rs_randint.argtypes = [P, I64, I64]
        L.ora_rs_randint.restype = I64
        L.ora_rs_normal.argtypes = [P, ctypes.c_double, ctypes.c_double]
        L.ora_rs_normal.restype = ctypes.c_double
        L.ora_rs_exponential.argtypes = [P, ctypes.c_double]
        L.ora_rs_exponential.restype = ctypes.c_double
        L.ora_rs_uniform.argtypes = [P, ctypes.c_double, ctypes.c_double]
        L.ora_rs_uniform.restype = ctypes.c_double
        _lib = L
    return _lib


def set_fundamental(series):
    """the ExternalFileOracle series (mxabides.fundamental.FundamentalSeries) of the hist_fund_*
    configs, for every oracle env created afterwards in this process"""
    _set_arrays(series.t, series.v)


def _set_arrays(t, v):
    global _fund_set
    L = lib()
    L.ora_set_fundamental.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    t = np.ascontiguousarray(t, dtype=np.int64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    L.ora_set_fundamental(t.ctypes.data, v.ctypes.data, len(t))
    _fund_set = True


# ora_mm_params (abides_oracle.h): config/rmsc03.py's market-maker options
MM_DTYPE = np.dtype([("mm_pov", "<f8"), ("mm_min_order_size", "<i4"), ("mm_window_size", "<i4"),
                     ("mm_num_ticks", "<i4"), ("pad", "<i4"), ("mm_wake_up_freq_ns", "<i8")])


class _Mm(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double if t == "<f8" else ctypes.c_int64 if t == "<i8" else ctypes.c_int32)
                for n, (t, _) in ((k, (MM_DTYPE.fields[k][0].str, 0)) for k in MM_DTYPE.names)]


_I, _Q, _F, _G = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, 8


class OraConfig(ctypes.Structure):
    """ora_config (abides_oracle.h): a runtime composition, the layout of include/mxa.h mxa_config"""
    _fields_ = ([(n, _I) for n in ("base", "log_orders", "n_noise", "n_value", "n_mm", "n_momentum", "n_zi_groups",
                                  "zi_q_max")] +
                [("zi_count", _I * _G), ("zi_r_min", _I * _G), ("zi_r_max", _I * _G), ("zi_eta", _F * _G)] +
                [(n, _F) for n in ("zi_sigma_n", "zi_r_bar", "zi_kappa", "zi_sigma_s", "zi_sigma_pv", "zi_lambda_a")] +
                [(n, _Q) for n in ("mkt_open_ns", "mkt_close_ns", "kernel_start_ns", "kernel_stop_ns",
                                  "noise_wake_open_ns", "noise_wake_close_ns", "date_ns", "starting_cash",
                                  "default_computation_delay_ns")] +
                [(n, _F) for n in ("r_bar", "kappa", "fund_vol", "megashock_lambda_a", "megashock_mean",
                                  "megashock_var", "value_sigma_n", "value_r_bar", "value_kappa", "value_sigma_s",
                                  "value_lambda_a")] +
                [("value_starting_cash", _Q), ("mm", _Mm), ("mom_min_size", _I), ("mom_max_size", _I),
                 ("mom_wake_up_freq_ns", _Q), ("lat_low", _F), ("lat_high", _F), ("queue_capacity", _I),
                 ("book_capacity", _I)])


def config_defaults(base):
    """ora_config_defaults: the base script's composition"""
    L = lib()
    L.ora_config_defaults.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    c = OraConfig()
    if L.ora_config_defaults(base.encode(), ctypes.byref(c)):
        raise ValueError("no such base %r" % base)
    return c


def as_config(cfg):
    """an ora_config from any object holding mxa_config's bytes (mxabides.composition.MarketConfig)"""
    b = bytes(cfg)
    if len(b) != ctypes.sizeof(OraConfig):
        raise ValueError("a composition is %d bytes, got %d" % (ctypes.sizeof(OraConfig), len(b)))
    return OraConfig.from_buffer_copy(b)


def config_log_orders(config):
    L = lib()
    L.ora_config_log_orders.argtypes = [ctypes.c_char_p]
    return L.ora_config_log_orders(config.encode())


class OracleEnv:
    """One reference-semantics simulation (config + seed); config "rmsc03" with `mm` (one
    MM_DTYPE record) runs config/rmsc03.py with those --mm-* options; a composition (an
    OraConfig, or a MarketConfig's bytes) runs ora_create_config."""

    def __init__(self, config, seed, trace_cap=0, mm=None):
        L = lib()
        self._h = ctypes.c_void_p()
        if not isinstance(config, str):
            self._cfg = as_config(config)
            L.ora_create_config.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
            rc = L.ora_create_config(ctypes.byref(self._cfg), seed & 0xFFFFFFFF, ctypes.byref(self._h))
            if rc:
                raise ValueError("oracle: bad composition")
        elif mm is not None:
            if config != "rmsc03":
                raise ValueError("market-maker options are config/rmsc03.py's")
            self._mm = np.ascontiguousarray(np.asarray(mm, dtype=MM_DTYPE).reshape(1))
            L.ora_create_mm.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
            rc = L.ora_create_mm(seed & 0xFFFFFFFF, self._mm.ctypes.data, ctypes.byref(self._h))
        else:
            _ensure_fundamental(config)
            rc = L.ora_create(config.encode(), seed & 0xFFFFFFFF, ctypes.byref(self._h))
        if rc:
            raise ValueError("oracle: bad config %r" % config)
        self.trace_buf = None
        if trace_cap:
            self.trace_buf = np.zeros((trace_cap, 10), dtype=np.int64)
            L.ora_set_trace(self._h, self.trace_buf.ctypes.data, trace_cap)

    def run(self, max_pops=-1):
        return lib().ora_run(self._h, max_pops)

    def finish(self):
        lib().ora_finish(self._h)

    def set_stop(self, t_stop):
        """Kernel.runner's stopTime (ns since midnight) instead of the config's; before run()"""
        L = lib()
        L.ora_set_stop.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.ora_set_stop(self._h, int(t_stop))

    @property
    def done(self):
        return bool(lib().ora_done(self._h))

    @property
    def error(self):
        L = lib()
        return L.ora_error(self._h), L.ora_error_str(self._h).decode()

    @property
    def hash(self):
        return lib().ora_hash(self._h)

    @property
    def events(self):
        return lib().ora_events(self._h)

    def trace(self):
        n = lib().ora_trace_len(self._h)
        return self.trace_buf[:n]

    def set_book_log(self, on=True):
        """keep OrderBook.book_log rows (ora_set_book_log); call before run()"""
        L = lib()
        L.ora_set_book_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_set_book_log(self._h, 1 if on else 0)

    def set_exchange_log(self, on=True):
        """the exchange's own log in the book records (ora_set_exchange_log); call before run()"""
        L = lib()
        L.ora_set_exchange_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_set_exchange_log(self._h, 1 if on else 0)

    def book_log(self):
        """the rows as flat int64 (mxabides.booklog format: t, n, executed qty, average price,
        n (price, volume) pairs, bids best-first then asks best-first)"""
        L = lib()
        L.ora_book_log.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.ora_book_log.restype = ctypes.c_int64
        n = L.ora_book_log(self._h, None, 0)
        buf = np.zeros(n, dtype=np.int64)
        L.ora_book_log(self._h, buf.ctypes.data, n)
        return buf

    def book_records(self):
        """the run as device book-update records: (t, price, qty) int64 rows"""
        L = lib()
        L.ora_book_records.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.ora_book_records.restype = ctypes.c_int64
        n = L.ora_book_records(self._h, None, 0)
        buf = np.zeros((n, 3), dtype=np.int64)
        L.ora_book_records(self._h, buf.ctypes.data, 3 * n)
        return buf

    def agents(self):
        L = lib()
        out = []
        for i in range(L.ora_n_agents(self._h)):
            c, s, n = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            L.ora_agent_state(self._h, i, ctypes.byref(c), ctypes.byref(s), ctypes.byref(n))
            out.append((c.value, s.value, n.value))
        return out

    def book(self, side):
        L = lib()
        n = L.ora_book(self._h, side, None, 0)
        buf = np.zeros(n, dtype=np.int64)
        L.ora_book(self._h, side, buf.ctypes.data, n)
        levels, k = [], 1
        for _ in range(buf[0]):
            m = buf[k]
            k += 1
            levels.append([buf[k + 4 * j:k + 4 * j + 4].tolist() for j in range(m)])
            k += 4 * m
        return levels

    @property
    def order_counter(self):
        return lib().ora_order_counter(self._h)

    @property
    def last_trade(self):
        return lib().ora_last_trade(self._h)

    SUMMARY_EVENTS = ["STARTING_CASH", "FINAL_CASH_POSITION", "ENDING_CASH", "FINAL_VALUATION"]

    def summary_log(self):
        """Kernel.summaryLog rows after finish(): dicts with AgentID, AgentStrategy, EventType, Event
        (Event an int or a float exactly as the reference logs it)."""
        L = lib()
        L.ora_summary.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 5 + [ctypes.c_int]
        L.ora_agent_type_name.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.ora_agent_type_name.restype = ctypes.c_char_p
        n = L.ora_summary(self._h, None, None, None, None, None, 0)
        ag, ty, isf = (np.zeros(n, dtype=np.int32) for _ in range(3))
        vi, vf = np.zeros(n, dtype=np.int64), np.zeros(n, dtype=np.float64)
        L.ora_summary(self._h, ag.ctypes.data, ty.ctypes.data, isf.ctypes.data, vi.ctypes.data, vf.ctypes.data, n)
        return [{"AgentID": int(a), "AgentStrategy": L.ora_agent_type_name(self._h, int(a)).decode(),
                 "EventType": self.SUMMARY_EVENTS[t], "Event": float(f) if s else int(i)}
                for a, t, s, i, f in zip(ag, ty, isf, vi, vf)]

    def report(self):
        L = lib()
        n = L.ora_report(self._h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        L.ora_report(self._h, buf, n + 1)
        return buf.value.decode().splitlines()

    def __del__(self):
        try:
            lib().ora_destroy(self._h)
        except Exception:
            pass


def run_batch(config, seeds, threads, max_pops=-1):
    L = lib()
    _ensure_fundamental(config)
    seeds = np.asarray(seeds, dtype=np.uint32)
    ev = np.zeros(len(seeds), dtype=np.int64)
    hs = np.zeros(len(seeds), dtype=np.uint64)
    sec = ctypes.c_double()
    rc = L.ora_run_batch(config.encode(), seeds.ctypes.data, len(seeds), threads, max_pops, ev.ctypes.data,
                         hs.ctypes.data, ctypes.byref(sec))
    if rc:
        raise RuntimeError("oracle batch failed")
    return ev, hs, sec.value


def run_batch_err(config, seeds, threads, max_pops=-1):
    """run_batch plus each env's oracle error code (0 ok, negative fail() code)"""
    L = lib()
    _ensure_fundamental(config)
    seeds = np.asarray(seeds, dtype=np.uint32)
    ev = np.zeros(len(seeds), dtype=np.int64)
    hs = np.zeros(len(seeds), dtype=np.uint64)
    er = np.zeros(len(seeds), dtype=np.int32)
    sec = ctypes.c_double()
    rc = L.ora_run_batch_err(config.encode(), seeds.ctypes.data, len(seeds), threads, max_pops, ev.ctypes.data,
                             hs.ctypes.data, er.ctypes.data, ctypes.byref(sec))
    if rc:
        raise RuntimeError("oracle batch failed")
    return ev, hs, er, sec.value


def batch_stats(config, seeds, threads):
    """[n][4] capacity statistics (max pending events, max resting orders, max open orders of one
    agent, max live transaction records) of each env run to completion"""
    L = lib()
    L.ora_run_batch_stats.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    _ensure_fundamental(config)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.zeros((len(seeds), 4), dtype=np.int64)
    if L.ora_run_batch_stats(config.encode(), seeds.ctypes.data, len(seeds), threads, out.ctypes.data):
        raise RuntimeError("oracle batch failed")
    return out


def run_batch_config(cfg, seeds, threads, max_pops=-1, stats=False):
    """one composition over many seeds: events, hashes, error codes, seconds (and [n][4] capacity
    statistics with stats=True)"""
    L = lib()
    L.ora_run_batch_config.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64] + \
        [ctypes.c_void_p] * 4 + [ctypes.POINTER(ctypes.c_double)]
    c = as_config(cfg)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    n = len(seeds)
    ev = np.zeros(n, dtype=np.int64)
    hs = np.zeros(n, dtype=np.uint64)
    er = np.zeros(n, dtype=np.int32)
    st = np.zeros((n, 4), dtype=np.int64)
    sec = ctypes.c_double()
    if L.ora_run_batch_config(ctypes.byref(c), seeds.ctypes.data, n, threads, max_pops, ev.ctypes.data, hs.ctypes.data,
                              er.ctypes.data, st.ctypes.data if stats else None, ctypes.byref(sec)):
        raise RuntimeError("oracle batch failed")
    return (ev, hs, er, sec.value, st) if stats else (ev, hs, er, sec.value)


def run_batch_mm(seeds, params, threads, max_pops=-1, stats=False):
    """rmsc03 envs with per-env market-maker options (params: MM_DTYPE [n]): events, hashes, error
    codes, seconds (and the [n][4] capacity statistics with stats=True)"""
    L = lib()
    L.ora_run_batch_mm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64] + \
        [ctypes.c_void_p] * 4 + [ctypes.POINTER(ctypes.c_double)]
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    prm = np.ascontiguousarray(np.asarray(params, dtype=MM_DTYPE))
    if len(prm) != len(seeds):
        raise ValueError("one parameter record per seed")
    n = len(seeds)
    ev = np.zeros(n, dtype=np.int64)
    hs = np.zeros(n, dtype=np.uint64)
    er = np.zeros(n, dtype=np.int32)
    st = np.zeros((n, 4), dtype=np.int64)
    sec = ctypes.c_double()
    if L.ora_run_batch_mm(seeds.ctypes.data, prm.ctypes.data, n, threads, max_pops, ev.ctypes.data, hs.ctypes.data,
                          er.ctypes.data, st.ctypes.data if stats else None, ctypes.byref(sec)):
        raise RuntimeError("oracle batch failed")
    return (ev, hs, er, sec.value, st) if stats else (ev, hs, er, sec.value)


def gym_batch(actions, threads, seeds=None, tape=None):
    """n GymKernel episodes on host threads: actions [n_steps][n][3]; seeds -> the rmsc03 + DummyRL
    composition, tape -> the replay composition.  Returns dict of per-env events, hash, err
    (oracle fail() code), steps and the last valid obs [n][9], plus seconds."""
    L = lib()
    L.ora_gym_batch.argtypes = [ctypes.c_char_p] + [ctypes.c_void_p] * 6 + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int] \
        + [ctypes.c_void_p] * 5 + [ctypes.POINTER(ctypes.c_double)]
    act = np.ascontiguousarray(actions, dtype=np.float64)
    n_steps, n = act.shape[0], act.shape[1]
    ev = np.zeros(n, dtype=np.int64)
    hs = np.zeros(n, dtype=np.uint64)
    er = np.zeros(n, dtype=np.int32)
    st = np.zeros(n, dtype=np.int32)
    obs = np.zeros((n, 9), dtype=np.float64)
    sec = ctypes.c_double()
    if tape is None:
        sd = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
        assert len(sd) == n
        rc = L.ora_gym_batch(b"rmsc03_rl", sd.ctypes.data, None, None, None, None, None, 0, n, n_steps, act.ctypes.data,
                             threads, ev.ctypes.data, hs.ctypes.data, er.ctypes.data, st.ctypes.data, obs.ctypes.data,
                             ctypes.byref(sec))
    else:
        rc = L.ora_gym_batch(None, None, tape.t.ctypes.data, tape.oid.ctypes.data, tape.price.ctypes.data,
                             tape.size.ctypes.data, tape.buy.ctypes.data, len(tape), n, n_steps, act.ctypes.data,
                             threads, ev.ctypes.data, hs.ctypes.data, er.ctypes.data, st.ctypes.data, obs.ctypes.data,
                             ctypes.byref(sec))
    if rc:
        raise RuntimeError("oracle gym batch failed")
    return dict(events=ev, hash=hs, err=er, steps=st, obs=obs, seconds=sec.value)


class OracleReplayRunner(OracleEnv):
    """config/marketreplay.py: the exchange and the MarketReplayAgent on a tape under Kernel.runner
    (run / finish / report / summary_log / book / agents as OracleEnv)"""

    def __init__(self, tape, symbol="IBM", trace_cap=0, twap=None):
        """twap: None = config/marketreplay.py; False / True = config/execution/marketreplay/
        execution_marketreplay.py without / with -e (the TWAP execution agent trades)"""
        L = lib()
        L.ora_create_mr_runner.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.ora_create_mr_twap.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.ora_set_symbol.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        self._h = ctypes.c_void_p()
        self._tape = tape
        args = (tape.t.ctypes.data, tape.oid.ctypes.data, tape.price.ctypes.data, tape.size.ctypes.data,
                tape.buy.ctypes.data, len(tape))
        if twap is None:
            rc = L.ora_create_mr_runner(*args, ctypes.byref(self._h))
        else:
            rc = L.ora_create_mr_twap(*args, 1 if twap else 0, ctypes.byref(self._h))
        if rc:
            raise ValueError("oracle: bad tape (%d)" % rc)
        L.ora_set_symbol(self._h, symbol.encode())
        self.trace_buf = None
        if trace_cap:
            self.trace_buf = np.zeros((trace_cap, 10), dtype=np.int64)
            L.ora_set_trace(self._h, self.trace_buf.ctypes.data, trace_cap)


class OracleGymEnv(OracleEnv):
    """GymKernel restatement: ABIDESEnv (Exchange + MarketReplayAgent + DummyRL on a LOBSTER tape),
    or with `tape=None, seed=s` the rmsc03 + DummyRL composition (config "rmsc03_rl")."""

    def __init__(self, tape=None, trace_cap=0, seed=None):
        L = lib()
        self._h = ctypes.c_void_p()
        self._tape = tape
        if tape is None:
            rc = L.ora_create(b"rmsc03_rl", int(seed) & 0xFFFFFFFF, ctypes.byref(self._h))
        else:
            rc = L.ora_create_mr(tape.t.ctypes.data, tape.oid.ctypes.data, tape.price.ctypes.data,
                                 tape.size.ctypes.data, tape.buy.ctypes.data, len(tape), ctypes.byref(self._h))
        if rc:
            raise ValueError("oracle: bad tape or config (%d)" % rc)
        self.trace_buf = None
        if trace_cap:
            self.trace_buf = np.zeros((trace_cap, 10), dtype=np.int64)
            L.ora_set_trace(self._h, self.trace_buf.ctypes.data, trace_cap)

    def reset(self, seed=None, trace_cap=0):
        """ABIDESEnv.reset in the same process (ora_gym_reset): a new episode (rmsc03_rl: from
        `seed`), Order.order_id / Order._order_ids carried over"""
        L = lib()
        L.ora_gym_reset.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32]
        rc = L.ora_gym_reset(ctypes.byref(self._h), (int(seed) if seed is not None else 0) & 0xFFFFFFFF)
        if rc:
            raise ValueError("oracle: gym reset failed (%d)" % rc)
        self.trace_buf = None
        if trace_cap:
            self.trace_buf = np.zeros((trace_cap, 10), dtype=np.int64)
            L.ora_set_trace(self._h, self.trace_buf.ctypes.data, trace_cap)

    def step(self, action):
        """-> (obs float64[9] or None, done, rc)"""
        a = np.ascontiguousarray(action, dtype=np.float64)
        obs = np.zeros(9, dtype=np.float64)
        has, done = ctypes.c_int(), ctypes.c_int()
        rc = lib().ora_gym_step(self._h, a.ctypes.data, obs.ctypes.data, ctypes.byref(has), ctypes.byref(done))
        return (obs if has.value else None), bool(done.value), rc

    def rl_state(self):
        out = np.zeros(4, dtype=np.int64)
        lib().ora_rl_state(self._h, out.ctypes.data)
        return out


class RandomState:
    """numpy-legacy RandomState restatement (for KAT tests)."""

    def __init__(self, seed):
        self._h = lib().ora_rs_new(seed)

    def u32(self):
        return lib().ora_rs_u32(self._h)

    def rand(self):
        return lib().ora_rs_double(self._h)

    def randint(self, lo, hi):
        return lib().ora_rs_randint(self._h, lo, hi)

    def normal(self, loc, scale):
        return lib().ora_rs_normal(self._h, loc, scale)

    def exponential(self, scale):
        return lib().ora_rs_exponential(self._h, scale)

    def uniform(self, lo, hi):
        return lib().ora_rs_uniform(self._h, lo, hi)

    def __del__(self):
        try:
            lib().ora_rs_free(self._h)
        except Exception:
            pass
