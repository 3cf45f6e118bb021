"""Runtime compositions: a config script's agent list given at run time (include/mxa.h mxa_config).

The reference's Kernel.runner(agents, startTime, stopTime, ...) (Kernel.py:50-64) runs whatever
list a config script builds.  A `MarketConfig` is that list for the scripts built from the
existing agent classes: its base names the script whose construction it follows (global-RNG
draw order, latency model) and the caller sets the counts and the per-class parameters:

  * "rmsc03"          config/rmsc03.py:95-197: exchange, n_noise NoiseAgent, n_value ValueAgent,
                      n_mm POVMarketMakerAgent (0 or 1), n_momentum MomentumAgent
  * "value_noise"     config/value_noise.py:98-161: exchange, noise and value agents, latency matrix
  * "sparse_zi_100"   config/sparse_zi_100.py:177-334: the ZI strategy table, cubic LatencyModel
  * "sparse_zi_1000"  config/sparse_zi_1000.py: the same agents on the symmetric latency matrix

The engine is specialised per composition, as it is per built-in configuration: `compile`
builds it once (hipcc, ~40 s, cached by key beside libmxa.so) and `VecMarket(cfg, seeds)` runs it.
Compile before the process touches the GPU where that is convenient; it uses no GPU itself.
"""
import ctypes

from . import _lib

ZI_GROUPS_MAX = 8  # include/mxa.h MXA_CONFIG_ZI_GROUPS
BASES = {"rmsc03": _lib.MXA_RMSC03, "value_noise": _lib.MXA_VALUE_NOISE, "sparse_zi_100": _lib.MXA_SPARSE_ZI_100,
         "sparse_zi_1000": _lib.MXA_SPARSE_ZI_1000}
BASE_NAMES = {v: k for k, v in BASES.items()}


class MmParams(ctypes.Structure):  # include/mxa.h mxa_mm_params
    _fields_ = [("mm_pov", ctypes.c_double), ("mm_min_order_size", ctypes.c_int32), ("mm_window_size", ctypes.c_int32),
                ("mm_num_ticks", ctypes.c_int32), ("pad", ctypes.c_int32), ("mm_wake_up_freq_ns", ctypes.c_int64)]


_I32, _I64, _D = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
_G = ZI_GROUPS_MAX


class MarketConfig(ctypes.Structure):
    """include/mxa.h mxa_config (the oracle's ora_config has the same layout)"""
    _fields_ = [("base", _I32), ("log_orders", _I32), ("n_noise", _I32), ("n_value", _I32), ("n_mm", _I32),
                ("n_momentum", _I32), ("n_zi_groups", _I32), ("zi_q_max", _I32),
                ("zi_count", _I32 * _G), ("zi_r_min", _I32 * _G), ("zi_r_max", _I32 * _G), ("zi_eta", _D * _G),
                ("zi_sigma_n", _D), ("zi_r_bar", _D), ("zi_kappa", _D), ("zi_sigma_s", _D), ("zi_sigma_pv", _D),
                ("zi_lambda_a", _D),
                ("mkt_open_ns", _I64), ("mkt_close_ns", _I64), ("kernel_start_ns", _I64), ("kernel_stop_ns", _I64),
                ("noise_wake_open_ns", _I64), ("noise_wake_close_ns", _I64), ("date_ns", _I64),
                ("starting_cash", _I64), ("default_computation_delay_ns", _I64),
                ("r_bar", _D), ("kappa", _D), ("fund_vol", _D), ("megashock_lambda_a", _D), ("megashock_mean", _D),
                ("megashock_var", _D),
                ("value_sigma_n", _D), ("value_r_bar", _D), ("value_kappa", _D), ("value_sigma_s", _D),
                ("value_lambda_a", _D), ("value_starting_cash", _I64),
                ("mm", MmParams), ("mom_min_size", _I32), ("mom_max_size", _I32), ("mom_wake_up_freq_ns", _I64),
                ("lat_low", _D), ("lat_high", _D), ("queue_capacity", _I32), ("book_capacity", _I32)]

    @property
    def base_name(self):
        return BASE_NAMES[self.base]

    @property
    def zi_table(self):
        """[(count, R_min, R_max, eta)] of the ZI strategy groups"""
        return [(self.zi_count[g], self.zi_r_min[g], self.zi_r_max[g], self.zi_eta[g]) for g in range(self.n_zi_groups)]

    @zi_table.setter
    def zi_table(self, rows):
        rows = list(rows)
        if len(rows) > ZI_GROUPS_MAX:
            raise ValueError("at most %d ZI groups" % ZI_GROUPS_MAX)
        self.n_zi_groups = len(rows)
        for g in range(ZI_GROUPS_MAX):
            c, lo, hi, eta = rows[g] if g < len(rows) else (0, 0, 0, 0.0)
            self.zi_count[g], self.zi_r_min[g], self.zi_r_max[g], self.zi_eta[g] = int(c), int(lo), int(hi), float(eta)

    @property
    def n_agents(self):
        return 1 + self.n_noise + self.n_value + self.n_mm + self.n_momentum + sum(c for c, _, _, _ in self.zi_table)

    def to_bytes(self):
        return bytes(self)

    def __repr__(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("zi_count", "zi_r_min", "zi_r_max", "zi_eta", "mm")}
        d["zi_table"] = self.zi_table
        d["mm"] = {k: getattr(self.mm, k) for k, _ in MmParams._fields_ if k != "pad"}
        return "MarketConfig(%r)" % d


def defaults(base):
    """the base script's own composition (mxa_config_defaults)"""
    L = _lib.load()
    c = MarketConfig()
    b = BASES[base] if isinstance(base, str) else int(base)
    if L.mxa_config_defaults(b, ctypes.byref(c)) != 0:
        raise ValueError(L.mxa_last_error(None).decode())
    return c


def make(script, zi_table=None, mm=None, **fields):
    """defaults(script) with the given fields replaced; zi_table = [(count, R_min, R_max, eta)],
    mm = dict of mxa_mm_params fields"""
    c = defaults(script)
    for k, v in fields.items():
        if not hasattr(c, k) or k in ("zi_count", "zi_r_min", "zi_r_max", "zi_eta"):
            raise AttributeError("MarketConfig has no field %r" % k)
        setattr(c, k, v)
    if zi_table is not None:
        c.zi_table = zi_table
    for k, v in (mm or {}).items():
        setattr(c.mm, k, v)
    return c


def to_dict(cfg):
    """the composition as plain JSON-able fields (mm a dict, the ZI arrays lists)"""
    d = {}
    for k, _ in MarketConfig._fields_:
        v = getattr(cfg, k)
        if k == "mm":
            d[k] = {n: getattr(v, n) for n, _ in MmParams._fields_}
        elif k in ("zi_count", "zi_r_min", "zi_r_max", "zi_eta"):
            d[k] = list(v)
        else:
            d[k] = v
    return d


def from_dict(d):
    """a MarketConfig from to_dict's fields (every field given; extra keys are ignored)"""
    c = MarketConfig()
    for k, _ in MarketConfig._fields_:
        v = d[k]
        if k == "mm":
            for n, _ in MmParams._fields_:
                setattr(c.mm, n, v[n])
        elif k in ("zi_count", "zi_r_min", "zi_r_max", "zi_eta"):
            arr = getattr(c, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(c, k, v)
    return c


def key(cfg):
    L = _lib.load()
    buf = ctypes.create_string_buffer(17)
    L.mxa_config_key(ctypes.byref(cfg), buf)
    return buf.value.decode()


def compile(cfg, cache_dir=None):
    """build (or find) the composition's specialised library; returns its path (mxa_config_compile)"""
    L = _lib.load()
    buf = ctypes.create_string_buffer(4096)
    rc = L.mxa_config_compile(ctypes.byref(cfg), cache_dir.encode() if cache_dir else None, buf, len(buf))
    if rc != 0:
        raise _lib.MxaError("mxa_config_compile failed (%d): %s" % (rc, L.mxa_last_error(None).decode()))
    return buf.value.decode()


def agent_names(cfg):
    """Agent.name of every agent as the base script names them (config/rmsc03.py:120-193,
    config/value_noise.py, config/sparse_zi_100.py:215-250)"""
    if cfg.base_name in ("sparse_zi_100", "sparse_zi_1000"):
        names, a = ["Exchange Agent 0"], 1
        for g, (cnt, lo, hi, eta) in enumerate(cfg.zi_table):
            for _ in range(cnt):
                names.append("ZI Agent %d Type %d [%d <= R <= %d, eta=%s]" % (a, g + 1, lo, hi, _py_num(eta)))
                a += 1
        return names
    ex = "Exchange Agent 0" if cfg.base_name == "value_noise" else "EXCHANGE_AGENT"
    a = 1
    names = [ex] + ["NoiseAgent %d" % j for j in range(a, a + cfg.n_noise)]
    a += cfg.n_noise
    names += ["Value Agent %d" % j for j in range(a, a + cfg.n_value)]
    a += cfg.n_value
    names += ["POV_MARKET_MAKER_AGENT_%d" % j for j in range(a, a + cfg.n_mm)]
    a += cfg.n_mm
    names += ["MOMENTUM_AGENT_%d" % j for j in range(a, a + cfg.n_momentum)]
    return names


def agent_type_names(cfg):
    """Agent.type of every agent (the summary log's AgentStrategy, Kernel's mean-value groups)"""
    if cfg.base_name in ("sparse_zi_100", "sparse_zi_1000"):
        out = ["ExchangeAgent"]
        for g, (cnt, lo, hi, eta) in enumerate(cfg.zi_table):
            out += ["ZeroIntelligenceAgent Type %d [%d <= R <= %d, eta=%s]" % (g + 1, lo, hi, _py_num(eta))] * cnt
        return out
    a = 1 + cfg.n_noise
    value = (["ValueAgent %d" % j for j in range(a, a + cfg.n_value)] if cfg.base_name == "value_noise"
             else ["ValueAgent"] * cfg.n_value)
    return (["ExchangeAgent"] + ["NoiseAgent"] * cfg.n_noise + value + ["POVMarketMakerAgent"] * cfg.n_mm +
            ["MomentumAgent"] * cfg.n_momentum)


def _py_num(x):
    """str() of the script's literal: an int eta prints as 1, a float as 0.8"""
    return str(int(x)) if float(x) == int(x) else repr(float(x))
