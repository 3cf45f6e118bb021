"""VecMarket: N independent ABIDES markets of one configuration on one MI355X.

Host mirror of the reference's batch entry point (`python abides.py -c <config> -s <seed>`,
abides.py:19-29 -> config/<config>.py -> Kernel.runner, Kernel.py:50-345): every env is
one reference simulation with its own seed, all simulated by libmxa's HIP kernels.
"""
import ctypes
import os

import numpy as np

from . import _lib
from .configs import (BOOK_FREQ, HIST_CONFIGS, MM_PARAMS_DTYPE, REPLAY_CONFIGS, agent_names, agent_type_names,
                      symbol_of)

CHUNK_DEFAULT = 1 << 20


class VecMarket:
    def __init__(self, config, seeds, device=0, trace_cap=0, book_log=0, symbol=None, fundamental=None,
                 book_freq="config", tape=None, mm_params=None, exchange_log=False):
        """book_log: records per env of the book-update log (0 off), the input of the exchange's
        order-book outputs (orderbook_snapshots, exchange_events; include/mxa.h
        mxa_set_book_log).  A limit order takes 2-4 records, a cancellation 1.
        symbol: the -t/--ticker of the configs that take one (output names only).
        fundamental: the ExternalFileOracle series of hist_fund_value / hist_fund_diverse
        (mxabides.fundamental.FundamentalSeries).  book_freq: the exchange's (default: the config
        script's, configs.BOOK_FREQ), which decides the order-book file write_logs writes.
        tape: the LOBSTER tape (mxabides.tape.Tape) of marketreplay_runner, config/marketreplay.py
        (the seeds only count the envs there: nothing in that composition draws).
        mm_params: rmsc03 only: config/rmsc03.py's --mm-* options per env (configs.mm_params, one
        record or one per env; include/mxa.h mxa_create_params).
        exchange_log: the exchange's own log (ExchangeAgent.log, EXCHANGE_AGENT.bz2) rides in the
        book-update log (include/mxa.h mxa_set_exchange_log; needs book_log)."""
        from .composition import MarketConfig
        self.composition = None
        if isinstance(config, MarketConfig):  # a runtime composition (mxabides.composition)
            self.composition = MarketConfig.from_buffer_copy(bytes(config))
            config = self.composition.base_name
        elif config not in _lib.CONFIG_IDS:
            raise ValueError("unknown config %r (supported: %s, or a composition.MarketConfig)" %
                             (config, sorted(_lib.CONFIG_IDS)))
        self.L = _lib.load()
        self.config = config
        if symbol is not None:
            symbol_of(config, symbol, tape)  # a fixed-symbol config refuses -t now, not at output time
        self._symbol = symbol
        self.tape = tape
        self.book_freq = BOOK_FREQ[config] if book_freq == "config" else book_freq
        self.seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
        self.n_envs = len(self.seeds)
        self.device = device
        self.trace_cap = trace_cap
        self._h = ctypes.c_void_p()
        self.fundamental = fundamental
        if config in REPLAY_CONFIGS:
            if tape is None:
                raise ValueError("%s replays a LOBSTER tape (tape=mxabides.tape.Tape)" % config)
            self.tape = tape
            tp = (tape.t.ctypes.data, tape.oid.ctypes.data, tape.price.ctypes.data, tape.size.ctypes.data,
                  tape.buy.ctypes.data, len(tape))
            if config == "marketreplay_runner":
                rc = self.L.mxa_create_replay_runner(*tp, self.n_envs, device, trace_cap, ctypes.byref(self._h))
            else:
                rc = self.L.mxa_create_replay_twap(*tp, 1 if config == "marketreplay_twap_e" else 0, self.n_envs,
                                                   device, trace_cap, ctypes.byref(self._h))
            self._check(rc, "mxa_create_replay_%s" % config.split("_", 1)[1])
        elif config in HIST_CONFIGS:
            if fundamental is None:
                raise ValueError("%s needs its ExternalFileOracle series (fundamental=FundamentalSeries)" % config)
            f = fundamental
            rc = self.L.mxa_create_hist(_lib.CONFIG_IDS[config], self.n_envs, self.seeds.ctypes.data, device, trace_cap,
                                        f.t.ctypes.data, f.v.ctypes.data, len(f), ctypes.byref(self._h))
            self._check(rc, "mxa_create_hist")
        elif self.composition is not None:
            if mm_params is not None or fundamental is not None or tape is not None:
                raise ValueError("a composition carries its own parameters (MarketConfig.mm)")
            rc = self.L.mxa_create_config(ctypes.byref(self.composition), self.n_envs, self.seeds.ctypes.data, device,
                                          trace_cap, None, ctypes.byref(self._h))
            if rc == -4:  # MXA_ERANGE: not compiled yet
                raise _lib.MxaError("%s; compile it first (mxabides.composition.compile)" %
                                    self.L.mxa_last_error(None).decode())
            if rc < 0:
                raise _lib.MxaError("mxa_create_config failed (%d): %s" % (rc, self.L.mxa_last_error(None).decode()))
        elif mm_params is not None:
            if config != "rmsc03":
                raise ValueError("mm_params are config/rmsc03.py's market-maker options")
            self.mm_params = self._mm_array(mm_params)
            rc = self.L.mxa_create_params(_lib.MXA_RMSC03, self.n_envs, self.seeds.ctypes.data,
                                          self.mm_params.ctypes.data, device, trace_cap, ctypes.byref(self._h))
            self._check(rc, "mxa_create_params")
        else:
            if fundamental is not None:
                raise ValueError("%s runs the SparseMeanRevertingOracle; a fundamental series is for %s" % (config, HIST_CONFIGS))
            rc = self.L.mxa_create(_lib.CONFIG_IDS[config], self.n_envs, self.seeds.ctypes.data, device, trace_cap,
                                   ctypes.byref(self._h))
            self._check(rc, "mxa_create")
        self.n_agents = self.L.mxa_n_agents(self._h)
        self.book_log_cap = int(book_log)
        if book_log:
            self._check(self.L.mxa_set_book_log(self._h, int(book_log)), "mxa_set_book_log")
        self.exchange_log_on = False
        if exchange_log:
            self.set_exchange_log(True)

    def _agent_names(self):
        if self.composition is not None:
            from .composition import agent_names as names
            return names(self.composition)
        return agent_names(self.config)

    def _agent_type_names(self):
        if self.composition is not None:
            from .composition import agent_type_names as names
            return names(self.composition)
        return agent_type_names(self.config)

    @property
    def symbol(self):
        """the outputs' ticker, resolved when an output needs it (a replay tape built in memory
        may carry none; configs.symbol_of)"""
        return symbol_of(self.config, self._symbol, self.tape)

    def _mm_array(self, p):
        p = np.asarray(p, dtype=MM_PARAMS_DTYPE).reshape(-1)
        if len(p) == 1:
            p = np.repeat(p, self.n_envs)
        if len(p) != self.n_envs:
            raise ValueError("mm_params: one record or one per env")
        return np.ascontiguousarray(p)

    def set_mm_params(self, mm_params):
        """the --mm-* options the next reset() builds with (a handle created with mm_params)"""
        self.mm_params = self._mm_array(mm_params)
        self._check(self.L.mxa_set_mm_params(self._h, self.mm_params.ctypes.data), "mxa_set_mm_params")

    @property
    def resident_envs(self):
        """envs resident on the device at once (occupancy x CUs; include/mxa.h mxa_resident_envs)"""
        return self._check(self.L.mxa_resident_envs(self._h), "mxa_resident_envs")

    def _check(self, rc, what):
        if rc < 0:
            msg = self.L.mxa_last_error(self._h).decode() if self._h else ""
            raise _lib.MxaError("%s failed (%d): %s" % (what, rc, msg))
        return rc

    # ---- lifecycle
    def reset(self, mask=None):
        self._finalized = False
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
        self._check(self.L.mxa_reset(self._h, m.ctypes.data if m is not None else None), "mxa_reset")

    def set_book_log(self, cap):
        """(Re)size the book-update log to `cap` records per env (0 off); every env's log
        restarts empty, so set it before the first launch of an episode."""
        self._check(self.L.mxa_set_book_log(self._h, int(cap)), "mxa_set_book_log")
        self.book_log_cap = int(cap)

    def set_exchange_log(self, on=True):
        """the exchange's own log (ExchangeAgent.log) in the book-update log, kept across resets
        (include/mxa.h mxa_set_exchange_log); a handle with book_log only"""
        if on and not self.book_log_cap:
            raise ValueError("the exchange log rides in the book-update log: create with book_log")
        self._check(self.L.mxa_set_exchange_log(self._h, 1 if on else 0), "mxa_set_exchange_log")
        self.exchange_log_on = bool(on)

    def set_seeds(self, seeds):
        self.seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
        assert len(self.seeds) == self.n_envs
        self._check(self.L.mxa_set_seeds(self._h, self.seeds.ctypes.data), "mxa_set_seeds")

    def set_parity_hash(self, on):
        """Per-pop parity hash (summary()["hash"]) on or off; market results are identical
        either way (include/mxa.h mxa_set_parity_hash)."""
        self._check(self.L.mxa_set_parity_hash(self._h, 1 if on else 0), "mxa_set_parity_hash")

    def set_stream(self, stream_ptr):
        """Run on an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream)."""
        self._check(self.L.mxa_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None),
                    "mxa_set_stream")

    def write_results(self, device_ptr):
        """Per-env (events, hash, status, current_time) int64 rows into device memory."""
        self._check(self.L.mxa_write_results(self._h, ctypes.c_void_p(device_ptr)), "mxa_write_results")

    def counters(self):
        """[n_envs][COUNTER_WORDS] int64 event-class counters since the last reset (kept by
        instrumented runs: parity hash on; include/mxa.h mxa_read_counters, mxabides.counters)"""
        out = np.zeros((self.n_envs, _lib.COUNTER_WORDS), dtype=np.int64)
        self._check(self.L.mxa_read_counters(self._h, out.ctypes.data), "mxa_read_counters")
        return out

    def write_records(self, device_ptr):
        """Per-env episode records [n][RECORD_WORDS] int64 into device memory (include/mxa.h
        mxa_write_records: events, hash, status, current_time, err, seed, last_trade, order_counter,
        cash, holdings, gain, 0), the rows bench.py all-gathers across ranks."""
        self._check(self.L.mxa_write_records(self._h, ctypes.c_void_p(device_ptr)), "mxa_write_records")

    def launch(self, max_pops):
        self._check(self.L.mxa_launch(self._h, max_pops), "mxa_launch")

    def sync(self):
        self._check(self.L.mxa_sync(self._h), "mxa_sync")

    def run(self, chunk=CHUNK_DEFAULT, max_launches=0):
        self._finalized = False
        n = ctypes.c_int32()
        self._check(self.L.mxa_run(self._h, chunk, max_launches, ctypes.byref(n)), "mxa_run")
        return n.value

    def set_launch_schedule(self, first_chunk):
        """run()'s launch sizes: a first launch of first_chunk pops, then launches of run()'s
        chunk, each over the envs still running; 0 = every launch `chunk`
        (include/mxa.h mxa_set_launch_schedule)"""
        self._check(self.L.mxa_set_launch_schedule(self._h, int(first_chunk)), "mxa_set_launch_schedule")

    def set_stop_time(self, t_stop_ns):
        """Kernel.runner's stopTime (ns since the simulated midnight) instead of the config
        script's kernelStopTime, kept across resets; None or <= 0 restores the config's
        (include/mxa.h mxa_set_stop_time)"""
        self._check(self.L.mxa_set_stop_time(self._h, int(t_stop_ns or 0)), "mxa_set_stop_time")

    def run_until(self, t_stop_ns):
        """Kernel.runner(startTime, stopTime=t_stop_ns) for every env: run to the first pop past
        t_stop_ns (handled, as in the reference); returns each env's ttl_messages"""
        ev = np.zeros(self.n_envs, dtype=np.int64)
        self._check(self.L.mxa_run_until(self._h, int(t_stop_ns), ev.ctypes.data), "mxa_run_until")
        return ev

    @property
    def last_kernel_ms(self):
        return self.L.mxa_last_kernel_ms(self._h)

    @property
    def env_bytes(self):
        return self.L.mxa_env_bytes(self._h)

    # ---- inspection
    def summary(self):
        arr = (_lib.EnvSummary * self.n_envs)()
        self._check(self.L.mxa_read_summary(self._h, arr), "mxa_read_summary")
        dt = {ctypes.c_int32: np.int32, ctypes.c_int64: np.int64, ctypes.c_uint64: np.uint64}
        return {k: np.array([getattr(a, k) for a in arr], dtype=dt[t]) for k, t in _lib.EnvSummary._fields_}

    def agents(self, env):
        arr = (_lib.AgentState * self.n_agents)()
        self._check(self.L.mxa_read_agents(self._h, env, arr, self.n_agents), "mxa_read_agents")
        return [dict(cash=a.cash, shares=a.shares, n_open=a.n_open, last_trade=a.last_trade, type=a.type,
                     flags=a.flags, starting_cash=a.starting_cash) for a in arr]

    def book(self, env, side):
        """OrderBook.bids (side 0) / asks (side 1): list of levels, each a FIFO list of
        [order_id, agent_id, quantity, price]."""
        cap = 4096
        while True:  # mxa_read_book returns the side's order count; a replay book holds thousands
            buf = np.zeros((cap, 4), dtype=np.int64)
            n = self._check(self.L.mxa_read_book(self._h, env, side, buf.ctypes.data, cap), "mxa_read_book")
            if n <= cap:
                break
            cap = n
        levels = []
        for o in buf[:n].tolist():
            if levels and levels[-1][0][3] == o[3]:
                levels[-1].append(o)
            else:
                levels.append([o])
        return levels

    def layout(self):
        o = np.zeros(8, dtype=np.int64)
        self._check(self.L.mxa_layout(self._h, o.ctypes.data), "mxa_layout")
        return dict(zip(["ag", "open", "rng", "lat", "q", "book", "tx", "trace"], o.tolist()))

    def raw(self, env, offset, nbytes):
        buf = np.zeros(nbytes, dtype=np.uint8)
        self._check(self.L.mxa_read_raw(self._h, env, offset, nbytes, buf.ctypes.data), "mxa_read_raw")
        return buf

    def trace(self, env):
        if not self.trace_cap:
            raise ValueError("created with trace_cap=0")
        buf = np.zeros((self.trace_cap, 10), dtype=np.int64)
        n = ctypes.c_int64()
        self._check(self.L.mxa_read_trace(self._h, env, buf.ctypes.data, self.trace_cap, ctypes.byref(n)),
                    "mxa_read_trace")
        return buf[:n.value]

    def report(self, env):
        """The reference's end-of-run stdout: TradingAgent.kernelStopping "Final holdings"
        lines (TradingAgent.py:121-126) and Kernel's mean ending value per agent type
        (Kernel.py:337-341)."""
        FL_LAST_FLOAT = 1024
        names, tnames, sym = self._agent_names(), self._agent_type_names(), self.symbol
        lines, gains, counts, order = [], {}, {}, []
        for a, st in enumerate(self.agents(env)):
            if a == 0:
                continue
            hold = "{ %s: %d, CASH: %d }" % (sym, st["shares"], st["cash"]) if st["shares"] else "{ CASH: %d }" % st["cash"]
            mtm = st["cash"] + (st["last_trade"] * st["shares"] if st["shares"] else 0)
            flt = bool(st["shares"]) and bool(st["flags"] & FL_LAST_FLOAT)
            lines.append("Final holdings for %s: %s.  Marked to market: %s" % (names[a], hold, ("%d.0" % mtm) if flt else str(mtm)))
            t = tnames[a]
            if t not in gains:
                gains[t], counts[t] = 0, 0
                order.append(t)
            gains[t] += mtm - st["starting_cash"]
            counts[t] += 1
        means = ["%s: %d" % (t, int(round(gains[t] / counts[t]))) for t in order]
        return lines, means

    SUMMARY_EVENTS = ("STARTING_CASH", "FINAL_CASH_POSITION", "ENDING_CASH", "FINAL_VALUATION")

    def finalize(self):
        """Kernel.runner's kernelStopping pass (Kernel.py:305-312) for every env, once the run is
        over: the agents' FINAL_VALUATION (oracle observed in agent order).  Idempotent."""
        self._check(self.L.mxa_finalize(self._h), "mxa_finalize")
        self._finalized = True

    def summary_log(self, env):
        """Kernel.summaryLog (Kernel.py:549-554) of one env as the reference builds it: STARTING_CASH
        of every trading agent (TradingAgent.kernelStarting, TradingAgent.py:101), then per agent
        FINAL_CASH_POSITION and ENDING_CASH (TradingAgent.py:118-123) and the FINAL_VALUATION of
        ZI / Noise / Value agents.  Rows are dicts AgentID, AgentStrategy, EventType, Event; Event
        is an int or a float exactly where the reference logs one."""
        if not getattr(self, "_finalized", False):
            self.finalize()
        fin = (_lib.AgentFinal * self.n_agents)()
        self._check(self.L.mxa_read_final(self._h, env, fin, self.n_agents), "mxa_read_final")
        tnames = self._agent_type_names()
        ag = self.agents(env)
        FL_LAST_FLOAT = 1024
        rows = [dict(AgentID=a, AgentStrategy=tnames[a], EventType="STARTING_CASH", Event=int(ag[a]["starting_cash"]))
                for a in range(1, self.n_agents)]
        for a in range(1, self.n_agents):
            st, f = ag[a], fin[a]
            if f.err:
                raise _lib.MxaError("env %d agent %d: the reference raises in kernelStopping (%s)"
                                    % (env, a, "KeyError" if f.err == 1 else "IndexError"))
            mtm = st["cash"] + (st["last_trade"] * st["shares"] if st["shares"] else 0)
            flt = bool(st["shares"]) and bool(st["flags"] & FL_LAST_FLOAT)
            rows.append(dict(AgentID=a, AgentStrategy=tnames[a], EventType="FINAL_CASH_POSITION", Event=int(st["cash"])))
            rows.append(dict(AgentID=a, AgentStrategy=tnames[a], EventType="ENDING_CASH",
                             Event=float(mtm) if flt else int(mtm)))
            if f.kind:
                rows.append(dict(AgentID=a, AgentStrategy=tnames[a], EventType="FINAL_VALUATION",
                                 Event=int(f.valuation_int) if f.kind == 1 else float(f.valuation)))
        return rows

    def write_summary_log(self, env, log_dir):
        """Kernel.writeSummaryLog (Kernel.py:556-565): log_dir/summary_log.bz2, a pandas DataFrame
        pickled with bz2 compression, as cli/stats.py and cli/read_agent_logs.py read it."""
        import pandas as pd
        os.makedirs(log_dir, exist_ok=True)
        path = os.path.join(log_dir, "summary_log.bz2")
        pd.DataFrame(self.summary_log(env)).to_pickle(path, compression="bz2")
        return path

    # ---- the exchange's order-book outputs (mxabides.booklog)
    def book_log_records(self, env, partial=False):
        """env's raw book-update records (structured array t, price, qty; include/mxa.h); an
        overflowed log raises unless partial (then its first book_log records)"""
        if not self.book_log_cap:
            raise ValueError("created with book_log=0")
        from .booklog import REC_DTYPE
        buf = np.zeros(self.book_log_cap, dtype=REC_DTYPE)
        n = ctypes.c_int64()
        self._check(self.L.mxa_read_book_log(self._h, env, buf.ctypes.data, self.book_log_cap, ctypes.byref(n)),
                    "mxa_read_book_log")
        if n.value > self.book_log_cap and not partial:
            raise _lib.MxaError("env %d: book-update log overflow (%d records > book_log=%d)"
                                % (env, n.value, self.book_log_cap))
        return buf[:min(n.value, self.book_log_cap)]

    def book_log_rows(self, env):
        """OrderBook.book_log of env as flat rows (mxabides.booklog format: t, n, executed qty,
        average price, n (price, volume) pairs)"""
        from .booklog import rows_from_records
        return rows_from_records(self.book_log_records(env))

    @property
    def date(self):
        """the simulated date of the outputs' timestamps: the replay tape's, else the configs'"""
        from .booklog import SESSION_DATE
        if self.config in REPLAY_CONFIGS and getattr(self.tape, "date", None):
            return self.tape.date
        if self.composition is not None:  # its -d historical date
            import pandas as pd
            return pd.Timestamp(int(self.composition.date_ns), unit="ns").strftime("%Y-%m-%d")
        return SESSION_DATE

    def exchange_events(self, env):
        """the exchange's BEST_BID / BEST_ASK / LAST_TRADE log rows (OrderBook.py:114-141) as a
        DataFrame indexed by EventTime"""
        from .booklog import exchange_events_frame
        return exchange_events_frame(self.book_log_rows(env), self.symbol, self.date)

    def exchange_log(self, env):
        """ExchangeAgent.log of env (Agent.logEvent rows, Agent.py:97-110): [(EventTime ns since
        midnight or None, EventType, Event)], order Events as dicts (mxabides.booklog.exchange_log)"""
        from .booklog import exchange_log
        if not self.exchange_log_on:
            raise ValueError("created without exchange_log")
        return exchange_log(self.book_log_records(env), self.symbol, self._agent_type_names()[0])

    def exchange_log_frame(self, env):
        """the DataFrame Agent.kernelTerminating writes to EXCHANGE_AGENT.bz2 (Agent.py:86-95)"""
        from .booklog import exchange_log_frame
        return exchange_log_frame(self.exchange_log(env), self.date)

    def write_exchange_log(self, env, log_dir):
        """log_dir/<exchange name without spaces>.bz2 as Kernel.writeLog pickles it
        (Kernel.py:520-547): EXCHANGE_AGENT.bz2, or ExchangeAgent0.bz2 for an "Exchange Agent 0"."""
        os.makedirs(log_dir, exist_ok=True)
        path = os.path.join(log_dir, "%s.bz2" % self._agent_names()[0].replace(" ", ""))
        self.exchange_log_frame(env).to_pickle(path, compression="bz2")
        return path

    def orderbook_snapshots(self, env, wide_book=False):
        """ExchangeAgent.logOrderBookSnapshots' DataFrame with book_freq 0 (ORDERBOOK_<sym>_FULL)"""
        from .booklog import orderbook_full
        return orderbook_full(self.book_log_rows(env), self.date, wide_book=wide_book)

    def fundamental_log(self, env):
        """the oracle's f_log of env as the DataFrame fundamental_<sym>.bz2 holds, after Kernel.runner's
        kernelStopping pass (whose oracle observations it includes): the SparseMeanRevertingOracle's,
        or the ExternalFileOracle's of hist_fund_* (ExternalFileOracle.py:19, 97)"""
        from .booklog import fundamental_frame
        if self.config in REPLAY_CONFIGS:
            raise ValueError("config/marketreplay.py runs without an oracle (oracle=None): no f_log")
        if not getattr(self, "_finalized", False):
            self.finalize()
        return fundamental_frame(self.book_log_records(env), self.date, external=self.config in HIST_CONFIGS)

    def write_logs(self, env, log_dir, wide_book=False):
        """env's run directory as the reference writes it at termination (Kernel.writeLog /
        writeSummaryLog, Kernel.py:520-565; ExchangeAgent.kernelTerminating, ExchangeAgent.py:106-126):
        summary_log.bz2, fundamental_<sym>.bz2, with book_freq 0 ORDERBOOK_<sym>_FULL.bz2 (with book_freq
        None no order-book file) and, on a handle with the exchange log, the exchange's own log
        (EXCHANGE_AGENT.bz2; Agent.kernelTerminating, Agent.py:86-95), each a bz2-pickled DataFrame.
        Returns the paths."""
        if self.book_freq is not None and self.book_freq != 0:
            # "M" (rmsc01) goes through pd.date_range(..., closed="right"), which pandas 2 rejects,
            # and "all" (obi_rmsc02) is no pandas frequency: the reference raises in both
            raise NotImplementedError("book_freq %r: the resampled ORDERBOOK_%s_FREQ_* file is not restated"
                                      % (self.book_freq, self.symbol))
        os.makedirs(log_dir, exist_ok=True)
        paths = [self.write_summary_log(env, log_dir)]
        if self.config not in REPLAY_CONFIGS:  # config/marketreplay.py: oracle=None, no f_log
            f = self.fundamental_log(env)
            if not f.empty:  # ExchangeAgent.kernelTerminating writes only a non-empty frame
                p = os.path.join(log_dir, "fundamental_%s.bz2" % self.symbol)
                f.to_pickle(p, compression="bz2")
                paths.append(p)
        if self.exchange_log_on:
            paths.append(self.write_exchange_log(env, log_dir))
        if self.book_freq == 0:
            paths.append(self.write_orderbook_log(env, log_dir, wide_book))
        return paths

    def write_orderbook_log(self, env, log_dir, wide_book=False):
        """log_dir/ORDERBOOK_<sym>_FULL.bz2 as Kernel.writeLog pickles it (Kernel.py:537-547)"""
        os.makedirs(log_dir, exist_ok=True)
        path = os.path.join(log_dir, "ORDERBOOK_%s_FULL.bz2" % self.symbol)
        self.orderbook_snapshots(env, wide_book).to_pickle(path, compression="bz2")
        return path

    def close(self):
        if self._h:
            self.L.mxa_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
