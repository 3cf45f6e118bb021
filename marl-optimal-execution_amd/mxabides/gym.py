"""ABIDESEnv on MI355X: the Gym surface of the reference (ABIDESEnv.py:7-57) over libmxa.

`VecABIDESEnv` steps n independent copies of the reference's ABIDESEnv composition
(ExchangeAgent + MarketReplayAgent on a LOBSTER tape + DummyRLExecutionAgent, with the
GymKernel step loop) in one kernel launch per step; envs differ by the actions they are fed.
With `tape=None, seeds=[...]` it steps the rmsc03 + DummyRL composition instead (BASELINE.json
configs[3]): rmsc03's 64 agents from each env's seed plus DummyRLExecutionAgent 64 under the
same GymKernel step loop (libmxa config MXA_RMSC03_RL).
`ABIDESEnv` is the single-env drop-in with the reference's signature and return values:
reset() -> None, step(action) -> (obs float64[9] or [] , reward None, done 0|1, info None).
"""
import ctypes
import os

import numpy as np

from . import _lib
from .tape import Tape, load_lobster

OBS_SIZE = 9      # get_observation returns 9 values (the declared space says 10: dummy_rl:317-322)
ACTION_SIZE = 3   # order_level 2 -> [total volume, level-1 share, level-2 share]
RL_STATE_WORDS = 8  # mxa_write_rl_state row (include/mxa.h MXA_RL_STATE_WORDS)


class VecABIDESEnv:
    def __init__(self, tape=None, n_envs=None, device=0, trace_cap=0, seeds=None):
        self.L = _lib.load()
        self.tape = tape
        self.trace_cap = trace_cap
        self._h = ctypes.c_void_p()
        if tape is None:  # rmsc03 + DummyRL, one env per seed
            if seeds is None:
                raise TypeError("either a Tape or seeds (rmsc03 + DummyRL) is required")
            sd = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
            if n_envs is not None and int(n_envs) != len(sd):
                raise ValueError("n_envs must equal len(seeds)")
            self.n_envs = len(sd)
            rc = self.L.mxa_create(_lib.MXA_RMSC03_RL, self.n_envs, sd.ctypes.data, device, trace_cap,
                                   ctypes.byref(self._h))
            self._check(rc, "mxa_create")
        else:
            if not isinstance(tape, Tape):
                raise TypeError("tape must be an mxabides.tape.Tape")
            self.n_envs = int(n_envs)
            rc = self.L.mxa_create_replay(tape.t.ctypes.data, tape.oid.ctypes.data, tape.price.ctypes.data,
                                          tape.size.ctypes.data, tape.buy.ctypes.data, len(tape), self.n_envs, device,
                                          trace_cap, ctypes.byref(self._h))
            self._check(rc, "mxa_create_replay")
        self.n_agents = self.L.mxa_n_agents(self._h)
        self.obs = np.zeros((self.n_envs, OBS_SIZE), dtype=np.float64)
        self.flags = np.zeros(self.n_envs, dtype=np.int32)

    def _check(self, rc, what):
        if rc < 0:
            msg = self.L.mxa_last_error(self._h).decode() if self._h else ""
            raise _lib.MxaError("%s failed (%d): %s" % (what, rc, msg))
        return rc

    def reset(self, seeds=None):
        """ABIDESEnv.reset for every env (ABIDESEnv.py:51-57).  Each env is one process running
        consecutive episodes: Order.order_id / Order._order_ids carry over from its previous
        episode (util/order/Order.py:8-9) unless
        set_id_persistence(False) made every reset a fresh process."""
        if seeds is not None:  # rmsc03 + DummyRL: new per-env seeds
            sd = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
            self._check(self.L.mxa_set_seeds(self._h, sd.ctypes.data), "mxa_set_seeds")
        self._check(self.L.mxa_reset(self._h, None), "mxa_reset")
        self.obs[:] = 0
        self.flags[:] = 0

    def set_id_persistence(self, on):
        """True (default): resets continue each env's order ids (one process); False: every
        reset starts a fresh process (ids from 0)"""
        self._check(self.L.mxa_set_id_persistence(self._h, 1 if on else 0), "mxa_set_id_persistence")

    def step(self, actions):
        """actions [n][3] -> (obs [n][9], done [n] bool, valid [n] bool, error [n] bool)"""
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.float64).reshape(self.n_envs, ACTION_SIZE))
        self._check(self.L.mxa_step(self._h, a.ctypes.data, self.obs.ctypes.data, self.flags.ctypes.data), "mxa_step")
        f = self.flags
        return self.obs.copy(), (f & 1) != 0, (f & 2) != 0, (f & 4) != 0

    def step_device(self, d_actions, d_obs, d_flags):
        """Asynchronous step on device buffers (e.g. torch tensors' data_ptr())."""
        self._check(self.L.mxa_step_device(self._h, ctypes.c_void_p(d_actions), ctypes.c_void_p(d_obs),
                                           ctypes.c_void_p(d_flags)), "mxa_step_device")

    def step_many_device(self, k, d_actions, d_obs, d_flags):
        """k steps in one asynchronous launch with the actions given up front: device buffers
        actions [k][n][3] -> obs [k][n][9], flags [k][n] (include/mxa.h mxa_step_many); step i
        equals the i-th of k step_device calls"""
        self._check(self.L.mxa_step_many(self._h, int(k), ctypes.c_void_p(d_actions), ctypes.c_void_p(d_obs),
                                         ctypes.c_void_p(d_flags)), "mxa_step_many")

    def set_parity_hash(self, on):
        """Per-pop parity hash (summary()["hash"]) on or off; market results are identical
        either way (include/mxa.h mxa_set_parity_hash)."""
        self._check(self.L.mxa_set_parity_hash(self._h, 1 if on else 0), "mxa_set_parity_hash")

    def set_stream(self, stream_ptr):
        """Step on an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream)."""
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

    def write_rl_state(self, device_ptr):
        """Per-env execution-agent state [n][RL_STATE_WORDS] float64 (CASH, holdings, executed,
        best bid, best ask, bid size, ask size, lob flags) into device memory, asynchronously."""
        self._check(self.L.mxa_write_rl_state(self._h, ctypes.c_void_p(device_ptr)), "mxa_write_rl_state")

    def summary(self):
        n = self.n_envs
        buf = (_lib.EnvSummary * n)()
        self._check(self.L.mxa_read_summary(self._h, buf), "mxa_read_summary")
        return {"events": np.array([b.events for b in buf], dtype=np.int64),
                "hash": np.array([b.hash for b in buf], dtype=np.uint64),
                "status": np.array([b.status for b in buf], dtype=np.int32),
                "err": np.array([b.err for b in buf], dtype=np.int32),
                "current_time": np.array([b.current_time for b in buf], dtype=np.int64),
                "order_counter": np.array([b.order_counter for b in buf], dtype=np.int64)}

    def agents(self, env):
        n = self.n_agents
        buf = (_lib.AgentState * n)()
        self._check(self.L.mxa_read_agents(self._h, env, buf, n), "mxa_read_agents")
        return [(b.cash, b.shares, b.n_open) for b in buf]

    def book(self, env, side):
        """levels best-first, FIFO within level: [[order_id, agent_id, qty, price], ...] per level"""
        n = self._check(self.L.mxa_read_book(self._h, env, side, None, 0), "mxa_read_book")
        buf = np.zeros((max(n, 1), 4), dtype=np.int64)
        self._check(self.L.mxa_read_book(self._h, env, side, buf.ctypes.data, n), "mxa_read_book")
        levels = []
        for o in buf[:n].tolist():
            if levels and levels[-1][0][3] == o[3]:
                levels[-1].append(o)
            else:
                levels.append([o])
        return levels

    def trace(self, env):
        out = np.zeros((self.trace_cap, 10), dtype=np.int64)
        n = ctypes.c_int64()
        self._check(self.L.mxa_read_trace(self._h, env, out.ctypes.data, self.trace_cap, ctypes.byref(n)),
                    "mxa_read_trace")
        return out[:n.value]

    @property
    def last_kernel_ms(self):
        return self.L.mxa_last_kernel_ms(self._h)

    @property
    def resident_envs(self):
        """envs resident on the device at once (step-kernel occupancy x CUs, at most n_envs;
        include/mxa.h mxa_resident_envs)"""
        return self._check(self.L.mxa_resident_envs(self._h), "mxa_resident_envs")

    def close(self):
        if self._h:
            self.L.mxa_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Box:
    """What a learner reads of the reference's gym.spaces.Box (ABIDESEnv.py:22-26; gym is not a
    dependency here): low, high, shape, dtype (float32 as gym's default), sample(), contains(),
    seed().  gym.spaces.Box(low, high) itself is used when gym is importable."""

    def __init__(self, low, high, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self.low = np.asarray(low, dtype=self.dtype)
        self.high = np.asarray(high, dtype=self.dtype)
        assert self.low.shape == self.high.shape
        self.shape = self.low.shape
        self._rs = np.random.RandomState()

    def seed(self, seed=None):
        self._rs = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        return self._rs.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    __contains__ = contains

    def __repr__(self):
        return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)


def _box(low, high):
    try:
        import gym
        return gym.spaces.Box(np.array(low), np.array(high))
    except ImportError:
        return Box(low, high)


class ABIDESEnv:
    """Drop-in for the reference ABIDESEnv(ticker, date, log_dir=None, seed=None) on a LOBSTER
    message file `data/lobster/LOBSTER_SampleFile_{ticker}_1/{ticker}_{date}_34200000_57600000_message_1.csv`
    under `data_root` (agent_config.py:57-60), or on an explicit Tape."""

    def __init__(self, ticker, date, log_dir=None, seed=None, data_root=".", tape=None, device=0):
        if tape is None:
            f = "%s_%s_34200000_57600000_message_1.csv" % (ticker, date)
            tape = load_lobster(os.path.join(data_root, "data", "lobster", "LOBSTER_SampleFile_%s_1" % ticker, f), date,
                                symbol=ticker)
        self.ticker, self.date, self.log_dir = ticker, date, log_dir
        self.seed = np.random.randint(low=0, high=2 ** 31 - 1) if seed is None else seed  # agents draw nothing
        self._v = VecABIDESEnv(tape, 1, device=device)
        self.action_space = _box([0.0] * ACTION_SIZE, [1.0] * ACTION_SIZE)
        self.observation_space = _box([0] * 10, [0] * 10)  # as declared by the reference (ABIDESEnv.py:23)
        self._obs = []

    def reset(self):
        self._v.reset()
        self._obs = []

    def step(self, action):
        obs, done, valid, err = self._v.step(np.asarray(action, dtype=np.float64).reshape(1, ACTION_SIZE))
        if err[0]:
            s = self._v.summary()
            raise _lib.MxaError("env error: %s" % _lib.ERR_NAMES.get(int(s["err"][0]), s["err"][0]))
        if valid[0]:
            self._obs = obs[0]
        return self._obs, None, int(done[0]), None
