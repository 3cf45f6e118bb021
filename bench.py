#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the rmsc03 market step on MI355X (BASELINE.json metric).

One env-step = one Kernel event pop in one env (the reference's ttl_messages,
Kernel.py:211, 321-326).  One bench "step" = one full episode (config build from seeds + the
whole session + stop-time tail, or a whole GymKernel episode) of every env on every GPU; the
per-env episode records (include/mxa.h mxa_write_records) are all-gathered over RCCL, the only
collective: envs are independent, so the batch shards with no data-path exchange (weak scaling,
`--envs` per GPU).  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--config rmsc03]

`--gpus N` without a launcher starts N rank processes itself (one per GPU, before anything
touches a GPU) with the same RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* environment that
`torch.distributed.run --nproc-per-node N` gives them; under such a launcher the world size
comes from WORLD_SIZE.  This replaces config/parallel.py:15-25 (one OS process per simulation).
`--stub` runs the same launcher, timing and all-gather on CPU (gloo) with a synthetic engine:
the harness self-test of tests/test_bench_launcher.py, never a bench number.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle")]

METRIC = "env-steps/sec (whole node), rmsc03 100-agent market ×4096 envs, 1/2/4/8 GPUs"
NOMINAL_BYTES_PER_EVENT = 256  # SURVEY.md §8(d) nominal figure (shown next to the counted one)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's bench size)")
    ap.add_argument("--config", default="rmsc03")
    ap.add_argument("--chunk", type=int, default=1 << 22, help="max pops per env per kernel launch")
    ap.add_argument("--ddqn-torch", action="store_true",
                    help="rmsc03_ddqn: the learner's per-period bookkeeping as PyTorch ops instead of "
                         "libmxa_ddqn.so's one kernel")
    ap.add_argument("--first-chunk", type=int, default=0,
                    help="Kernel.runner configurations: a first launch of this many pops, then launches of --chunk "
                         "over the envs still running (mxa_set_launch_schedule); 0 = launches of --chunk only. "
                         "Measured slower for every configuration (DESIGN.md Appendix R.6)")
    ap.add_argument("--cpu-envs", type=int, default=None, help="CPU-baseline sample size (envs)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU-baseline threads (default: the cores this process may run on, capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--per-step", action="store_true",
                    help="GymKernel configs: one launch per ABIDESEnv.step instead of one per episode")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample: at least this much wall time")
    ap.add_argument("--no-latency", action="store_true", help="skip the solo-latency run of the latency bound")
    ap.add_argument("--parity-hash", action="store_true",
                    help="also compute the per-pop parity hash (test instrumentation, off by default: "
                         "tests/test_gpu_hash_switch.py shows every market result is identical either way)")
    ap.add_argument("--ddqn-batch", type=int, default=32, help="rmsc03_ddqn: learner batch size (reference 32)")
    ap.add_argument("--tape", default=None, help="marketreplay tape under tests/golden (IBM_2003-01-14, GOOG_2012-06-21)")
    ap.add_argument("--stub", action="store_true", help="launcher self-test on CPU/gloo with a synthetic engine")
    ap.add_argument("--no-count", action="store_true",
                    help="skip the instrumented batch that counts the algorithmic bytes (PMC passes of "
                         "tools/profile_round.sh: only the timed kernel launches)")
    return ap.parse_args()


# scripts/rmsc03.sh:5-13: the options its sweep passes to config/rmsc03.py (--config rmsc03_sweep)
SWEEP_OPTIONS = dict(pov=0.05, min_order_size=25, window_size=5, num_ticks=50, wake_up_freq="10S")
DEFAULT_ENVS = {"marketreplay": 512, "sparse_zi_1000": 1024, "random_fund_value": 2048, "random_fund_diverse": 2048,
                "hist_fund_value": 2048, "hist_fund_diverse": 2048}
FUND = os.path.join(ROOT, "tests", "golden", "fund_JPM_20190628.npz")  # hist_fund_*: the JPM mid-price series


def composition_of(name):
    """--config cfg.NAME: the runtime composition of tests/golden/cfg_NAME_*.json (the agent list of
    gen_config_fixtures.py, e.g. cfg.rmsc03_n100_v20 = rmsc03 with 100 noise and 20 value agents)"""
    import glob
    from mxabides import composition
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "cfg_%s_*.json" % name.split(".", 1)[1])))
    files = [f for f in files if not f.endswith("_summary.json")]
    if not files:
        raise SystemExit("no composition %s under tests/golden" % name)
    with open(files[0]) as f:
        return composition.from_dict(json.load(f)["composition"])


# ----------------------------------------------------------------------------------------------
# rank processes
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """Start n rank processes of this same command (rank r on GPU r), wait for all, return the
    worst exit status.  Runs before this process touches any GPU; a rank that fails ends the
    others (their exact PIDs), so no rank waits forever in a collective."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or c
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


class Ctx:
    """this rank's place in the job (env of torch.distributed.run, or of spawn_ranks)"""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus > 1 and self.world != args.gpus:
            raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, self.world))
        self.stub = args.stub
        if self.stub:
            self.device = torch.device("cpu")
            backend = "gloo"
        else:
            torch.cuda.set_device(self.local)
            self.device = torch.device("cuda", self.local)
            backend = "nccl"  # RCCL over xGMI on ROCm
        if self.world > 1:
            kw = {} if self.stub else {"device_id": self.device}
            dist.init_process_group(backend, **kw)

    def sync(self):
        if not self.stub:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------
# engines: one full episode of this rank's envs per step, records written and all-gathered
class Engine:
    kernel = "?"
    launches = 0
    kernel_ms = 0.0

    def __init__(self, args, ctx):
        import torch
        from mxabides import shard
        self.args, self.ctx, self.torch, self.shard = args, ctx, torch, shard
        self.n = args.envs
        self.records = torch.zeros((self.n, shard.RECORD_WORDS), dtype=torch.int64, device=ctx.device)
        self.gathered = None
        self.last_batch = None
        self.errs = torch.zeros((), dtype=torch.int64, device=ctx.device)  # envs in error, every timed batch
        self.errs_warm = torch.zeros((), dtype=torch.int64, device=ctx.device)

    def seeds(self, k):
        return self.shard.env_seeds(k, self.ctx.rank, self.ctx.world, self.n)

    def gather(self, k, timed=False):
        self.last_batch = k
        self.gathered = self.shard.gather_records(self.records, self.ctx.world)
        # the same torch kernels in warmup and timed steps (their first launch loads code objects)
        e = (self.records[:, self.shard.R_STATUS] == 2).sum()
        if timed:
            self.errs += e
        else:
            self.errs_warm += e
        return self.records[:, self.shard.R_EVENTS].sum()

    def check_gathered(self):
        """rank 0: the gathered rows are in global env order (seed column) and hold this rank's
        own rows where they belong"""
        sh, g, n = self.shard, self.gathered, self.n
        own = bool((g[self.ctx.rank * n:(self.ctx.rank + 1) * n] == self.records).all())
        if not self.has_seeds:
            return {"own_rows_in_place": own}
        import numpy as np
        want = np.concatenate([sh.env_seeds(self.last_batch, r, self.ctx.world, n) for r in range(self.ctx.world)])
        got = g[:, sh.R_SEED].cpu().numpy().astype(np.uint32)
        return {"own_rows_in_place": own, "global_env_order": bool((got == want).all())}

    def env_errors(self):
        """envs that ended in an error over every timed batch of every rank (their events are
        counted like any other's: the reference's own crash paths end an env the same way)"""
        e = self.errs.clone()
        if self.ctx.world > 1:
            self.ctx.dist.all_reduce(e, op=self.ctx.dist.ReduceOp.SUM)
        return int(e.item())

    has_seeds = True


class StubEngine(Engine):
    """launcher self-test: records from the seeds, no market (CPU, gloo)"""
    kernel = "stub"

    def step(self, k, timed):
        torch, sh = self.torch, self.shard
        s = torch.from_numpy(self.seeds(k).astype("int64"))
        r = self.records
        r.zero_()
        r[:, sh.R_EVENTS] = 1000 + s % 997
        r[:, sh.R_HASH] = s * 31
        r[:, sh.R_STATUS] = 1
        r[:, sh.R_SEED] = s
        self.launches += 1
        return self.gather(k, timed)

    def describe(self):
        return {"metric": "launcher self-test (stub engine, no market)", "dtype": "int64", "data": "synthetic",
                "workload": "stub x%d envs per rank" % self.n}

    def algo_bytes(self):
        return None


class MarketEngine(Engine):
    """Kernel.runner configurations (VecMarket): one launch per env chunk until every env is done"""

    def __init__(self, args, ctx):
        super().__init__(args, ctx)
        import mxabides
        from mxabides.configs import REPLAY_CONFIGS
        from mxabides.fundamental import FundamentalSeries
        self.mx = mxabides
        kw = {"fundamental": FundamentalSeries.load(FUND)} if args.config.startswith("hist_fund") else {}
        self.tname = None
        if args.config in REPLAY_CONFIGS:  # config/marketreplay.py & co. replay a LOBSTER tape (--tape)
            from mxabides import tape
            self.tname = args.tape or "IBM_2003-01-14"
            kw["tape"] = tape.Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % self.tname))
            self.has_seeds = False  # nothing in these compositions draws
        cfg = args.config
        if cfg == "rmsc03_sweep":  # config/rmsc03.py with scripts/rmsc03.sh's --mm-* options in every env
            from mxabides.configs import mm_params
            kw["mm_params"] = mm_params(self.n, **SWEEP_OPTIONS)
            cfg = "rmsc03"
        self.composition = None
        if cfg.startswith("cfg."):  # a runtime composition of the reference-run fixtures (mxa_create_config)
            self.composition = composition_of(cfg)
            cfg = self.composition
        self.m = mxabides.VecMarket(cfg, self.seeds(0), device=ctx.local, **kw)
        self.stream = self.torch.cuda.Stream()  # a real stream object (the legacy default stream's handle is 0)
        self.torch.cuda.set_stream(self.stream)
        self.m.set_stream(self.stream.cuda_stream)
        self.m.set_parity_hash(args.parity_hash)
        self.m.set_launch_schedule(args.first_chunk)
        cid = (self.composition.base if self.composition is not None else mxabides.CONFIG_IDS[cfg]
               if args.config != "rmsc03_sweep" else mxabides._lib.MXA_RMSC03_MM)
        self.kernel = "mxa_run_kernel<%d> (%s%s)" % (cid, args.config,
                                                      ", specialised" if self.composition is not None else "")

    def step(self, k, timed):
        m = self.m
        m.set_seeds(self.seeds(k))
        m.reset()
        nl = m.run(chunk=self.args.chunk)
        if timed:
            self.launches += nl
            self.kernel_ms += m.last_kernel_ms
        m.write_records(self.records.data_ptr())
        return self.gather(k, timed)

    def count(self, k):
        """one batch of the timed workload (batch k's seeds) with the instrumentation on: the
        event-class counters of the algorithmic-byte count (mxabides.counters)"""
        m = self.m
        m.set_parity_hash(True)
        m.set_seeds(self.seeds(k))
        m.reset()
        m.run(chunk=self.args.chunk)
        c = m.counters()
        m.set_parity_hash(self.args.parity_hash)
        return c

    def describe(self):
        a, n = self.args, self.n
        metric = METRIC if a.config == "rmsc03" else "env-steps/sec, %s x%d envs per GPU" % (a.config, n)
        if a.config == "rmsc03_sweep":
            return {"metric": metric, "dtype": "int64", "data": "synthetic (per-env seeds; every input built on the device)",
                    "workload": "config/rmsc03.py with scripts/rmsc03.sh's options (--mm-pov 0.05 --mm-min-order-size 25 "
                                "--mm-window-size 5 --mm-num-ticks 50 --mm-wake-up-freq 10S) x%d envs per GPU, full "
                                "episode per step, seeds %d+global_env" % (n, self.shard.SEED0),
                    "agents_per_env": self.m.n_agents}
        if self.tname:
            return {"metric": metric + " (%s LOBSTER tape)" % self.tname, "dtype": "int64",
                    "data": "LOBSTER sample tape %s (every env replays it; nothing draws)" % self.tname,
                    "workload": "%s x%d envs per GPU, full Kernel.runner episode per step" % (a.config, n),
                    "agents_per_env": self.m.n_agents}
        return {"metric": metric, "dtype": "int64", "data": "synthetic (per-env seeds; every input built on the device)",
                "workload": "%s x%d envs per GPU, full episode per step (config build from seeds + the config's "
                            "session), seeds %d+global_env" % (a.config, n, self.shard.SEED0),
                "agents_per_env": self.m.n_agents}

    def cpu_baseline(self, threads, min_s):
        """the C oracle on `threads` host threads over whole episodes of this workload's seeds,
        batch after batch until at least min_s of wall time: (env-steps/s, sample text)"""
        import numpy as np
        import pyoracle
        if self.tname:  # identical envs: Kernel.runner episodes of the oracle, single-threaded
            cfg = self.args.config
            ev, sec, k = 0, 0.0, 0
            while sec < min_s:
                t0 = time.perf_counter()
                o = pyoracle.OracleReplayRunner(self.m.tape, symbol=self.m.symbol,
                                                twap=None if cfg == "marketreplay_runner" else cfg.endswith("_e"))
                o.run()
                sec += time.perf_counter() - t0
                ev += o.events
                k += 1
            return float(ev) / sec, "%d %s episodes on %s, C oracle (oracle/abides_oracle.c), 1 thread, %.1f s " \
                "wall (every env is the same episode)" % (k, cfg, self.tname, sec), 1
        k = self.args.cpu_envs or max(2 * threads, 256 if self.args.config in ("rmsc03", "sparse_zi_100", "value_noise")
                                      else 4 * threads)
        ev, sec, first = 0, 0.0, 0
        while sec < min_s:
            cseeds = ((self.shard.SEED0 + first + np.arange(k, dtype=np.int64)) & 0xFFFFFFFF).astype(np.uint32)
            if self.args.config == "rmsc03_sweep":
                cev, _, _, csec = pyoracle.run_batch_mm(cseeds, self.m.mm_params[:1].repeat(k), threads)
            elif self.composition is not None:
                cev, _, _, csec = pyoracle.run_batch_config(self.composition, cseeds, threads)
            else:
                cev, _, csec = pyoracle.run_batch(self.args.config, cseeds, threads)
            ev += int(cev.sum())
            sec += csec
            first += k
        return float(ev) / sec, "%d %s envs (seeds %d..%d), full episodes, C oracle (oracle/abides_oracle.c), " \
            "%d threads, %.1f s wall" % (first, self.args.config, self.shard.SEED0, self.shard.SEED0 + first - 1, threads,
                                        sec), threads

    def latency_bound(self):
        """SURVEY.md §8(d)'s latency bound: resident envs / the per-event latency of one env's
        serial chain, measured here on one env per CU (256 envs of this workload's seeds, so no
        wave shares its SIMD): the throughput if every resident wave kept its solo pace"""
        seeds = self.seeds(0)[:256]
        kw = {"mm_params": self.m.mm_params[:256]} if getattr(self.m, "mm_params", None) is not None else {}
        if self.args.config.startswith("hist_fund"):
            kw["fundamental"] = self.m.fundamental
        if self.tname:
            kw["tape"] = self.m.tape
        s = self.mx.VecMarket(self.composition if self.composition is not None else self.m.config, seeds,
                              device=self.ctx.local, **kw)
        s.set_stream(self.stream.cuda_stream)
        s.set_parity_hash(self.args.parity_hash)
        s.run(chunk=self.args.chunk)
        ms = s.last_kernel_ms
        ev = s.summary()["events"]
        s.close()
        ns = ms * 1e6 / max(1, int(ev.max()))  # the longest env's chain sets the launch's length
        res = self.m.resident_envs
        return {"resident_envs": res, "solo_envs": len(seeds), "solo_kernel_ms": ms, "solo_ns_per_event": ns,
                "bound_env_steps_per_s": res / (ns * 1e-9),
                "how": "256 envs (one per CU) of this workload's seeds: kernel time / the longest env's events; "
                       "resident envs = run-kernel occupancy x CUs (mxa_resident_envs)"}


class GymEngine(Engine):
    """GymKernel handles (rmsc03 + DummyRL from seeds, or the ABIDESEnv replay on a tape): a full
    episode of ABIDESEnv.step calls with device-drawn actions (x ~ U(0, 0.01), level shares
    U(0, 1), torch Philox per rank) through mxa_step_device, nothing crossing PCIe"""

    def __init__(self, args, ctx):
        super().__init__(args, ctx)
        torch = self.torch
        from mxabides import tape
        from mxabides.gym import ACTION_SIZE, OBS_SIZE, VecABIDESEnv
        self.replay = args.config == "marketreplay"
        if self.replay:
            self.tname = args.tape or "IBM_2003-01-14"
            self.tp = tape.Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % self.tname))
            self.v = VecABIDESEnv(self.tp, self.n, device=ctx.local)
            self.n_steps = 761  # pd.date_range(09:40, 16:00, freq="30S")
            self.has_seeds = False
        else:
            self.v = VecABIDESEnv(seeds=self.seeds(0), device=ctx.local)
            self.n_steps = 27  # pd.date_range(09:31, 09:44, "30S")
        self.stream = torch.cuda.Stream()
        torch.cuda.set_stream(self.stream)
        self.v.set_stream(self.stream.cuda_stream)
        self.v.set_parity_hash(args.parity_hash)
        self.gen = torch.Generator(device="cuda")
        self.gen.manual_seed(1000 + ctx.rank)
        self.act = torch.empty((self.n_steps, self.n, ACTION_SIZE), dtype=torch.float64, device="cuda")
        # the episode's actions are drawn up front, so its steps go to the device in one launch
        # (mxa_step_many: every step the same code and results as a one-step launch); --per-step
        # launches them one by one
        self.many = not args.per_step
        k = self.n_steps if self.many else 1
        self.obs = torch.empty((k, self.n, OBS_SIZE), dtype=torch.float64, device="cuda")
        self.flags = torch.empty((k, self.n), dtype=torch.int32, device="cuda")
        self.ev_pairs = []
        self.kernel = "mxa_step_kernel<%d> (%s%s)" % (3 if self.replay else 4, args.config,
                                                      ", %d steps per launch" % self.n_steps if self.many else "")

    def step(self, k, timed):
        torch = self.torch
        self.v.reset(seeds=None if self.replay else self.seeds(k))
        torch.rand(self.act.shape, generator=self.gen, dtype=torch.float64, device="cuda", out=self.act)
        self.act[:, :, 0] *= 0.01
        for i in range(1 if self.many else self.n_steps):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(self.stream)
            if self.many:
                self.v.step_many_device(self.n_steps, self.act.data_ptr(), self.obs.data_ptr(), self.flags.data_ptr())
            else:
                self.v.step_device(self.act[i].data_ptr(), self.obs.data_ptr(), self.flags.data_ptr())
            if timed:
                e1.record(self.stream)
                self.ev_pairs.append((e0, e1))
        self.v.write_records(self.records.data_ptr())
        return self.gather(k, timed)

    def finish_timing(self):
        kms = [a.elapsed_time(b) for a, b in self.ev_pairs]
        self.launches, self.kernel_ms = len(kms), sum(kms)

    def count(self, k):
        """one more episode of the same workload (batch k's seeds, fresh actions of the same
        distribution) with the instrumentation on: the algorithmic-byte counters"""
        self.v.set_parity_hash(True)
        self.step(k, False)
        self.ctx.sync()
        c = self.v.counters()
        self.v.set_parity_hash(self.args.parity_hash)
        return c

    def describe(self):
        n = self.n
        if self.replay:
            return {"metric": "env-steps/sec, ABIDESEnv market replay (%s LOBSTER tape) x%d envs per GPU" % (self.tname, n),
                    "dtype": "int64", "data": "LOBSTER sample tape %s + device-drawn actions x~U(0,0.01), shares~U(0,1)"
                    % self.tname, "workload": "marketreplay x%d envs per GPU, full episode (reset + %d ABIDESEnv.step) "
                    "per bench step" % (n, self.n_steps), "tape_records": len(self.tp)}
        return {"metric": "env-steps/sec, rmsc03 + DummyRL execution agent (GymKernel) x%d envs per GPU" % n,
                "dtype": "int64", "data": "synthetic (seeds) + device-drawn actions x~U(0,0.01), shares~U(0,1)",
                "workload": "rmsc03_rl x%d envs per GPU, full episode (config build + %d ABIDESEnv.step) per bench "
                            "step, seeds %d+global_env" % (n, self.n_steps, self.shard.SEED0),
                "agents_per_env": self.v.n_agents}

    def gym_steps(self):
        return self.n * self.ctx.world * self.n_steps

    def latency_bound(self):
        """SURVEY.md §8(d)'s latency bound for the step kernel: resident envs / the per-event
        latency of one env's serial chain, measured on one env per CU (256 envs, a full episode of
        the same action distribution, step kernels timed on the handle's stream)"""
        torch = self.torch
        from mxabides.gym import ACTION_SIZE, OBS_SIZE, VecABIDESEnv
        n = 256
        s = (VecABIDESEnv(self.tp, n, device=self.ctx.local) if self.replay else
             VecABIDESEnv(seeds=self.seeds(0)[:n], device=self.ctx.local))
        s.set_stream(self.stream.cuda_stream)
        s.set_parity_hash(self.args.parity_hash)
        g = torch.Generator(device="cuda")
        g.manual_seed(7)
        act = torch.rand((self.n_steps, n, ACTION_SIZE), generator=g, dtype=torch.float64, device="cuda")
        act[:, :, 0] *= 0.01
        obs = torch.empty((n, OBS_SIZE), dtype=torch.float64, device="cuda")
        flags = torch.empty((n,), dtype=torch.int32, device="cuda")
        s.reset()
        pairs = []
        for i in range(self.n_steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
            s.step_device(act[i].data_ptr(), obs.data_ptr(), flags.data_ptr())
            e1.record(self.stream)
            pairs.append((e0, e1))
        self.stream.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in pairs)
        ev = s.summary()["events"]
        s.close()
        ns = ms * 1e6 / max(1, int(ev.max()))
        res = self.v.resident_envs
        return {"resident_envs": res, "solo_envs": n, "solo_kernel_ms": ms, "solo_ns_per_event": ns,
                "bound_env_steps_per_s": res / (ns * 1e-9),
                "how": "256 envs (one per CU), one episode of %d step launches: summed step-kernel time / the "
                       "longest env's events; resident envs = step-kernel occupancy x CUs, at most the "
                       "workload's envs (mxa_resident_envs)" % self.n_steps}

    def cpu_baseline(self, threads, min_s):
        import numpy as np
        import pyoracle
        k = self.args.cpu_envs or (4 * threads if self.replay else 16 * threads)
        ev, sec, first, b = 0, 0.0, 0, 0
        while sec < min_s:
            rs = np.random.RandomState(b)
            acts = rs.uniform(0, 1, (self.n_steps, k, 3))
            acts[:, :, 0] *= 0.01
            if self.replay:
                r = pyoracle.gym_batch(acts, threads, tape=self.tp)
            else:
                sd = ((self.shard.SEED0 + first + np.arange(k, dtype=np.int64)) & 0xFFFFFFFF).astype(np.uint32)
                r = pyoracle.gym_batch(acts, threads, seeds=sd)
            ev += int(r["events"].sum())
            sec += r["seconds"]
            first += k
            b += 1
        what = ("%d %s episodes" % (first, self.tname) if self.replay else
                "%d rmsc03_rl episodes (seeds %d..%d)" % (first, self.shard.SEED0, self.shard.SEED0 + first - 1))
        return float(ev) / sec, "%s, U(0, 0.01) actions, C oracle GymKernel batch (oracle/abides_oracle.c " \
            "ora_gym_batch), %d threads, %.1f s wall" % (what, threads, sec), threads


class DDQNEngine(Engine):
    """rmsc03 + DummyRL with the DDQN execution learner in the loop (mxabides.ddqn): actions from
    the shared Q-network (epsilon-greedy), transitions to the device replay ring, a training
    update every 5 periods as the reference agent does.  Learner state persists across steps."""

    def __init__(self, args, ctx):
        super().__init__(args, ctx)
        from mxabides import ddqn
        from mxabides.gym import VecABIDESEnv
        torch = self.torch
        self.ddqn = ddqn
        self.v = VecABIDESEnv(seeds=self.seeds(0), device=ctx.local)
        self.stream = torch.cuda.Stream()
        torch.cuda.set_stream(self.stream)
        self.v.set_stream(self.stream.cuda_stream)
        self.v.set_parity_hash(args.parity_hash)
        # one policy for the node: synchronous data parallelism over the ranks (gradient all-reduce
        # per update, rank 0's initialisation; mxabides.ddqn module docstring)
        group = ctx.dist.group.WORLD if ctx.world > 1 else None
        self.learner = ddqn.DDQNLearner(device="cuda", seed=1000 + ctx.rank, batch_size=args.ddqn_batch, group=group)
        self.task = ddqn.ExecutionTask(device="cuda")
        self.timing = []
        self.env_steps = torch.zeros((), dtype=torch.int64, device="cuda")
        self.learns0 = 0
        self.kernel = "mxa_step_kernel<4> (rmsc03_rl)"

    def step(self, k, timed):
        sh = self.shard
        if timed and not self.timing:
            self.learns0 = self.learner.learn_step_counter
        r = self.ddqn.run_episode(self.v, self.learner, self.task, seeds=self.seeds(k),
                                  timing=self.timing if timed else None, fused=not self.args.ddqn_torch)
        if timed:
            self.env_steps += r["env_steps"].sum()
        self.v.write_records(self.records.data_ptr())
        # word R_RETURN: the learner's per-env episode return (float64 bits)
        self.records[:, sh.R_RETURN] = r["returns"].to(self.torch.float64).view(self.torch.int64)
        return self.gather(k, timed)

    def finish_timing(self):
        kms = [a.elapsed_time(b) for a, b in self.timing]
        self.launches, self.kernel_ms = len(kms), sum(kms)

    def count(self, k):
        """one more learner-driven episode (batch k's seeds) with the instrumentation on (rank 0
        only, after the timed region: its updates stay local, no collective)"""
        self.v.set_parity_hash(True)
        world, self.learner.world = self.learner.world, 1
        try:
            self.ddqn.run_episode(self.v, self.learner, self.task, seeds=self.seeds(k))
        finally:
            self.learner.world = world
        self.ctx.sync()
        c = self.v.counters()
        self.v.set_parity_hash(self.args.parity_hash)
        return c

    def describe(self):
        n = self.n
        return {"metric": "env-steps/sec, rmsc03 + DDQN execution learner (GymKernel) x%d envs per GPU" % n,
                "dtype": "int64 (market), fp32 (Q-network)", "data": "synthetic (seeds); actions from the DDQN learner",
                "workload": "rmsc03_rl x%d envs per GPU + DDQN learner (NNModel_1, batch %d, train every 5 periods), "
                            "full episode per bench step, seeds %d+global_env" % (n, self.args.ddqn_batch, self.shard.SEED0),
                "agents_per_env": self.v.n_agents, "learn_steps": self.learner.learn_step_counter - self.learns0,
                "learner_period": "torch ops" if self.args.ddqn_torch or self.ddqn.period_lib() is None
                else "one kernel (libmxa_ddqn.so, include/mxa_ddqn.h)"}

    def gym_steps(self):
        return int(self.env_steps.item()) * self.ctx.world  # every rank steps its own envs alike

    def cpu_baseline(self, threads, min_s):
        """the market side on the host: the same rmsc03 + DummyRL GymKernel composition in the C
        oracle under random actions (no learner on the host side)"""
        g = GymEngine.__new__(GymEngine)
        g.args, g.shard, g.replay, g.n_steps = self.args, self.shard, False, 27
        v, sample, th = GymEngine.cpu_baseline(g, threads, min_s)
        return v, sample + "; market only, the learner is not part of the CPU figure", th


# ----------------------------------------------------------------------------------------------
def traffic_record(config, envs, parity_hash, tape=None):
    """HBM bytes per run-kernel launch from the PMC record of THIS build (profiles/hbm_traffic_<config>.json,
    written by tools/hbm_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
    this same bench command).  A record is attached only when its build id (mxa_build_id(): a hash
    of the kernel sources and flags), config, env count and parity-hash setting all match the
    running bench; otherwise traffic is null and traffic_record says why."""
    import mxabides
    name = config if tape in (None, "IBM_2003-01-14") else "%s_%s" % (config, tape)  # a replay tape's own record
    prof = os.path.join(ROOT, "profiles", "hbm_traffic_%s.json" % name)
    if not os.path.exists(prof):
        return None, {"file": None, "match": False, "why": "no PMC record for this config"}
    with open(prof) as f:
        p = json.load(f)
    bid = mxabides.build_id()
    src = {"file": os.path.relpath(prof, ROOT), "build_id": p.get("build_id"), "running_build_id": bid}
    why = []
    if p.get("build_id") != bid:
        why.append("measured on another build")
    if p.get("config") != config or p.get("envs") != envs:
        why.append("other workload")
    if config == "marketreplay" and p.get("tape", "IBM_2003-01-14") != (tape or "IBM_2003-01-14"):
        why.append("other tape")  # records without a tape field were measured on the default tape
    if bool(p.get("parity_hash")) != parity_hash:
        why.append("parity hash setting differs")
    src["match"] = not why
    if why:
        src["why"] = "; ".join(why)
        return None, src
    return p.get("bytes_per_launch"), src


def issue_record(config, envs, parity_hash, tape=None):
    """The dominant kernel's instruction issue rates from the SQ counter record of THIS build
    (profiles/issue_<config>.json, tools/sq_counters.sh + tools/issue_summary.py: separate rocprofv3
    --pmc passes of this bench command): instructions of each type per CU per elapsed cycle.  A CU
    issues at most one instruction of a type per cycle (one scalar unit per CU), so SALU near 1.0
    means the scalar unit bounds the kernel.  Matched like traffic_record."""
    import mxabides
    name = config if tape in (None, "IBM_2003-01-14") else "%s_%s" % (config, tape)
    prof = os.path.join(ROOT, "profiles", "issue_%s.json" % name)
    if not os.path.exists(prof):
        return None
    with open(prof) as f:
        p = json.load(f)
    bid = mxabides.build_id()
    ok = (p.get("build_id") == bid and p.get("config") == config and p.get("envs") == envs
          and bool(p.get("parity_hash")) == parity_hash)
    out = {"record": os.path.relpath(prof, ROOT), "build_id": p.get("build_id"), "match": ok}
    if ok:
        out["per_cu_cycle"] = p["per_cu_cycle"]
        out["per_event"] = p["per_event"]
        out["ceiling"] = "1.0 instruction of a type per CU per cycle"
    return out


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    phys = set()
    try:  # distinct (package, core) pairs: the physical cores of the host
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                t = os.path.join(base, d, "topology")
                with open(os.path.join(t, "physical_package_id")) as f1, open(os.path.join(t, "core_id")) as f2:
                    phys.add((f1.read().strip(), f2.read().strip()))
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": avail, "cpu_model": model,
            "physical_cores": len(phys) or os.cpu_count()}


def cpu_threads(args, info):
    if args.cpu_threads:
        return args.cpu_threads
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(info["affinity_cpus"], omp) if omp > 0 else info["affinity_cpus"])


def main():
    args = parse()
    if args.envs is None:
        args.envs = 4 if args.stub else DEFAULT_ENVS.get(args.config, 4096)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))  # before anything touches a GPU
    ctx = Ctx(args)
    torch = ctx.torch
    if args.stub:
        eng = StubEngine(args, ctx)
    elif args.config in ("marketreplay", "rmsc03_rl"):
        eng = GymEngine(args, ctx)
    elif args.config == "rmsc03_ddqn":
        eng = DDQNEngine(args, ctx)
    else:
        eng = MarketEngine(args, ctx)

    dev = ctx.device
    evw = torch.zeros((), dtype=torch.int64, device=dev)
    for k in range(args.warmup):  # the timed loop's exact ops (first launches of torch's kernels included)
        evw += eng.step(k, False)
    ctx.sync()
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    ev = torch.zeros((), dtype=torch.int64, device=dev)
    for k in range(args.warmup, args.warmup + args.steps):
        ev += eng.step(k, True)
    ctx.sync()
    ctx.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if ctx.world > 1:
        ctx.dist.all_reduce(el, op=ctx.dist.ReduceOp.MAX)
        ctx.dist.all_reduce(ev, op=ctx.dist.ReduceOp.SUM)
    elapsed, events = float(el.item()), int(ev.item())
    if hasattr(eng, "finish_timing"):
        eng.finish_timing()
    chk = eng.check_gathered() if ctx.rank == 0 else None
    n_err = eng.env_errors()

    if ctx.rank == 0:
        d = eng.describe()
        out = {"metric": d["metric"], "value": events / elapsed, "unit": "env-steps/s", "n_gpus": ctx.world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": d["dtype"], "data": d["data"],
               "config": {"workload": d["workload"], "envs_per_gpu": eng.n, "global_envs": eng.n * ctx.world,
                          "events_per_step": events / args.steps, "parallelism": "envs sharded, dp%d" % ctx.world,
                          "parity_hash": bool(args.parity_hash), "env_errors": n_err, "gathered_records": chk}}
        for key in ("agents_per_env", "tape_records", "learn_steps", "learner_period"):
            if key in d:
                out["config"][key] = d[key]
        if isinstance(eng, GymEngine):
            out["config"]["steps_per_launch"] = eng.n_steps if eng.many else 1
        if hasattr(eng, "gym_steps"):
            out["config"]["gym_steps_per_s"] = eng.gym_steps() * (args.steps if not isinstance(eng, DDQNEngine) else 1) / elapsed
        if not args.stub:
            out["config"]["device"] = torch.cuda.get_device_name(ctx.local)
            out["config"]["cus"] = torch.cuda.get_device_properties(ctx.local).multi_processor_count
            avg_ms = eng.kernel_ms / max(1, eng.launches)
            my_ev_per_launch = events / ctx.world / max(1, eng.launches)
            from mxabides import counters as mc
            if args.no_count:
                bpe, bparts, bunits = float(NOMINAL_BYTES_PER_EVENT), None, None
            else:
                eng.last_counters = eng.count(args.warmup)
                bpe, bparts, bunits = mc.bytes_per_event(eng.last_counters)
            achieved = bpe * my_ev_per_launch / (avg_ms * 1e-3) / 1e9
            # (the DDQN line's record is a PMC pass of the same bench command: its step kernel)
            traffic, tsrc = traffic_record(args.config, eng.n, bool(args.parity_hash), args.tape)
            out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_record": tsrc,
                               "kernel": eng.kernel, "avg_launch_ms": avg_ms, "launches": eng.launches,
                               "algo_bytes_per_event": bpe, "algo_bytes_source": "nominal (--no-count)" if args.no_count else
                               "counted: device event-class counters of one instrumented batch of this workload "
                               "(mxabides/counters.py, SURVEY.md §8(d) unit sizes)",
                               "algo_bytes_breakdown": bparts, "algo_units_per_event": bunits,
                               "nominal_bytes_per_event": NOMINAL_BYTES_PER_EVENT}
            if traffic:
                out["roofline"]["traffic_per_event"] = traffic / my_ev_per_launch
            iss = issue_record(args.config, eng.n, bool(args.parity_hash), args.tape)
            if iss:
                out["roofline"]["issue"] = iss
            if not args.no_count:
                strict = mc.strict_bytes_per_event(eng.last_counters)
                a_strict = strict * my_ev_per_launch / (avg_ms * 1e-3) / 1e9
                out["roofline"]["strict"] = {
                    "algo_bytes_per_event": strict, "achieved": a_strict, "frac": a_strict / HBM_PEAK_GBS,
                    "rule": "SURVEY.md §8(d) read literally: 2 x 64 B agent record on every pop (the counted figure "
                            "charges it only where an event loads the recipient's state)"}
            if hasattr(eng, "latency_bound") and not args.no_latency:
                lb = eng.latency_bound()
                lb["achieved_env_steps_per_s"] = my_ev_per_launch / (avg_ms * 1e-3)
                lb["frac"] = lb["achieved_env_steps_per_s"] / lb["bound_env_steps_per_s"]
                out["roofline"]["latency_bound"] = lb
            if not args.no_cpu and hasattr(eng, "cpu_baseline"):
                info = host_info()
                th = cpu_threads(args, info)
                v, sample, used = eng.cpu_baseline(th, args.cpu_seconds)
                v1, sample1, _ = eng.cpu_baseline(1, min(5.0, args.cpu_seconds))
                phys = info["physical_cores"]
                out["cpu_baseline"] = {
                    "value": v, "unit": "env-steps/s", "cores": used, "kind": "port", "sample": sample, "per_core": v / used,
                    "single_thread": {"value": v1, "sample": sample1},
                    "physical_cores_extrapolated": {
                        "value": v1 * phys, "cores": phys,
                        "how": "single-thread figure x physical cores (SMT siblings not counted); NOT measured: a "
                               "GPU box grants this process %d CPUs, so the host's other cores are not ours to load; "
                               "the %d-thread figure / (%d x single-thread) = %.2f is the scaling seen up to that "
                               "share" % (used, used, used, v / (used * v1))},
                    **info}
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
