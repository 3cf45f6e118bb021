#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the rmsc03 market step on MI355X (BASELINE.json metric).

One env-step = one Kernel event pop in one env (the reference's ttl_messages,
Kernel.py:211, 321-326).  One bench "step" = one full rmsc03 episode (config build from
seeds + the whole 15-minute session + stop-time tail) of every env on every GPU; the
per-env episode records are all-gathered over RCCL (the only collective: envs are
independent, so the batch shards with no data-path exchange — weak scaling, 4096 envs
per GPU).  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--config rmsc03]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle")]

import numpy as np
import torch
import torch.distributed as dist

import mxabides
from mxabides import shard

METRIC = "env-steps/sec (whole node), rmsc03 100-agent market ×4096 envs, 1/2/4/8 GPUs"
SEED0 = shard.SEED0
ALGO_BYTES_PER_EVENT = 256  # nominal algorithmic HBM bytes per event
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def traffic_record(config, envs, parity_hash):
    """HBM bytes per run-kernel launch from the PMC record of THIS build (profiles/hbm_traffic_<config>.json,
    written by tools/hbm_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
    this same bench command).  A record is attached only when its build id (mxa_build_id(): a hash
    of the kernel sources and flags), config, env count and parity-hash setting all match the
    running bench; otherwise traffic is null and traffic_record says why."""
    prof = os.path.join(ROOT, "profiles", "hbm_traffic_%s.json" % config)
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
    if bool(p.get("parity_hash")) != parity_hash:
        why.append("parity hash setting differs")
    src["match"] = not why
    if why:
        src["why"] = "; ".join(why)
        return None, src
    return p.get("bytes_per_launch"), src


def replay_bench(args):
    """ABIDESEnv / market replay (BASELINE configs[4] shape): n envs stepping the reference's
    composition (Exchange + MarketReplayAgent + DummyRL) on a LOBSTER tape (IBM 2003-01-14 by
    default; --tape GOOG_2012-06-21 has ORDER_ID 0 records) with per-env random actions.  One
    bench step = one full episode: reset + the 761 ABIDESEnv.step calls of DummyRL's horizon
    (09:40-16:00 every 30 s).  Actions x ~ U(0, 0.01), level shares U(0, 1) are drawn on the
    device (torch Philox, per-rank seed) and stepped through mxa_step_device on the bench's
    stream, so nothing crosses PCIe inside the timed region; envs that finish early stay
    finished (the step kernel skips them)."""
    from mxabides import tape
    from mxabides.gym import ACTION_SIZE, OBS_SIZE, VecABIDESEnv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    tname = args.tape or "IBM_2003-01-14"
    tp = tape.Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % tname))
    n = args.envs
    n_steps = 761  # pd.date_range(09:40, 16:00, freq="30S")
    v = VecABIDESEnv(tp, n, device=local)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    v.set_stream(stream.cuda_stream)
    v.set_parity_hash(args.parity_hash)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000 + rank)
    act = torch.empty((n_steps, n, ACTION_SIZE), dtype=torch.float64, device="cuda")
    obs = torch.empty((n, OBS_SIZE), dtype=torch.float64, device="cuda")
    flags = torch.empty((n,), dtype=torch.int32, device="cuda")
    res = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    ev_pairs = []

    def episode(timed):
        v.reset()
        torch.rand(act.shape, generator=gen, dtype=torch.float64, device="cuda", out=act)
        act[:, :, 0] *= 0.01
        for i in range(n_steps):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            v.step_device(act[i].data_ptr(), obs.data_ptr(), flags.data_ptr())
            if timed:
                e1.record(stream)
                ev_pairs.append((e0, e1))
        v.write_results(res.data_ptr())
        shard.gather_records(res, world)
        return res[:, 0].sum()

    evw = torch.zeros((), dtype=torch.int64, device="cuda")
    for _ in range(args.warmup):  # the timed loop's exact ops
        evw += episode(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = torch.zeros((), dtype=torch.int64, device="cuda")
    for _ in range(args.steps):
        ev += episode(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    el = float(elt.item())
    events = int(ev.item())
    s = v.summary()
    nerr = int((s["status"] == 2).sum())
    if rank == 0:
        kms = [a.elapsed_time(b) for a, b in ev_pairs]
        avg_ms = sum(kms) / len(kms)
        achieved = ALGO_BYTES_PER_EVENT * (events / world / len(kms)) / (avg_ms * 1e-3) / 1e9
        out = {"metric": "env-steps/sec, ABIDESEnv market replay (%s LOBSTER tape) x%d envs per GPU" % (tname, n),
               "value": events / el, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int64",
               "data": "LOBSTER sample tape %s + device-drawn actions x~U(0,0.01), shares~U(0,1)" % tname,
               "config": {"workload": "marketreplay x%d envs per GPU, full episode (reset + %d ABIDESEnv.step) per bench "
                                      "step" % (n, n_steps),
                          "envs_per_gpu": n, "global_envs": n * world, "tape_records": len(tp),
                          "gym_steps_per_s": n * world * n_steps * args.steps / el,
                          "events_per_step": events / args.steps, "parallelism": "envs sharded, dp%d" % world,
                          "parity_hash": bool(args.parity_hash),
                          "env_errors": nerr},
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                            "kernel": "mxa_step_kernel<3> (marketreplay)", "avg_launch_ms": avg_ms,
                            "launches": len(kms), "algo_bytes_per_event": ALGO_BYTES_PER_EVENT}}
        if not args.no_cpu:
            import pyoracle
            k = 512  # ~10 s of one host core (8.4 M env-steps/s, ~144 k events per IBM episode)
            t1 = time.perf_counter()
            cev = 0
            for i in range(k):
                e = pyoracle.OracleGymEnv(tp)
                r2 = np.random.RandomState(i)
                while True:
                    _, d_, rc = e.step([r2.uniform(0, 0.01), r2.uniform(), r2.uniform()])
                    if d_ or rc:
                        break
                cev += e.events
            cs = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": cev / cs, "unit": "env-steps/s", "cores": 1, "kind": "port",
                                   "sample": "%d %s episodes, C oracle, 1 thread, %.1f s" % (k, tname, cs)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rl_bench(args):
    """rmsc03 + DummyRL under the GymKernel step loop (BASELINE configs[3]): n envs per GPU,
    each an rmsc03 market from its own seed with DummyRLExecutionAgent 64 stepped every 30 s
    (09:31-09:44, 27 ABIDESEnv.step calls per episode).  Actions (x ~ U(0, 0.01), level shares
    U(0, 1)) are drawn on the device (torch Philox, per-rank seed) and stepped through mxa_step_device on torch's
    stream, so nothing crosses PCIe inside the timed region.  One bench step = one full
    episode of every env (config build from seeds + 27 gym steps) + the RCCL all-gather of the
    per-env episode records."""
    from mxabides.gym import ACTION_SIZE, OBS_SIZE, VecABIDESEnv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    n = args.envs
    n_steps = 27  # pd.date_range(09:31, 09:44, "30S")
    ACT_XMAX = 0.01  # total-volume action x ~ U(0, 0.01): up to 1,000 of the 1e5 shares per step
    v = VecABIDESEnv(seeds=shard.env_seeds(0, rank, world, n), device=local)
    stream = torch.cuda.Stream()  # a real stream object (the legacy default stream's handle is 0)
    torch.cuda.set_stream(stream)
    v.set_stream(stream.cuda_stream)
    v.set_parity_hash(args.parity_hash)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000 + rank)
    act = torch.empty((n_steps, n, ACTION_SIZE), dtype=torch.float64, device="cuda")
    obs = torch.empty((n, OBS_SIZE), dtype=torch.float64, device="cuda")
    flags = torch.empty((n,), dtype=torch.int32, device="cuda")
    res = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    ev_pairs = []

    def episode(k, timed):
        v.reset(seeds=shard.env_seeds(k, rank, world, n))
        torch.rand(act.shape, generator=gen, dtype=torch.float64, device="cuda", out=act)
        act[:, :, 0] *= ACT_XMAX
        for i in range(n_steps):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            v.step_device(act[i].data_ptr(), obs.data_ptr(), flags.data_ptr())
            if timed:
                e1.record(stream)
                ev_pairs.append((e0, e1))
        v.write_results(res.data_ptr())
        shard.gather_records(res, world)
        return res[:, 0].sum(), flags

    evw = torch.zeros((), dtype=torch.int64, device="cuda")
    dw = torch.ones((), dtype=torch.bool, device="cuda")
    for k in range(args.warmup):  # the timed loop's exact ops (first launches of torch's kernels included)
        e, f = episode(k, False)
        evw += e
        dw &= (((f & 1) != 0) | ((f & 4) != 0)).all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = torch.zeros((), dtype=torch.int64, device="cuda")
    done_all = torch.ones((), dtype=torch.bool, device="cuda")
    for k in range(args.warmup, args.warmup + args.steps):
        e, f = episode(k, True)
        ev += e
        done_all &= (((f & 1) != 0) | ((f & 4) != 0)).all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    el = float(elt.item())
    events = int(ev.item())
    s = v.summary()
    n_err = int((s["status"] == 2).sum())
    if rank == 0:
        kms = [a.elapsed_time(b) for a, b in ev_pairs]
        avg_ms = sum(kms) / len(kms)
        my_ev_per_launch = events / world / len(kms)
        achieved = ALGO_BYTES_PER_EVENT * my_ev_per_launch / (avg_ms * 1e-3) / 1e9
        out = {"metric": "env-steps/sec, rmsc03 + DummyRL execution agent (GymKernel) x%d envs per GPU" % n,
               "value": events / el, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic (seeds) + device-drawn actions x~U(0,0.01), shares~U(0,1)",
               "config": {"workload": "rmsc03_rl x%d envs per GPU, full episode (config build + %d ABIDESEnv.step) per "
                                      "bench step, seeds %d+global_env" % (n, n_steps, SEED0),
                          "envs_per_gpu": n, "global_envs": n * world, "agents_per_env": v.n_agents,
                          "gym_steps_per_s": n * world * n_steps * args.steps / el,
                          "events_per_step": events / args.steps, "parallelism": "envs sharded, dp%d" % world,
                          "parity_hash": bool(args.parity_hash),
                          "env_errors": n_err, "all_done": bool(done_all.item())},
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                            "kernel": "mxa_step_kernel<4> (rmsc03_rl)", "avg_launch_ms": avg_ms, "launches": len(kms),
                            "algo_bytes_per_event": ALGO_BYTES_PER_EVENT}}
        if not args.no_cpu:
            import pyoracle
            k = 1024  # ~12 s of one host core
            t1 = time.perf_counter()
            cev = 0
            for i in range(k):
                e = pyoracle.OracleGymEnv(seed=int(SEED0 + i))
                r2 = np.random.RandomState(i)
                while True:
                    _, d_, rc = e.step([r2.uniform(0, 0.01), r2.uniform(), r2.uniform()])
                    if d_ or rc:
                        break
                cev += e.events
            cs = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": cev / cs, "unit": "env-steps/s", "cores": 1, "kind": "port",
                                   "sample": "%d rmsc03_rl episodes, C oracle, 1 thread, %.1f s" % (k, cs)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ddqn_bench(args):
    """rmsc03 + DummyRL (BASELINE configs[3]) with the DDQN execution learner in the loop
    (mxabides.ddqn: the reference's DDQLearningExecutionAgent learner on PyTorch-ROCm): every
    env's actions come from the shared Q-network (epsilon-greedy), transitions go to the device
    replay ring and the learner trains every 5 periods, as the reference agent does. One bench
    step = one full episode of every env (config build + 27 gym steps + learner) + the RCCL
    all-gather of the episode records. Learner state persists across bench steps."""
    from mxabides import ddqn
    from mxabides.gym import VecABIDESEnv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    n = args.envs
    v = VecABIDESEnv(seeds=shard.env_seeds(0, rank, world, n), device=local)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    v.set_stream(stream.cuda_stream)
    v.set_parity_hash(args.parity_hash)
    learner = ddqn.DDQNLearner(device="cuda", seed=1000 + rank, batch_size=args.ddqn_batch)
    task = ddqn.ExecutionTask(device="cuda")
    res = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    timing = []

    def episode(k, timed):
        r = ddqn.run_episode(v, learner, task, seeds=shard.env_seeds(k, rank, world, n),
                             timing=timing if timed else None)
        v.write_results(res.data_ptr())
        shard.gather_records(res, world)
        return res[:, 0].sum(), r["steps"]

    evw = torch.zeros((), dtype=torch.int64, device="cuda")
    for k in range(args.warmup):  # the timed loop's exact ops
        evw += episode(k, False)[0]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    learns0 = learner.learn_step_counter
    t0 = time.perf_counter()
    ev = torch.zeros((), dtype=torch.int64, device="cuda")
    gym_steps = 0
    for k in range(args.warmup, args.warmup + args.steps):
        e, ns = episode(k, True)
        ev += e
        gym_steps += ns
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    el = float(elt.item())
    events = int(ev.item())
    s = v.summary()
    if rank == 0:
        kms = [a.elapsed_time(b) for a, b in timing]
        avg_ms = sum(kms) / len(kms)
        my_ev_per_launch = events / world / len(kms)
        achieved = ALGO_BYTES_PER_EVENT * my_ev_per_launch / (avg_ms * 1e-3) / 1e9
        out = {"metric": "env-steps/sec, rmsc03 + DDQN execution learner (GymKernel) x%d envs per GPU" % n,
               "value": events / el, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "int64 (market), fp32 (Q-network)",
               "data": "synthetic (seeds); actions from the DDQN learner",
               "config": {"workload": "rmsc03_rl x%d envs per GPU + DDQN learner (NNModel_1, batch %d, train every "
                                      "5 periods), full episode per bench step, seeds %d+global_env"
                                      % (n, args.ddqn_batch, SEED0),
                          "envs_per_gpu": n, "global_envs": n * world, "agents_per_env": v.n_agents,
                          "gym_steps_per_s": n * world * gym_steps / el,
                          "learn_steps": learner.learn_step_counter - learns0,
                          "step_kernel_ms_total": sum(kms), "wall_ms_total": 1000.0 * el,
                          "events_per_step": events / args.steps, "parallelism": "envs sharded, dp%d" % world,
                          "parity_hash": bool(args.parity_hash),
                          "env_errors": int((s["status"] == 2).sum())},
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                            "kernel": "mxa_step_kernel<4> (rmsc03_rl)", "avg_launch_ms": avg_ms, "launches": len(kms),
                            "algo_bytes_per_event": ALGO_BYTES_PER_EVENT}}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--config", default="rmsc03")
    ap.add_argument("--chunk", type=int, default=1 << 22, help="max pops per env per kernel launch")
    ap.add_argument("--cpu-envs", type=int, default=2048, help="CPU-baseline sample size (envs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--parity-hash", action="store_true",
                    help="also compute the per-pop parity hash (test instrumentation, off by default: "
                         "tests/test_gpu_hash_switch.py shows every market result is identical either way)")
    ap.add_argument("--ddqn-batch", type=int, default=32, help="rmsc03_ddqn: learner batch size (reference 32)")
    ap.add_argument("--tape", default=None, help="marketreplay tape under tests/golden (IBM_2003-01-14, GOOG_2012-06-21)")
    args = ap.parse_args()
    if args.config == "marketreplay":
        return replay_bench(args)
    if args.config == "rmsc03_rl":
        return rl_bench(args)
    if args.config == "rmsc03_ddqn":
        return ddqn_bench(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    n = args.envs

    def seeds_for(step):
        return shard.env_seeds(step, rank, world, n)

    m = mxabides.VecMarket(args.config, seeds_for(0), device=local)
    stream = torch.cuda.Stream()  # a real stream object (the legacy default stream's handle is 0)
    torch.cuda.set_stream(stream)
    m.set_stream(stream.cuda_stream)
    m.set_parity_hash(args.parity_hash)
    res = torch.zeros((n, 4), dtype=torch.int64, device="cuda")

    kernel_ms, launches = [0.0], [0]

    def step(k):
        m.set_seeds(seeds_for(k))
        m.reset()
        launches[0] += m.run(chunk=args.chunk)
        kernel_ms[0] += m.last_kernel_ms
        m.write_results(res.data_ptr())
        shard.gather_records(res, world)  # episode records over RCCL/xGMI (the only collective)
        return res[:, 0].sum()

    evw = torch.zeros((), dtype=torch.int64, device="cuda")
    for k in range(args.warmup):
        evw += step(k)  # the same ops as a timed step (first launches of torch's kernels included)
    torch.cuda.synchronize()
    kernel_ms[0], launches[0] = 0.0, 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = torch.zeros((), dtype=torch.int64, device="cuda")
    for k in range(args.warmup, args.warmup + args.steps):
        ev += step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
    elapsed = float(elapsed.item())
    events = int(ev.item())
    summ = m.summary()
    n_err = int((summ["status"] == 2).sum())

    if rank == 0:
        ms_step = 1000.0 * elapsed / args.steps
        my_events_per_launch = events / world / max(1, launches[0])
        avg_launch_ms = kernel_ms[0] / max(1, launches[0])
        achieved = ALGO_BYTES_PER_EVENT * my_events_per_launch / (avg_launch_ms * 1e-3) / 1e9
        traffic, traffic_src = traffic_record(args.config, n, bool(args.parity_hash))
        metric = METRIC if args.config == "rmsc03" else "env-steps/sec, %s x%d envs per GPU" % (args.config, n)
        out = {
            "metric": metric, "value": events / elapsed, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": "%s x%d envs per GPU, full episode per step (config build from seeds + "
                                   "the config's session), seeds %d+global_env" % (args.config, n, SEED0),
                       "envs_per_gpu": n, "global_envs": n * world, "agents_per_env": m.n_agents,
                       "events_per_step": events / args.steps, "parallelism": "envs sharded, dp%d" % world,
                          "parity_hash": bool(args.parity_hash),
                       "env_errors": n_err, "device": torch.cuda.get_device_name(local),
                       "cus": torch.cuda.get_device_properties(local).multi_processor_count},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_record": traffic_src,
                         "kernel": "mxa_run_kernel<%d> (%s)" % (mxabides.CONFIG_IDS[args.config], args.config), "avg_launch_ms": avg_launch_ms,
                         "launches": launches[0], "algo_bytes_per_event": ALGO_BYTES_PER_EVENT},
        }
        if not args.no_cpu:
            import pyoracle
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            cseeds = (SEED0 + np.arange(args.cpu_envs, dtype=np.int64)) & 0xFFFFFFFF
            cev, _, csec = pyoracle.run_batch(args.config, cseeds.astype(np.uint32), threads)
            out["cpu_baseline"] = {"value": float(cev.sum()) / csec, "unit": "env-steps/s", "cores": threads,
                                   "kind": "port",
                                   "sample": "%d %s envs (seeds %d..), full episodes, C oracle, %d threads, %.1f s wall "
                                             "(~%.0f core-s)" % (args.cpu_envs, args.config, SEED0, threads, csec, csec * threads)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
