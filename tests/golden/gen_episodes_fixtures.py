#!/usr/bin/env python3
"""Golden fixtures for consecutive episodes in ONE process:
`Order.order_id` and `Order._order_ids` are class attributes (util/order/Order.py:8-9, 27-42),
so a second `ABIDESEnv.reset()` (ABIDESEnv.py:51-57: new agents and kernel, same process)
continues the auto order ids from the first episode's counter and skips every id used before;
and `MarketReplayAgent.orders.get(0)` (MarketReplayAgent.py:69-75) can no longer find an order
with auto id 0.

CONTAINER-ONLY TEST INFRASTRUCTURE (see gen_fixtures.py, gen_mr_fixtures.py, gen_rl_fixtures.py:
same stubs, same recording).  Two modes:

  python tests/golden/gen_episodes_fixtures.py mr TICKER DATE SEED ACTION_SEED EPISODES
      ABIDESEnv(ticker, date, seed): EPISODES episodes, env.reset() between them; actions from one
      RandomState(ACTION_SEED) across all episodes (x ~ U(0, 0.01), shares U(0, 1))
  python tests/golden/gen_episodes_fixtures.py rl ACTION_SEED XMAX SEED1 SEED2 ...
      the rmsc03 + DummyRL composition of gen_rl_fixtures.py, one episode per seed, all in this
      process (config/rmsc03.py re-run for each seed)

Writes eps_<mode>_<...>.json (per episode: steps, events, hash, hash checkpoints, order-id
counter, book, holdings) and .npz (per episode: actions, trace head).
"""
import importlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import gen_fixtures as G  # noqa: E402
import gen_mr_fixtures as M  # noqa: E402

TRACE_HEAD = 20000


class Recorder:
    """per-episode trace head + rolling hash of every Kernel pop"""

    def __init__(self):
        self.reset()

    def reset(self):
        self.head, self.ck, self.h, self.n = [], [], G.FNV_OFF, 0

    def pq_class(self):
        import queue
        rec = self

        class RecPQ(queue.PriorityQueue):
            def get(self, *a, **k):
                item = super().get(*a, **k)
                t, (rcp, mtype, msg) = item
                r = G.encode(int(t.value) - G.MIDNIGHT, int(rcp), int(mtype.value), msg)
                rec.h = G.fnv_words(rec.h, r)
                rec.n += 1
                if len(rec.head) < TRACE_HEAD:
                    rec.head.append(r)
                if rec.n % 1000 == 0:
                    rec.ck.append(rec.h)
                return item
        return RecPQ


def book_levels(side):
    return [[[int(o.order_id), int(o.agent_id), int(o.quantity), G._price(o.limit_price)] for o in level]
            for level in side]


def run_mr(ticker, date, seed, aseed, episodes):
    M.install_stubs()
    import pandas as pd
    import util.util as U
    U.silent_mode = True
    os.chdir(REF)  # the replay agent opens data/lobster/... relative to the cwd
    tmpd = tempfile.mkdtemp(prefix="mr_proc_") + "/"
    from agent.examples import MarketReplayAgent as MRA
    orig_proc = MRA.LOBSTEROrdersProcessor.__init__

    def proc_init(self, symbol, date_, start_time, end_time, orders_file_path, processed_orders_folder_path):
        # a fresh folder every time: the processor parses the LOBSTER CSV itself (never a cached pickle)
        shutil.rmtree(tmpd, ignore_errors=True)
        os.makedirs(tmpd)
        orig_proc(self, symbol, date_, start_time, end_time, orders_file_path, tmpd)

    MRA.LOBSTEROrdersProcessor.__init__ = proc_init
    G.MIDNIGHT = int(pd.Timestamp(date).value)
    rec = Recorder()
    import Kernel as K
    orig_init = K.Kernel.__init__
    PQ = rec.pq_class()

    def kinit(self, *a, **k):
        orig_init(self, *a, **k)
        self.messages = PQ()

    K.Kernel.__init__ = kinit
    K.Kernel.writeLog = lambda *a, **k: None
    K.Kernel.writeSummaryLog = lambda *a, **k: None
    from agent.ExchangeAgent import ExchangeAgent
    ExchangeAgent.logOrderBookSnapshots = lambda *a, **k: None
    from ABIDESEnv import ABIDESEnv
    from util.order.Order import Order

    real = sys.stdout
    rs = np.random.RandomState(aseed)
    eps, arrays = [], {}
    sys.stdout = io.StringIO()
    try:
        env = ABIDESEnv(ticker=ticker, date=date, seed=seed)
        for e in range(episodes):
            if e:
                env.reset()
            rec.reset()
            id0 = int(Order.order_id)
            actions, steps = [], []
            while True:
                a = [float(rs.uniform(0, 0.01)), float(rs.uniform()), float(rs.uniform())]
                actions.append(a)
                sys.stdout = io.StringIO()
                obs, rew, done, info = env.step(a)
                steps.append({"obs": [float(x) for x in obs] if obs is not None and len(obs) else [],
                              "done": int(done), "events": int(env.kernel.ttl_messages)})
                if done:
                    break
            agents = env.agents.agent_list
            ob = agents[0].order_books[ticker]
            d = {"episode": e + 1, "order_id_counter_start": id0, "order_id_counter": int(Order.order_id),
                 "steps": steps, "events": rec.n, "hash": "%016x" % rec.h, "hash_checkpoints": ["%016x" % x for x in rec.ck],
                 "bids": book_levels(ob.bids), "asks": book_levels(ob.asks), "agents": []}
            for a in agents[1:]:
                d["agents"].append({"id": a.id, "holdings": {k: float(v) for k, v in a.holdings.items()},
                                    "open_orders": [[int(o.order_id), 1 if o.is_buy_order else 0, float(o.quantity),
                                                     G._price(o.limit_price)] for o in a.orders.values()]})
            eps.append(d)
            arrays["actions_%d" % (e + 1)] = np.asarray(actions, dtype=np.float64)
            arrays["trace_%d" % (e + 1)] = np.asarray(rec.head, dtype=np.int64)
            real.write("episode %d: steps %d events %d hash %s ids %d -> %d\n" % (e + 1, len(steps), rec.n, d["hash"], id0,
                                                                                d["order_id_counter"]))
    finally:
        sys.stdout = real
    out = os.path.join(HERE, "eps_mr_%s_%s_%d_%d" % (ticker, date, seed, aseed))
    with open(out + ".json", "w") as f:
        json.dump({"ticker": ticker, "date": date, "seed": seed, "action_seed": aseed, "episodes": eps}, f)
    np.savez_compressed(out + ".npz", **arrays)


def run_rl(aseed, xmax, seeds):
    M.install_stubs()
    import pandas as pd
    import util.util as U
    U.silent_mode = True
    import Kernel as K
    cap = {}

    def fake_runner(self, **kw):
        cap["kernel"] = self
        cap["kw"] = kw

    K.Kernel.runner = fake_runner
    K.Kernel.writeLog = lambda *a, **k: None
    K.Kernel.writeSummaryLog = lambda *a, **k: None
    from agent.ExchangeAgent import ExchangeAgent
    ExchangeAgent.logOrderBookSnapshots = lambda *a, **k: None
    from agent.TradingAgent import TradingAgent
    TradingAgent.getTransactedVolume = TradingAgent.get_transacted_volume
    from agent.execution.rl.dummy_rl_execution_agent import DummyRLExecutionAgent
    from GymKernel import GymKernel
    from util.order.Order import Order
    date = pd.Timestamp("2019-06-28")
    G.MIDNIGHT = int(date.value)
    rec = Recorder()
    PQ = rec.pq_class()
    rs = np.random.RandomState(aseed)
    real = sys.stdout
    eps, arrays = [], {}
    mod = None
    for e, seed in enumerate(seeds):
        sys.argv = ["abides.py", "-c", "rmsc03", "-s", str(seed), "-t", "ABM", "-d", "20190628"]
        sys.stdout = io.StringIO()
        try:  # config/rmsc03.py runs at import: a fresh import per episode, same process
            if mod is None:
                mod = importlib.import_module("config.rmsc03")
            else:
                mod = importlib.reload(mod)
        finally:
            sys.stdout = real
        kw, k0 = cap["kw"], cap["kernel"]
        agents = list(kw["agents"])
        hz = pd.date_range(start=date + pd.to_timedelta("09:31:00"), end=date + pd.to_timedelta("09:44:00"), freq="30S")
        rl = DummyRLExecutionAgent(id=len(agents), name="%d_DUMMY_RL_EXECUTION_AGENT" % len(agents),
                                   type="DummyRLExecutionAgent", symbol="ABM", starting_cash=0, direction="BUY",
                                   quantity=1e5, execution_time_horizon=hz, freq="30S", trade=True, log_events=False,
                                   log_orders=False, random_state=np.random.RandomState(0), order_level=2,
                                   a_q_map_steep_factor=0.5)
        agents.append(rl)
        rec.reset()
        id0 = int(Order.order_id)
        kern = GymKernel("rmsc03 + DummyRL", RL_agent=rl, agents=agents, random_state=k0.random_state)
        kern.messages = PQ()
        n = len(agents)
        actions, steps = [], []
        sys.stdout = io.StringIO()
        try:
            kern.initRunner(startTime=kw["startTime"], stopTime=kw["stopTime"], agentLatency=np.zeros((n, n)),
                            latencyNoise=[0.0], defaultComputationDelay=kw["defaultComputationDelay"], defaultLatency=0,
                            oracle=kw["oracle"], log_dir=None)
            while True:
                a = [float(rs.uniform(0, xmax)), float(rs.uniform()), float(rs.uniform())]
                actions.append(a)
                sys.stdout = io.StringIO()
                try:
                    rew, obs = kern.stepRunner(a)
                except Exception as exc:  # the reference raises mid-step (e.g. empty book side)
                    steps.append({"error": type(exc).__name__, "events": int(kern.ttl_messages)})
                    break
                done = 0 if (not kern.messages.empty() and kern.currentTime <= kern.stopTime) else 1
                steps.append({"obs": [float(x) for x in obs] if obs is not None and len(obs) else [], "done": done,
                              "events": int(kern.ttl_messages)})
                if done:
                    break
        finally:
            sys.stdout = real
        ob = agents[0].order_books["ABM"]
        d = {"episode": e + 1, "seed": seed, "order_id_counter_start": id0, "order_id_counter": int(Order.order_id),
             "steps": steps, "events": rec.n, "hash": "%016x" % rec.h, "hash_checkpoints": ["%016x" % x for x in rec.ck],
             "bids": book_levels(ob.bids), "asks": book_levels(ob.asks), "agents": []}
        for a in agents[1:]:
            h = {k: float(v) for k, v in a.holdings.items()}
            d["agents"].append({"id": a.id, "cash": h.get("CASH"), "shares": h.get("ABM", 0.0), "n_open": len(a.orders)})
        eps.append(d)
        arrays["actions_%d" % (e + 1)] = np.asarray(actions, dtype=np.float64)
        arrays["trace_%d" % (e + 1)] = np.asarray(rec.head, dtype=np.int64)
        print("episode %d seed %d: steps %d events %d hash %s ids %d -> %d" % (e + 1, seed, len(steps), rec.n, d["hash"],
                                                                              id0, d["order_id_counter"]))
    out = os.path.join(HERE, "eps_rl_%d_%s" % (aseed, "_".join(str(s) for s in seeds)))
    with open(out + ".json", "w") as f:
        json.dump({"action_seed": aseed, "xmax": xmax, "seeds": list(seeds), "episodes": eps}, f)
    np.savez_compressed(out + ".npz", **arrays)


if __name__ == "__main__":
    if sys.argv[1] == "mr":
        run_mr(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]))
    else:
        run_rl(int(sys.argv[2]), float(sys.argv[3]), [int(x) for x in sys.argv[4:]])
