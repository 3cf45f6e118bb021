#!/usr/bin/env python3
"""Golden fixtures for the DummyRL-in-rmsc03-background composition (BASELINE.json configs[3],
SURVEY.md §8(d) "RL" row: a build-defined composition, horizon inside the 15-min session).

CONTAINER-ONLY TEST INFRASTRUCTURE (see gen_fixtures.py).  The composition is assembled from
the reference's own classes, nothing restated:
  * config/rmsc03.py builds its 64 agents, oracle and kernel exactly as for `-s SEED`
    (Kernel.runner is intercepted so the script only constructs);
  * a DummyRLExecutionAgent (agent_config.py:115-137 parameters: BUY 1e5, 30 s, order_level 2,
    steep 0.5) is appended as agent 64 with horizon pd.date_range(09:31, 09:44, "30S");
  * a GymKernel (GymKernel.py) runs them with rmsc03's kernel RandomState, latency zeros,
    noise [0.0], compute delay 0, rmsc03's start/stop and oracle;
  * env.step(action) = GymKernel.stepRunner(action); done as in ABIDESEnv.step.
Recorded: actions, per-step obs / done / events, trace head, FNV hash, final book, holdings.
A step on which the reference raises is recorded as {"error": exception type, "events"}.

Usage: python tests/golden/gen_rl_fixtures.py SEED ACTION_SEED [XMAX]  (x ~ U(0, XMAX), default 0.002)
"""
import importlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_fixtures as G  # noqa: E402
import gen_mr_fixtures as M  # noqa: E402


def main():
    seed, aseed = int(sys.argv[1]), int(sys.argv[2])
    xmax = float(sys.argv[3]) if len(sys.argv) > 3 else 0.002
    out = os.path.join(HERE, "rl_rmsc03_%d_%d" % (seed, aseed))
    M.install_stubs()
    import queue

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
    sys.argv = ["abides.py", "-c", "rmsc03", "-s", str(seed), "-t", "ABM", "-d", "20190628"]
    real = sys.stdout
    sys.stdout = io.StringIO()
    try:
        importlib.import_module("config.rmsc03")
    finally:
        sys.stdout = real
    kw, k0 = cap["kw"], cap["kernel"]
    agents = list(kw["agents"])
    date = pd.Timestamp("2019-06-28")
    G.MIDNIGHT = int(date.value)
    from agent.execution.rl.dummy_rl_execution_agent import DummyRLExecutionAgent
    from GymKernel import GymKernel
    hz = pd.date_range(start=date + pd.to_timedelta("09:31:00"), end=date + pd.to_timedelta("09:44:00"), freq="30S")
    rl = DummyRLExecutionAgent(id=len(agents), name="%d_DUMMY_RL_EXECUTION_AGENT" % len(agents),
                               type="DummyRLExecutionAgent", symbol="ABM", starting_cash=0, direction="BUY",
                               quantity=1e5, execution_time_horizon=hz, freq="30S", trade=True, log_events=False,
                               log_orders=False, random_state=np.random.RandomState(0), order_level=2,
                               a_q_map_steep_factor=0.5)
    agents.append(rl)

    trace_head, ck, state = [], [], {"h": G.FNV_OFF, "n": 0}

    class RecPQ(queue.PriorityQueue):
        def get(self, *a, **k):
            item = super().get(*a, **k)
            t, (rcp, mtype, msg) = item
            rec = G.encode(int(t.value) - G.MIDNIGHT, int(rcp), int(mtype.value), msg)
            state["h"] = G.fnv_words(state["h"], rec)
            state["n"] += 1
            if len(trace_head) < 20000:
                trace_head.append(rec)
            if state["n"] % 1000 == 0:
                ck.append(state["h"])
            return item

    kern = GymKernel("rmsc03 + DummyRL", RL_agent=rl, agents=agents, random_state=k0.random_state)
    kern.messages = RecPQ()
    n = len(agents)
    sys.stdout = io.StringIO()
    try:
        kern.initRunner(startTime=kw["startTime"], stopTime=kw["stopTime"], agentLatency=np.zeros((n, n)),
                        latencyNoise=[0.0], defaultComputationDelay=kw["defaultComputationDelay"], defaultLatency=0,
                        oracle=kw["oracle"], log_dir=None)
        rs = np.random.RandomState(aseed)
        actions, steps = [], []
        while True:
            a = [float(rs.uniform(0, xmax)), float(rs.uniform()), float(rs.uniform())]
            actions.append(a)
            sys.stdout = io.StringIO()
            try:
                rew, obs = kern.stepRunner(a)
            except Exception as exc:  # the reference raises mid-step (e.g. empty book side)
                steps.append({"error": type(exc).__name__, "events": int(kern.ttl_messages),
                              "t": int(kern.currentTime.value) - G.MIDNIGHT})
                break
            done = 0 if (not kern.messages.empty() and kern.currentTime <= kern.stopTime) else 1
            steps.append({"obs": [float(x) for x in obs] if obs is not None and len(obs) else [], "done": done,
                          "events": int(kern.ttl_messages), "t": int(kern.currentTime.value) - G.MIDNIGHT})
            if done:
                break
    finally:
        sys.stdout = real

    from util.order.Order import Order
    ob = agents[0].order_books["ABM"]

    def lvl(side):
        return [[[int(o.order_id), int(o.agent_id), int(o.quantity), G._price(o.limit_price)] for o in level]
                for level in side]

    final = {"seed": seed, "action_seed": aseed, "xmax": xmax, "steps": steps, "events": state["n"], "hash": "%016x" % state["h"],
             "hash_checkpoints": ["%016x" % x for x in ck], "order_id_counter": int(Order.order_id),
             "bids": lvl(ob.bids), "asks": lvl(ob.asks), "agents": []}
    for a in agents[1:]:
        h = {k: float(v) for k, v in a.holdings.items()}
        final["agents"].append({"id": a.id, "cash": h.get("CASH"), "shares": h.get("ABM", 0.0),
                                "n_open": len(a.orders)})
    final["rl"] = {"rem_quantity": float(rl.rem_quantity), "trade": bool(rl.trade)}
    with open(out + ".json", "w") as f:
        json.dump(final, f)
    np.savez_compressed(out + ".npz", trace=np.asarray(trace_head, dtype=np.int64),
                        actions=np.asarray(actions, dtype=np.float64))
    print("steps", len(steps), "events", state["n"], "hash", final["hash"], "rl rem", rl.rem_quantity)


if __name__ == "__main__":
    main()
