#!/usr/bin/env python3
"""Golden fixtures for the ABIDESEnv / market-replay path.

CONTAINER-ONLY TEST INFRASTRUCTURE, like gen_fixtures.py: it imports the *reference*
ABIDESEnv read-only from /root/reference and records what the build must reproduce.
Nothing on the product path imports it; /root/reference does not exist on the GPU box.

Stubs (logging/UI only; none touches simulated arithmetic): `jsons.dump`, the pandas 2
renames, `gym` (ABIDESEnv only subclasses gym.Env and builds two Box spaces), and
`IPython.display.clear_output` (GymKernel clears the notebook output per event).
`util.silent_mode = True` as SURVEY §8(c) prescribes.  The processed-orders folder is
redirected to a temp dir so the LOBSTER CSV of the tape is parsed by the reference's own
LOBSTEROrdersProcessor.  The reference's committed pickles are never loaded.

Recorded per episode (ticker, date, seed, action seed):
  * the actions fed to env.step (float64 [steps][3]) and, per step, the observation
    (float64[9] or empty), done flag, ttl_messages and kernel time;
  * the first 20000 event records (same 10-word encoding as gen_fixtures.encode) plus a
    rolling FNV-1a hash with checkpoints every 1000 pops over the whole episode;
  * the final exchange book, the RL and replay agents' holdings and open orders, the
    order-id counter.

Usage: python tests/golden/gen_mr_fixtures.py IBM 2003-01-14 789 1 [max_steps]
"""
import io
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import gen_fixtures as G  # noqa: E402


def install_stubs():
    G.install_stubs()
    gym = types.ModuleType("gym")
    gym.Env = object
    spaces = types.ModuleType("gym.spaces")

    class Box:
        def __init__(self, low, high):
            self.low, self.high = low, high

    spaces.Box = Box
    gym.spaces = spaces
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    ipy = types.ModuleType("IPython")
    disp = types.ModuleType("IPython.display")
    disp.clear_output = lambda wait=False: None
    ipy.display = disp
    sys.modules["IPython"] = ipy
    sys.modules["IPython.display"] = disp


def main():
    ticker, date, seed, aseed = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    max_steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10 ** 9
    out = os.path.join(HERE, "mr_%s_%s_%d_%d" % (ticker, date, seed, aseed))
    install_stubs()
    import queue

    import pandas as pd
    import util.util as U
    U.silent_mode = True
    os.chdir(REF)  # the replay agent opens data/lobster/... relative to the cwd
    tmpd = tempfile.mkdtemp(prefix="mr_proc_") + "/"
    from agent.examples import MarketReplayAgent as MRA
    orig_proc = MRA.LOBSTEROrdersProcessor.__init__

    def proc_init(self, symbol, date_, start_time, end_time, orders_file_path, processed_orders_folder_path):
        orig_proc(self, symbol, date_, start_time, end_time, orders_file_path, tmpd)

    MRA.LOBSTEROrdersProcessor.__init__ = proc_init

    G.MIDNIGHT = int(pd.Timestamp(date).value)
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

    import Kernel as K
    orig_init = K.Kernel.__init__

    def kinit(self, *a, **k):
        orig_init(self, *a, **k)
        self.messages = RecPQ()

    K.Kernel.__init__ = kinit
    K.Kernel.writeLog = lambda *a, **k: None
    K.Kernel.writeSummaryLog = lambda *a, **k: None
    from agent.ExchangeAgent import ExchangeAgent
    ExchangeAgent.logOrderBookSnapshots = lambda *a, **k: None
    from ABIDESEnv import ABIDESEnv

    real = sys.stdout
    sys.stdout = io.StringIO()
    try:
        env = ABIDESEnv(ticker=ticker, date=date, seed=seed)
        rs = np.random.RandomState(aseed)
        actions, steps = [], []
        for i in range(max_steps):
            a = [float(rs.uniform(0, 0.01)), float(rs.uniform()), float(rs.uniform())]
            actions.append(a)
            sys.stdout = io.StringIO()
            obs, rew, done, info = env.step(a)
            steps.append({"obs": [float(x) for x in obs] if obs is not None and len(obs) else [],
                          "done": int(done), "events": int(env.kernel.ttl_messages),
                          "t": int(env.kernel.currentTime.value) - G.MIDNIGHT, "reward": rew})
            if done:
                break
    finally:
        sys.stdout = real

    from util.order.Order import Order
    agents = env.agents.agent_list
    ob = agents[0].order_books[ticker]

    def lvl(side):
        return [[[int(o.order_id), int(o.agent_id), int(o.quantity), G._price(o.limit_price)] for o in level]
                for level in side]

    final = {"ticker": ticker, "date": date, "seed": seed, "action_seed": aseed, "steps": steps,
             "events": state["n"], "hash": "%016x" % state["h"], "hash_checkpoints": ["%016x" % x for x in ck],
             "order_id_counter": int(Order.order_id), "bids": lvl(ob.bids), "asks": lvl(ob.asks),
             "last_trade": G._price(ob.last_trade), "agents": []}
    for a in agents[1:]:
        final["agents"].append({
            "id": a.id, "holdings": {k: float(v) for k, v in a.holdings.items()},
            "open_orders": [[int(o.order_id), 1 if o.is_buy_order else 0, float(o.quantity), G._price(o.limit_price)]
                            for o in a.orders.values()]})
    rl = agents[2]
    final["rl"] = {"rem_quantity": float(rl.rem_quantity), "executed": len(rl.executed_orders),
                   "trade": bool(rl.trade)}
    with open(out + ".json", "w") as f:
        json.dump(final, f)
    np.savez_compressed(out + ".npz", trace=np.asarray(trace_head, dtype=np.int64),
                        actions=np.asarray(actions, dtype=np.float64))
    print("steps", len(steps), "events", state["n"], "hash", final["hash"])


if __name__ == "__main__":
    main()
