"""Replay episode on the GPU vs the C oracle with full traces: first differing event record.
usage: python tools/gpu_mr_diff.py TICKER DATE [max_steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np

import pyoracle
from golden_util import first_mismatch
from mxabides import tape
from mxabides.gym import VecABIDESEnv

ticker, date = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
G = os.path.join(ROOT, "tests", "golden")
tp = tape.Tape.load(os.path.join(G, "tape_%s_%s.npz" % (ticker, date)))
acts = np.load(os.path.join(G, "mr_%s_%s_789_1.npz" % (ticker, date)))["actions"][:steps]
cap = 400000
v = VecABIDESEnv(tp, 1, trace_cap=cap)
o = pyoracle.OracleGymEnv(tp, trace_cap=cap)
for i, a in enumerate(acts):
    v.step(a[None, :])
    o.step(a)
    if v.summary()["events"][0] != o.events:
        print("step", i, "gpu events", v.summary()["events"][0], "oracle", o.events)
        break
tg, to = v.trace(0), o.trace()
j = first_mismatch(tg, to)
print("gpu", len(tg), "oracle", len(to), "first mismatch", j, "err", v.summary()["err"][0])
for k in range(max(0, j - 12), min(j + 4, len(tg), len(to))):
    print("  %d gpu %s\n      ora %s" % (k, tg[k].tolist(), to[k].tolist()))
