"""First divergence of a device trace from a reference fixture, with context (parity debugging).
usage: python tools/trace_diff.py CONFIG SEED [CONTEXT]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import mxabides
from golden_util import first_mismatch, load, market_kw

cfg, seed = sys.argv[1], int(sys.argv[2])
ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 6
d, ref = load(cfg, seed)
m = mxabides.VecMarket(cfg, [seed], trace_cap=len(ref) + 16, **market_kw(cfg))
m.run()
s = m.summary()
tr = m.trace(0)
i = first_mismatch(tr, ref)
print(cfg, seed, "status", int(s["status"][0]), "err", int(s["err"][0]), "events", int(s["events"][0]), "ref", d["events"],
      "first mismatch", i)
if i >= 0:
    for k in range(max(0, i - ctx), min(max(len(tr), len(ref)), i + 3)):
        a = tr[k].tolist() if k < len(tr) else None
        b = ref[k].tolist() if k < len(ref) else None
        print("%7d %s dev %s" % (k, "==" if a == b else "!=", a))
        if a != b:
            print("%7s    ref %s" % ("", b))
