"""Diagnostics: where do the HBM env blocks of a hash-on and a hash-off run differ?"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
import mxabides
from mxabides import shard
cfg, n = (sys.argv[1] if len(sys.argv) > 1 else "rmsc03"), 64
seeds = shard.env_seeds(0, 0, 1, n)
on = mxabides.VecMarket(cfg, seeds)
on.run()
off = mxabides.VecMarket(cfg, seeds)
off.set_parity_hash(False)
off.run()
lay = on.layout()
print("layout", lay, "env_bytes", on.env_bytes)
secs = sorted(lay.items(), key=lambda kv: kv[1])
for e in range(n):
    a, b = on.raw(e, 0, on.env_bytes), off.raw(e, 0, off.env_bytes)
    a[16:24] = 0
    b[16:24] = 0
    d = np.nonzero(a != b)[0]
    if len(d):
        sec = [k for k, o in secs if o <= d[0]]
        print("env", e, "ndiff", len(d), "first", d[0], "last", d[-1], "section", sec[-1] if sec else "hdr",
              "on", a[d[0]:d[0] + 16].tolist(), "off", b[d[0]:d[0] + 16].tolist())
