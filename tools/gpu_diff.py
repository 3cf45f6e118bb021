"""Find envs whose GPU hash differs from the oracle; print the first differing trace record."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np

import mxabides
import pyoracle
from golden_util import first_mismatch

cfg = sys.argv[1]
seeds = (np.arange(int(sys.argv[2]), dtype=np.int64) * 7919 + 11) & 0xFFFFFFFF
m = mxabides.VecMarket(cfg, seeds)
m.run()
s = m.summary()
ev, hs, _ = pyoracle.run_batch(cfg, seeds.astype(np.uint32), threads=8)
bad = np.nonzero((s["hash"] != hs) | (s["events"] != ev))[0]
print(cfg, "envs", len(seeds), "mismatching", len(bad), bad[:20].tolist(), flush=True)
for i in bad[:3]:
    seed = int(seeds[i])
    n = int(max(ev[i], s["events"][i])) + 10
    g = mxabides.VecMarket(cfg, [seed], trace_cap=n)
    g.run()
    tg = g.trace(0)
    o = pyoracle.OracleEnv(cfg, seed, trace_cap=n)
    o.run()
    to = o.trace()
    j = first_mismatch(tg, to)
    print("seed", seed, "gpu events", len(tg), "oracle", len(to), "first mismatch", j)
    for k in range(max(0, j - 6), min(j + 3, len(tg), len(to))):
        print("  %d gpu %s\n      ora %s" % (k, tg[k].tolist(), to[k].tolist()))
