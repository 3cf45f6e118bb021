"""Quick GPU bring-up: probes + one env per config with trace vs golden (prints first mismatch)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np

import mxabides
from golden_util import first_mismatch, load

L = mxabides.load()
out = np.zeros(8)
print("rng probe rc", L.mxa_rng_probe(0, 5489, 0, 0.0, 0.0, 8, out.ctypes.data), out.astype(np.int64), flush=True)
cfgs = sys.argv[1:] or ["rmsc03:123456789", "sparse_zi_100:123456789", "sparse_zi_1000:123456789"]
for spec in cfgs:
    cfg, seed = spec.split(":")
    seed = int(seed)
    d, ref = load(cfg, seed)
    t = time.time()
    m = mxabides.VecMarket(cfg, [seed], trace_cap=len(ref))
    t1 = time.time()
    nl = m.run(chunk=1 << 22)
    t2 = time.time()
    s = m.summary()
    tr = m.trace(0)
    i = first_mismatch(tr, ref)
    print(cfg, seed, "build %.2fs run %.2fs launches %d" % (t1 - t, t2 - t1, nl), "status", s["status"][0], "err",
          s["err"][0], "events", s["events"][0], d["events"], "hash ok", "%016x" % int(s["hash"][0]) == d["hash"],
          "first mismatch", i, "maxq", s["max_queue"][0], "maxbook", s["max_book"][0], flush=True)
    if i >= 0:
        for j in range(max(0, i - 3), min(i + 2, len(tr), len(ref))):
            print("  %d gpu %s\n      ref %s" % (j, tr[j].tolist(), ref[j].tolist()))
