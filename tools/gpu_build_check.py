"""Compare the device-built env (after mxa_reset) with the oracle's config construction."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd"), os.path.join(ROOT, "oracle")]
import numpy as np

import mxabides

for cfg in sys.argv[1:] or ["sparse_zi_100", "sparse_zi_1000"]:
    m = mxabides.VecMarket(cfg, [123456789])
    lay = m.layout()
    n = m.n_agents
    lat = m.raw(0, lay["lat"], 8 * (2 * n if cfg == "sparse_zi_100" else n)).view(np.float64)
    G = np.random.RandomState(123456789)
    G.randint(0, 2**32); G.randint(0, 2**32)
    if cfg == "sparse_zi_100":
        G.randint(0, 2**32)
    G.exponential(1 / 2.77778e-13)
    for _ in range(n):
        G.randint(0, 2**32)
    M = G.uniform(21000, 100000 if cfg == "sparse_zi_100" else 13000000, (n, n))
    ok_row = np.array_equal(lat[:n][1:], M[0][1:])
    print(cfg, "row0 ok", ok_row, "first bad", np.nonzero(lat[:n] != M[0])[0][:5], lat[:4], M[0][:4])
    if cfg == "sparse_zi_100":
        print(" col0 ok", np.array_equal(lat[n:], M[:, 0]), np.nonzero(lat[n:] != M[:, 0])[0][:5])
    hdr = m.raw(0, 0, 320)
    print(" hdr status/err", hdr[32:40].view(np.int32))
