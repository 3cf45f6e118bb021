"""Wall time of the build kernel (mxa_reset: config construction from seeds) per config and env
count: a latency-bound build takes about as long at 256 envs (one wave per CU) as at the bench
size; a throughput-bound one scales with the envs per CU.
usage: python tools/time_build.py CONFIG N [N ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-optimal-execution_amd"))
import mxabides  # noqa: E402


def main():
    cfg = sys.argv[1]
    for n in map(int, sys.argv[2:]):
        m = mxabides.VecMarket(cfg, (123456789 + np.arange(n, dtype=np.int64)) & 0xFFFFFFFF)
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            m.reset()
            best = min(best, time.perf_counter() - t0)
        print("%s x%d: build %.3f ms (best of 5, host wall incl. launch)" % (cfg, n, best * 1e3), flush=True)
        del m


if __name__ == "__main__":
    main()
