"""mxa_run's launch schedule (mxa_set_launch_schedule): run-kernel ms of the first launch of
FC pops and of the rest (the envs still running, compacted into the grid), per FC;
python tools/ab_sched.py CONFIG N_ENVS "FC1 FC2 ..." [REPS]   (FC 0 = one launch)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
import mxabides

cfg, n = sys.argv[1], int(sys.argv[2])
fcs = [int(x) for x in sys.argv[3].split()]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
BIG = 1 << 22
m = mxabides.VecMarket(cfg, (123456789 + np.arange(n)) & 0xFFFFFFFF)


def digest():
    s = m.summary()
    return hashlib.sha1(np.ascontiguousarray(s["events"]).tobytes() +
                        np.ascontiguousarray(s["hash"]).tobytes()).hexdigest()[:16], s


for fc in fcs:
    m.set_parity_hash(False)
    rows = []
    for r in range(reps):
        m.reset()
        if fc:
            m.run(chunk=fc, max_launches=1)
            t1 = m.last_kernel_ms
            left = int((m.summary()["status"] == 0).sum())  # include/mxa.h: 0 running
            nl = m.run(chunk=BIG)
            t2 = m.last_kernel_ms
        else:
            m.run(chunk=BIG)
            t1, t2, left, nl = m.last_kernel_ms, 0.0, n, 0
        rows.append((t1 + t2, t1, t2, left, nl))
    m.set_parity_hash(True)
    m.reset()
    m.set_launch_schedule(fc)
    m.run(chunk=BIG)
    m.set_launch_schedule(0)
    dig, s = digest()
    best = min(rows)
    print("%s x%d first_chunk %d: total %s ms (best %.2f = %.2f + %.2f; %d envs running after the first launch, "
          "%d more launches), %.1f M env-steps/s, digest %s" % (
              cfg, n, fc, ["%.2f" % x[0] for x in rows], best[0], best[1], best[2], best[3], best[4],
              int(s["events"].sum()) / best[0] / 1e3, dig), flush=True)
