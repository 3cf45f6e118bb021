"""A/B of one configuration's run kernel between two libmxa builds (MXA_LIB selects the library):
python tools/ab_config.py CONFIG N_ENVS [REPS]  ->  run-kernel ms per episode batch."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
import mxabides

cfg, n = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
m = mxabides.VecMarket(cfg, (123456789 + np.arange(n)) & 0xFFFFFFFF)
m.set_parity_hash(False)
fc = int(os.environ.get("MXA_FIRST_CHUNK", "0"))  # mxa_set_launch_schedule (0: one launch)
if fc and hasattr(m.L, "mxa_set_launch_schedule"):
    m.set_launch_schedule(fc)
ms, nl = [], 0
for r in range(reps):
    m.reset()
    nl = m.run(chunk=1 << 22)
    ms.append(m.last_kernel_ms)
ev = int(m.summary()["events"].sum())
# one more episode with the parity hash on: a digest over every env's (events, hash) for A/B parity
m.set_parity_hash(True)
m.reset()
m.run(chunk=1 << 22)
s = m.summary()
dig = hashlib.sha1(np.ascontiguousarray(s["events"]).tobytes() + np.ascontiguousarray(s["hash"]).tobytes()).hexdigest()[:16]
print("%s%s %s x%d: run kernel %s ms (best %.1f), %.1f M env-steps/s, digest %s" % (
    os.path.basename(os.environ.get("MXA_LIB", "libmxa.so")), " first_chunk %d (%d launches)" % (fc, nl) if fc else "",
    cfg, n, ["%.1f" % x for x in ms], min(ms), ev / min(ms) / 1e3, dig))
