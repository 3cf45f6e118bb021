"""Per-phase cycle breakdown of the ABIDESEnv replay step kernel (MXA_PROF build of config 3):
one whole episode of N envs on a tape with random actions.
usage: MXA_LIB=.../libmxa_prof3.so python tools/prof_replay.py [tape] [n_envs]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
from mxabides import _lib, tape
from mxabides.gym import VecABIDESEnv

tname = sys.argv[1] if len(sys.argv) > 1 else "IBM_2003-01-14"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
tp = tape.Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % tname))
v = VecABIDESEnv(tp, n)
v.set_parity_hash(False)
lib = _lib.load()
buf = (ctypes.c_uint64 * 128)()
rs = np.random.RandomState(0)
lib.mxa_prof_read(buf)
for i in range(761):
    a = rs.uniform(0, 1, (n, 3))
    a[:, 0] *= 0.01
    v.step(a)
lib.mxa_prof_read(buf)
p = list(buf)
ev = int(v.summary()["events"].sum())
print("tape %s envs %d events %d (%.0f per env)" % (tname, n, ev, ev / n))
phases = [(0, "pop+rec_load", None), (1, "requeue", None), (30, "rng_maint", None), (31, "tail+rec_store", None),
          (32, "account/hash", None), (33, "q_remove", None), (14, "ACCEPTED fast", 28), (92, "REPLAY msg", 124),
          (93, "REPLAY wake", 125), (94, "DUMMYRL msg", 126), (95, "DUMMYRL wake", 127), (48, "EX SPREAD_REQ", 56),
          (50, "EX LIMIT", 58), (51, "EX CANCEL", 59), (52, "EX other (MODIFY)", 60)]
tot = sum(p[b] for b, _, _ in phases)
print("phase cycles per event (sum over waves): total %.0f" % (tot / ev))
for b, nm, c in phases:
    extra = " %8.0f cyc/call (%d calls)" % (p[b] / p[c], p[c]) if c is not None and p[c] else ""
    print("  %-22s %8.0f cyc/event %5.1f%%%s" % (nm, p[b] / ev, 100 * p[b] / max(1, tot), extra))
print("inclusive function timers (cycles per call, calls per event)")
for b, nm in [(84, "rp_handle_limit"), (85, "rp_modify"), (86, "rp_cancel"), (87, "mr_wakeup"), (91, "mr_place_record"),
              (88, "mr_receive"), (89, "rl_receive"), (90, "rl_place_orders"), (64, "send"), (65, "q_push"),
              (73, "ex_receive"), (74, "ta_receive"), (75, "ta_wakeup"), (77, "rec_load"),
              (76, " limit: gather"), (79, " limit: enter"), (80, " limit: notify"),
              (81, " wakeup: gather"), (82, " wakeup: setWakeup"), (83, " wakeup: place record")]:
    c = p[b + 32]
    if c:
        print("  %-22s %8.0f cyc/call %6.3f calls/event %8.0f cyc/event" % (nm, p[b] / c, c / ev, p[b] / ev))
