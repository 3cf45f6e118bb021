"""Per-phase cycle breakdown of the run kernel (MXA_PROF build): one rmsc03 episode batch.
usage: MXA_LIB=.../libmxa_prof.so python tools/prof_phases.py [config] [n_envs]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
import mxabides
from mxabides import _lib

cfg = sys.argv[1] if len(sys.argv) > 1 else "rmsc03"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
m = mxabides.VecMarket(cfg, (123456789 + np.arange(n)) & 0xFFFFFFFF)
m.set_parity_hash(os.environ.get("MXA_PROF_HASH", "0") == "1")  # off, as bench.py times it
buf = (ctypes.c_uint64 * 128)()
lib = _lib.load()
lib.mxa_prof_read(buf)  # clear
m.reset()
m.run()
lib.mxa_prof_read(buf)
v = list(buf)
ev = int(m.summary()["events"].sum())
names = ["pop+hash+rec_load", "requeue"] + ["%s.%s" % (a, w) for a in ["EX", "ZI", "NOISE", "VALUE", "MM", "MOM"] for w in ["msg", "wake"]]
names += ["ACCEPTED fast", "CANCELLED fast"]  # phases 14, 15 (counts 28, 29)
tot = v[0] + v[1] + sum(v[2:16]) + v[30] + v[31] + v[32] + v[33] + sum(v[34:38]) + v[46] + v[47] + sum(v[48:56]) + v[79] + sum(v[80:84])
print("events %d  total cycles/event (sum over waves) %.0f" % (ev, tot / ev))
print("%-20s %8s %10s %12s" % ("phase", "share", "cyc/event", "cyc/call"))
for i, nm in enumerate(names):
    c = v[16 + i - 2] if i >= 2 else 0
    print("%-20s %7.1f%% %10.0f %12s" % (nm, 100 * v[i] / tot, v[i] / ev, ("%.0f (%d calls)" % (v[i] / c, c)) if c else ""))
print("%-20s %7.1f%% %10.0f" % ("rng_maint", 100 * v[30] / tot, v[30] / ev))
print("%-20s %7.1f%% %10.0f" % ("tail+rec_store", 100 * v[31] / tot, v[31] / ev))
print("%-20s %7.1f%% %10.0f" % ("encode+hash(+trace)", 100 * v[32] / tot, v[32] / ev))
print("%-20s %7.1f%% %10.0f" % ("q_remove", 100 * v[33] / tot, v[33] / ev))
# event runs (phases 34-37, calls 38-41, member pops 42-45; 46 = detection that fell back)
for i, nm in enumerate(["run EX.CANCEL", "run EX.LIMIT", "run ACCEPTED", "run CANCELLED"]):
    c, mem = v[38 + i], v[42 + i]
    print("%-20s %7.1f%% %10.0f %12s  members %d (%.1f%% of pops, %.1f per run)"
          % (nm, 100 * v[34 + i] / tot, v[34 + i] / ev, ("%.0f (%d calls)" % (v[34 + i] / c, c)) if c else "",
             mem, 100 * mem / ev, mem / c if c else 0))
print("%-20s %7.1f%% %10.0f" % ("run fallback", 100 * v[46] / tot, v[46] / ev))
for i, nm in enumerate(["EX SPREAD_REQ", "EX TV_REQ", "EX LIMIT (single)", "EX CANCEL (single)", "EX other",
                        "VALUE SPREAD (place)", "MM SPREAD", "MM TV"]):
    c = v[56 + i]
    print("%-20s %7.1f%% %10.0f %12s" % (nm, 100 * v[48 + i] / tot, v[48 + i] / ev, ("%.0f (%d calls)" % (v[48 + i] / c, c)) if c else ""))
for i, nm in enumerate(["ZI SPREAD (place)", "ZI ACCEPTED", "ZI EXECUTED", "ZI other msg"]):
    c = v[112 + i]
    print("%-20s %7.1f%% %10.0f %12s" % (nm, 100 * v[80 + i] / tot, v[80 + i] / ev, ("%.0f (%d calls)" % (v[80 + i] / c, c)) if c else ""))
print("inclusive function timers (nested inside the phases above; cycles per call)")
for slot, nm in [(64, "send"), (65, "q_push"), (66, "handle_limit"), (67, "cancel_order"), (68, "b_best"),
                 (69, "o_observe"), (70, "bayes_r_T"), (71, "cancel_all"), (72, "place_limit"), (73, "ex_receive"),
                 (74, "ta_receive"), (75, "ta_wakeup"), (77, "rec_load"), (78, "rng_maint")]:
    c = v[slot + 32]
    if c:
        print("%-20s %10.0f cyc/event %8.0f cyc/call %6.2f calls/event" % (nm, v[slot] / ev, v[slot] / c, c / ev))
if v[47] or v[79]:  # MXA_PROF_WAITS builds
    print("%-20s %7.1f%% %10.0f" % ("payload wait", 100 * v[47] / tot, v[47] / ev))
    print("%-20s %7.1f%% %10.0f" % ("record wait", 100 * v[79] / tot, v[79] / ev))
