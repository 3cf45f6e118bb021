"""Per-phase cycle totals of the GymKernel step kernel (MXA_PROF single-configuration build
with -DMXA_ONLY_CFG=3): one ABIDESEnv replay episode of n envs with zero actions.
usage: MXA_LIB=.../libmxa_profr.so python tools/prof_phases_replay.py [tape] [n_envs]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
from mxabides import _lib
from mxabides.gym import VecABIDESEnv
from mxabides.tape import Tape

tape = sys.argv[1] if len(sys.argv) > 1 else "IBM_2003-01-14"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
v = VecABIDESEnv(Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % tape)), n)
v.set_parity_hash(False)
buf = (ctypes.c_uint64 * 64)()
lib = _lib.load()
lib.mxa_prof_read(buf)
v.reset()
act = np.zeros((n, 3))
steps = 0
while True:
    obs, done, valid, err = v.step(act)
    steps += 1
    if done.all() or steps > 2000:
        break
lib.mxa_prof_read(buf)
vals = list(buf)
ev = int(v.summary()["events"].sum())
tot = sum(vals[0:16]) + sum(vals[30:38]) + vals[46] + sum(vals[48:56])
print("tape %s, %d envs, %d steps, events %d, cycles/event (sum over waves) %.0f" % (tape, n, steps, ev, tot / ev))
# buckets 2 + 2 * agent type (+1 wakeup); calls counted at bucket + 14. AG_REPLAY = 6 shares
# buckets 14/15 with the ACCEPTED/CANCELLED fast paths
names = ["pop+hash+rec_load", "requeue"] + ["%s.%s" % (a, w) for a in ["EX", "ZI", "NOISE", "VALUE", "MM", "MOM"]
                                              for w in ["msg", "wake"]] + ["REPLAY.msg+ACK", "REPLAY.wake+CXL"]
print("%-20s %8s %10s %12s %10s" % ("phase", "share", "cyc/event", "calls", "cyc/call"))
for i, nm in enumerate(names):
    if vals[i]:
        c = vals[i + 14] if i >= 2 else 0
        print("%-20s %7.1f%% %10.0f %12d %10.0f" % (nm, 100 * vals[i] / tot, vals[i] / ev, c, vals[i] / c if c else 0))
for i, nm in ((30, "rng_maint"), (31, "tail+rec_store"), (32, "encode+hash(+trace)"), (33, "q_remove")):
    print("%-20s %7.1f%% %10.0f" % (nm, 100 * vals[i] / tot, vals[i] / ev))
other = tot - sum(vals[i] for i in list(range(16)) + [30, 31, 32, 33])
print("%-20s %7.1f%% %10.0f" % ("(other buckets)", 100 * other / tot, other / ev))
