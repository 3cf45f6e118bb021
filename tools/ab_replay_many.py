"""A/B of the replay step kernel in one k-step launch per episode (mxa_step_many, as bench.py
runs it) between libmxa builds (MXA_LIB selects the library):
python tools/ab_replay_many.py [TAPE] [N_ENVS] [REPS] -> kernel ms per episode (761 steps) and a
digest of every env's (events, hash) from one more episode with the parity hash on."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import numpy as np
import torch
from mxabides import tape
from mxabides.gym import VecABIDESEnv

tname = sys.argv[1] if len(sys.argv) > 1 else "IBM_2003-01-14"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
K = 761
tp = tape.Tape.load(os.path.join(ROOT, "tests", "golden", "tape_%s.npz" % tname))
v = VecABIDESEnv(tp, n)
rs = np.random.RandomState(0)
a = rs.uniform(0, 1, (K, n, 3))
a[:, :, 0] *= 0.01
act = torch.from_numpy(a).cuda()
obs = torch.empty((K, n, 9), dtype=torch.float64, device="cuda")
flags = torch.empty((K, n), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
v.set_stream(s.cuda_stream)
res = []
for rep in range(reps + 1):
    v.set_parity_hash(rep == reps)
    v.reset()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    v.step_many_device(K, act.data_ptr(), obs.data_ptr(), flags.data_ptr())
    e1.record(s)
    s.synchronize()
    if rep < reps:
        res.append(e0.elapsed_time(e1))
sm = v.summary()
dig = hashlib.sha1(np.ascontiguousarray(sm["events"]).tobytes() + np.ascontiguousarray(sm["hash"]).tobytes()).hexdigest()[:16]
print("%s replay %s x%d, %d steps in one launch: %s ms (best %.2f, %.4f ms per step), digest %s" % (
    os.path.basename(os.environ.get("MXA_LIB", "libmxa.so")), tname, n, K, ["%.2f" % x for x in res], min(res),
    min(res) / K, dig), flush=True)
