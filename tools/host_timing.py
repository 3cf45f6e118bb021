"""Wall time of each host call of one bench.py step (rmsc03 x4096), synchronized after each:
where the bench step's time goes outside the run kernel."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-optimal-execution_amd")]
import torch
import mxabides
from mxabides import shard

n = 4096
m = mxabides.VecMarket("rmsc03", shard.env_seeds(0, 0, 1, n), device=0)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
m.set_stream(stream.cuda_stream)
m.set_parity_hash(False)
res = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
for k in range(5):
    t = [time.perf_counter()]
    s = shard.env_seeds(k, 0, 1, n); t.append(time.perf_counter())
    m.set_seeds(s); t.append(time.perf_counter())
    m.reset(); t.append(time.perf_counter())
    nl = m.run(chunk=1 << 22); t.append(time.perf_counter())
    m.write_results(res.data_ptr()); x = res[:, 0].sum(); torch.cuda.synchronize(); t.append(time.perf_counter())
    d = [1000 * (b - a) for a, b in zip(t, t[1:])]
    print("step %d: seeds %.2f set_seeds %.2f reset %.2f run %.2f (kernel %.2f, %d launches) results %.2f  total %.2f ms"
          % (k, d[0], d[1], d[2], d[3], m.last_kernel_ms, nl, d[4], sum(d)), flush=True)
