"""World-size-2 rehearsal (gloo, CPU) of the DDQN learner's multi-GPU semantics (mxabides.ddqn,
BASELINE configs[3] on 8 GPUs): synchronous data parallelism.  Both ranks start from rank 0's
eval / target initialisation, every update all-reduces the gradient (mean over ranks) and the
live flag, so the two ranks hold the same policy after every update, and that policy equals one
learner's trained on the union of the two ranks' batches (ddqlearning_execution_agent.py:448-530
restated by oracle/ddqn_ref.train_step, dropout masks included).  On the GPU box the same code
runs over RCCL."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_UPDATES = 8
BATCH = 32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(rank, it):
    rs = np.random.RandomState(1000 * it + rank)
    return (rs.randint(0, 200, (BATCH, 2)).astype(np.float64), rs.randint(0, 24, BATCH),
            rs.randint(0, 200, (BATCH, 2)).astype(np.float64), rs.normal(0, 50, BATCH))


def _masks(rank, it, widths, rate=0.1):
    rs = np.random.RandomState(7 + 1000 * it + rank)
    return [rs.uniform(size=(BATCH, w)) >= rate for w in widths]


def _worker(rank, world, port, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "marl-optimal-execution_amd"),):
        sys.path.insert(0, p)
    from mxabides import ddqn
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # distinct seeds: without the broadcast the ranks would start from different nets
        L = ddqn.DDQNLearner(device="cpu", dropout=0.1, seed=11 + rank, dtype=torch.float64, group=dist.group.WORLD)
        widths = L.eval_model.dropout_widths()
        live = torch.tensor(rank == 0)  # one rank live is enough for the update to run everywhere
        for it in range(N_UPDATES):
            s, a, s2, r = _batch(rank, it)
            L.learn_on(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(s2), torch.from_numpy(r), live=live,
                       masks=[torch.from_numpy(m) for m in _masks(rank, it, widths)])
        np.save(os.path.join(out_dir, "eval_%d.npy" % rank), L.eflat.numpy())
        np.save(os.path.join(out_dir, "target_%d.npy" % rank), L.tflat.numpy())
        np.save(os.path.join(out_dir, "counter_%d.npy" % rank), np.asarray(L.learn_step_counter))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_learner_is_one_policy_on_the_union_of_batches(tmp_path):
    import ddqn_ref
    from mxabides import ddqn
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ev = [np.load(tmp_path / ("eval_%d.npy" % r)) for r in range(world)]
    tg = [np.load(tmp_path / ("target_%d.npy" % r)) for r in range(world)]
    assert np.array_equal(ev[0], ev[1]) and np.array_equal(tg[0], tg[1])  # one policy on the node
    assert int(np.load(tmp_path / "counter_1.npy")) == N_UPDATES
    # the single-learner reference: rank 0's initialisation, every update on the union of the
    # two ranks' batches (and masks); mean MSE over the union = the mean of the ranks' means
    L = ddqn.DDQNLearner(device="cpu", dropout=0.1, seed=11, dtype=torch.float64)
    layers = lambda net: [(l.weight.detach().numpy().T.copy(), l.bias.detach().numpy().copy())
                          for l in list(net.hidden) + [net.logits]]
    e, t = layers(L.eval_model), layers(L.target_model)
    rms = [(np.zeros_like(W), np.zeros_like(b)) for W, b in e]
    widths = L.eval_model.dropout_widths()
    c = 0
    for it in range(N_UPDATES):
        bs = [_batch(r, it) for r in range(world)]
        batch = tuple(np.concatenate([b[k] for b in bs]) for k in range(4))
        ms = [np.concatenate([_masks(r, it, widths)[j] for r in range(world)]).astype(np.float64)
              for j in range(len(widths))]
        e, t, rms, c, _ = ddqn_ref.train_step(e, t, rms, c, batch, masks=ms)
    flat = np.concatenate([np.concatenate([W.T.reshape(-1), b]) for W, b in e])
    np.testing.assert_allclose(ev[0], flat, rtol=1e-9, atol=1e-12)
    tflat = np.concatenate([np.concatenate([W.T.reshape(-1), b]) for W, b in t])
    np.testing.assert_allclose(tg[0], tflat, rtol=1e-9, atol=1e-12)
