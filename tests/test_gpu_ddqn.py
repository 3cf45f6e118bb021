"""DDQN learner driving the rmsc03 + DummyRL composition on the GPU (mxabides.ddqn.run_episode):
the actions the learner chose are replayed through the C oracle's GymKernel env, and the
device episode must match it bit-exactly (event count and trace hash of every env, the
execution agent's cash and holdings), the per-step rewards must equal compute_reward summed
over the oracle's fills (float64, 1e-9), and the learner must have trained."""
import numpy as np
import pytest
import torch

import pyoracle
from mxabides import ddqn
from mxabides.gym import RL_STATE_WORDS, VecABIDESEnv

pytestmark = pytest.mark.gpu
SEEDS = [123456789, 2024, 7, 123, 99991, 31337, 4242, 555, 1, 2, 3, 4, 5, 6, 8, 9]


def _oracle_rl(o, rl_id):
    cash, shares, _ = o.agents()[rl_id]
    return float(cash), float(o.rl_state()[1])


def test_gpu_ddqn_episode_matches_oracle_replay():
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    v = VecABIDESEnv(seeds=SEEDS)
    v.set_stream(stream.cuda_stream)
    learner = ddqn.DDQNLearner(device="cuda", seed=1, batch_size=32)
    task = ddqn.ExecutionTask(device="cuda")
    oras = [None] * len(SEEDS)  # one oracle "process" per env: episode 2 continues its order ids
    for ep in range(2):
        seeds = [s + 1000 * ep for s in SEEDS]
        rec = []
        res = ddqn.run_episode(v, learner, task, seeds=seeds, record=rec)
        torch.cuda.synchronize()
        acts = torch.stack(rec).cpu().numpy()
        rewards = res["rewards"].cpu().numpy()
        arrival = res["arrival"].cpu().numpy()
        summ = v.summary()
        st = torch.zeros((len(SEEDS), RL_STATE_WORDS), dtype=torch.float64, device="cuda")
        v.write_rl_state(st.data_ptr())
        st = st.cpu().numpy()
        rl_id = v.n_agents - 1
        for e, seed in enumerate(seeds):
            if oras[e] is None:
                oras[e] = pyoracle.OracleGymEnv(seed=seed)
            else:
                oras[e].reset(seed=seed)
            o = oras[e]
            cash0, ex0 = _oracle_rl(o, rl_id)
            ref_r = []
            for i in range(len(acts)):
                _, done, rc = o.step(acts[i, e])
                cash1, ex1 = _oracle_rl(o, rl_id)
                if i >= 1:
                    dq = ex1 - ex0
                    ref_r.append(1e4 / 1e5 * (2 * dq + (cash1 - cash0) / arrival[e]) if dq > 0 else 0.0)
                cash0, ex0 = cash1, ex1
                if done or rc:
                    break
            assert summ["events"][e] == o.events and summ["hash"][e] == o.hash, (ep, e)
            assert v.agents(e)[rl_id][:2] == tuple(o.agents()[rl_id][:2]), (ep, e)
            assert st[e, 0] == o.agents()[rl_id][0] and st[e, 2] == o.rl_state()[1], (ep, e)
            n = len(ref_r)
            np.testing.assert_allclose(rewards[:n, e], ref_r, rtol=1e-9, atol=1e-9, err_msg="ep %d env %d" % (ep, e))
        assert res["stored"] > 0
    assert learner.learn_step_counter > 0
    assert all(np.isfinite(float(c)) for c in learner.cost_hist)
    assert len(set(acts[1:, :, 0].ravel().tolist())) > 3  # the learner varied its order sizes
    assert (rewards != 0).any()  # some orders filled


def test_gpu_qnet_matches_host():
    torch.manual_seed(0)
    net = ddqn.QNet(2, 24)
    x = torch.randint(0, 200, (4096, 2)).float()
    net.eval()
    with torch.no_grad():
        ref = net(x)
        got = net.cuda()(x.cuda()).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3)


def _layers(net):
    return [(lin.weight.detach().cpu().numpy().T.astype(np.float64), lin.bias.detach().cpu().numpy().astype(np.float64))
            for lin in list(net.hidden) + [net.logits]]


def _batch(n, seed):
    rs = np.random.RandomState(seed)
    return (rs.randint(0, 200, (n, 2)).astype(np.float64), rs.randint(0, 24, n), rs.randint(0, 200, (n, 2)).astype(np.float64),
            rs.normal(0, 50, n))


@pytest.mark.parametrize("dtype,rtol,atol", [(torch.float64, 1e-9, 1e-9), (torch.float32, 2e-3, 2e-4)])
def test_gpu_learner_updates_match_numpy_reference(dtype, rtol, atol):
    """train_neural_nets on the device against oracle/ddqn_ref.train_step, which owns the whole
    update (ddqlearning_execution_agent.py:448-530: target from the target net as it stands,
    THEN the eval -> target copy every replace_target_iter steps, then MSE + Keras RMSprop):
    the test only feeds batches. 18 updates spanning 4 target copies from distinct eval/target
    inits (QNets.py:54-60); exact to 1e-9 in float64 over the whole sequence, and for the fp32
    learner the bench runs, every update within fp32 tolerance of the reference step taken from
    the learner's own state"""
    import ddqn_ref
    L = ddqn.DDQNLearner(device="cuda", dropout=0.0, seed=3, batch_size=32, dtype=dtype)
    ev, tg = _layers(L.eval_model), _layers(L.target_model)
    assert not np.array_equal(ev[0][0], tg[0][0])
    rms = [(np.zeros_like(W), np.zeros_like(b)) for W, b in ev]
    counter = 0
    dv = lambda x: torch.from_numpy(x).to("cuda", dtype)
    for it in range(18):
        s, a, s2, r = _batch(32, 100 + it)
        if dtype == torch.float32:
            # fp32: each update against the reference step from the learner's own current state, so
            # the tolerance measures one update's rounding, not 18 updates of fp32 drift
            ev, tg = _layers(L.eval_model), _layers(L.target_model)
            rr = L.rms.detach().cpu().double().numpy()
            rms, off = [], 0
            for W, b in ev:
                rms.append((rr[off:off + W.size].reshape(W.shape[1], W.shape[0]).T.copy(),
                            rr[off + W.size:off + W.size + b.size].copy()))
                off += W.size + b.size
        ev, tg, rms, counter, loss = ddqn_ref.train_step(ev, tg, rms, counter, (s, a, s2, r))
        cost = L.learn_on(dv(s), torch.from_numpy(a).cuda(), dv(s2), dv(r))
        assert abs(float(cost) - loss) <= max(rtol, 1e-9) * max(1.0, loss) * (1 if dtype == torch.float64 else 10), it
        for net, ref in ((L.eval_model, ev), (L.target_model, tg)):
            for (W, b), (W2, b2) in zip(_layers(net), ref):
                np.testing.assert_allclose(W, W2, rtol=rtol, atol=atol, err_msg="update %d" % it)
                np.testing.assert_allclose(b, b2, rtol=rtol, atol=atol, err_msg="update %d" % it)
    assert L.learn_step_counter == 18


def test_gpu_learner_masked_update_is_a_no_op():
    """run_episode's device-side guard: an update with live == False changes nothing"""
    L = ddqn.DDQNLearner(device="cuda", dropout=0.0, seed=3, batch_size=32)
    e0, t0, r0 = L.eflat.clone(), L.tflat.clone(), L.rms.clone()
    s, a, s2, r = _batch(32, 7)
    dv = lambda x: torch.from_numpy(x).to("cuda", torch.float32)
    L.learn_on(dv(s), torch.from_numpy(a).cuda(), dv(s2), dv(r), live=torch.zeros((), dtype=torch.bool, device="cuda"))
    assert torch.equal(L.eflat, e0) and torch.equal(L.tflat, t0) and torch.equal(L.rms, r0)
    assert L.learn_step_counter == 0


def test_gpu_ddqn_fused_period_equals_torch_ops():
    """include/mxa_ddqn.h: run_episode's one-kernel bookkeeping (libmxa_ddqn.so) and the PyTorch
    ops give bitwise the same episodes: actions, rewards, step counts, replay rows, and the learner
    after its updates (weights, RMSprop state, counter, losses)"""
    assert ddqn.period_lib() is not None, "libmxa_ddqn.so not built"
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    seeds = SEEDS * 4  # 64 envs
    out = {}
    for fused in (False, True):
        v = VecABIDESEnv(seeds=seeds)
        v.set_stream(stream.cuda_stream)
        learner = ddqn.DDQNLearner(device="cuda", seed=5, batch_size=32)
        task = ddqn.ExecutionTask(device="cuda")
        eps = []
        for ep in range(3):
            rec = []
            res = ddqn.run_episode(v, learner, task, seeds=[s + 77 * ep for s in seeds], fused=fused, record=rec)
            eps.append({k: res[k].clone() for k in ("rewards", "actions", "returns", "env_steps", "stored", "flags")})
            eps[-1]["action_vectors"] = torch.stack(rec)  # ExecutionTask.actions (mxa_ddqn_actions when fused)
        torch.cuda.synchronize()
        m = learner.memory
        k = int(m.n_dev.item())
        out[fused] = (eps, m.s[:k].clone(), m.s2[:k].clone(), m.a[:k].clone(), m.r[:k].clone(), k,
                      learner.eflat.clone(), learner.tflat.clone(), learner.rms.clone(), learner.learn_step_counter,
                      learner.cost_hist)
    a, b = out[False], out[True]
    for ea, eb in zip(a[0], b[0]):
        for key in ea:
            assert torch.equal(ea[key], eb[key]), key
    assert a[5] == b[5] and a[5] > 0 and a[9] == b[9] and a[9] > 0
    for x, y in zip(a[1:5] + a[6:9], b[1:5] + b[6:9]):
        assert torch.equal(x, y)
    assert a[10] == b[10]
