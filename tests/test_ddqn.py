"""DDQN learner (mxabides.ddqn) against the float64 numpy restatement of the reference's
arithmetic (oracle/ddqn_ref.py): action table, state discretization, Q-network forward,
train_neural_nets target, one Keras-RMSprop update, epsilon schedule, reward, replay ring.
CPU only (torch on the host); the device loop is tests/test_gpu_ddqn.py."""
import numpy as np
import pytest
import torch

import ddqn_ref
from mxabides import ddqn

REF_ACTIONS = {0: (0, 0.1), 5: (0, 2.5), 6: (1, 0.1), 13: (2, 0.5), 23: (3, 2.5)}


def _layers(net):
    lins = list(net.hidden) + [net.logits]
    return [(l.weight.detach().double().numpy().T.copy(), l.bias.detach().double().numpy().copy()) for l in lins]


def test_action_table_matches_reference_construction():
    ref = ddqn_ref.action_table(ddqn.SIZE_ALLOCATION, ddqn.SIZE_SCALE)
    assert ddqn.ACTIONS == ref and ddqn.N_ACTIONS == 24
    for k, v in REF_ACTIONS.items():
        assert ddqn.ACTIONS[k] == v
    assert ddqn.SIZE_SCALE == [0.1, 0.5, 1.0, 1.5, 2.0, 2.5]


def test_state_discretization_matches_np_digitize():
    task = ddqn.ExecutionTask(device="cpu")
    grid = ddqn.create_uniform_grid([0, 0], [1.0, 1.0], (200, 200))
    rs = np.random.RandomState(0)
    rem_t = rs.randint(0, 28, 4000).astype(np.float64)
    rem_q = np.concatenate([rs.randint(0, 100001, 3990), [0, 100000, 50000, 50250, 50500, 99500, 75000, 1, 2, 3]])
    rem_q = rem_q.astype(np.float64)
    obs = np.zeros((4000, 9))
    obs[:, 0], obs[:, 1] = rem_t, rem_q
    got = task.state(torch.from_numpy(obs)).numpy()
    for i in range(len(obs)):
        feats = [2 * (rem_t[i] / 27) - 1, 2 * (rem_q[i] / 100000.0) - 1, 0.1, 0.2, 0.3, 0.4]
        assert list(got[i]) == ddqn.discretize(feats, grid), i
    assert got.max() <= 199 and got.min() >= 0


def test_qnet_forward_matches_numpy():
    torch.manual_seed(0)
    for model in ("NNModel_1", "NNModel_2"):
        net = ddqn.QNet(2, 24, model, dropout=0.1).double().eval()
        x = np.random.RandomState(1).randint(0, 200, (64, 2)).astype(np.float64)
        ref = ddqn_ref.forward(_layers(net), x)[-1]
        with torch.no_grad():
            got = net(torch.from_numpy(x)).numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
        # glorot_uniform limits, zero biases (Keras Dense defaults)
        for lin in list(net.hidden) + [net.logits]:
            lim = np.sqrt(6.0 / (lin.in_features + lin.out_features))
            assert float(lin.weight.detach().abs().max()) <= lim and float(lin.bias.detach().abs().max()) == 0.0


def test_dropout_only_in_training():
    torch.manual_seed(0)
    net = ddqn.QNet(2, 24, dropout=0.5).double()
    x = torch.rand(256, 2, dtype=torch.float64) * 200
    net.eval()
    a, b = net(x), net(x)
    assert torch.equal(a, b)
    net.train()
    assert not torch.equal(net(x), a)


def _learner(**kw):
    return ddqn.DDQNLearner(device="cpu", dropout=0.0, seed=3, dtype=torch.float64, **kw)


def _batch(n=32, seed=5):
    rs = np.random.RandomState(seed)
    s = rs.randint(0, 200, (n, 2)).astype(np.float64)
    s2 = rs.randint(0, 200, (n, 2)).astype(np.float64)
    a = rs.randint(0, 24, n)
    r = rs.normal(0, 50, n)
    return s, a, s2, r


def test_q_target_matches_reference_target():
    L = _learner()
    with torch.no_grad():  # make target differ from eval
        for p in L.target_model.parameters():
            p.mul_(1.3)
    s, a, s2, r = _batch()
    got = L.q_target(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(s2), torch.from_numpy(r)).numpy()
    ref = ddqn_ref.q_target(_layers(L.eval_model), _layers(L.target_model), s, a, s2, r, 0.98)
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-9)


def test_target_and_eval_are_initialised_independently():
    """EvalModel and TargetModel are separate Keras models (QNets.py:54-60), not a copy"""
    L = _learner()
    for (W, b), (W2, b2) in zip(_layers(L.eval_model), _layers(L.target_model)):
        assert not np.array_equal(W, W2)


def test_learn_steps_match_reference_train_step():
    """ddqn_ref.train_step owns the whole update, target copy included (stale target first,
    then eval -> target every 5th learn step, then RMSprop): 17 updates over 4 target copies
    from distinct eval/target inits; the test only feeds batches"""
    L = _learner()
    ev, tg = _layers(L.eval_model), _layers(L.target_model)
    rms = [(np.zeros_like(W), np.zeros_like(b)) for W, b in ev]
    counter = 0
    for it in range(17):
        batch = _batch(seed=10 + it)
        ev, tg, rms, counter, loss = ddqn_ref.train_step(ev, tg, rms, counter, batch)
        cost = L.learn_on(*(torch.from_numpy(x) for x in batch))
        assert abs(float(cost) - loss) <= 1e-9 * max(1.0, loss), it
        for (W, b), (W2, b2) in zip(_layers(L.eval_model), ev):
            np.testing.assert_allclose(W, W2, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(b, b2, rtol=1e-9, atol=1e-9)
        for (W, b), (W2, b2) in zip(_layers(L.target_model), tg):
            np.testing.assert_allclose(W, W2, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(b, b2, rtol=1e-9, atol=1e-9)
    assert L.learn_step_counter == counter == 17


def test_masked_update_is_a_no_op():
    """learn_on(live=False): no target copy, no RMSprop step or state change, no counter/epsilon
    advance (the device-side guard run_episode uses once every env is done)"""
    L = _learner(epsilon_increment=0.1)
    e0, t0, r0 = L.eflat.clone(), L.tflat.clone(), L.rms.clone()
    batch = [torch.from_numpy(x) for x in _batch()]
    L.learn_on(*batch, live=torch.tensor(False))
    assert torch.equal(L.eflat, e0) and torch.equal(L.tflat, t0) and torch.equal(L.rms, r0)
    assert L.learn_step_counter == 0 and L.epsilon == 0 and L.cost_hist == []
    L.learn_on(*batch, live=torch.tensor(True))
    assert not torch.equal(L.eflat, e0) and torch.equal(L.tflat, e0)  # copied before the update
    assert L.learn_step_counter == 1 and len(L.cost_hist) == 1


def test_epsilon_schedule_overshoots_like_reference():
    L = _learner(epsilon_increment=0.4, epsilon_max=0.9)
    assert L.epsilon == 0
    seq = []
    s, a, s2, r = (torch.from_numpy(x) for x in _batch())
    for _ in range(4):
        L.learn_on(s, a, s2, r)
        seq.append(L.epsilon)
    assert seq == pytest.approx([0.4, 0.8, 1.2000000000000002, 0.9])
    assert _learner().epsilon == 0.9  # no increment: epsilon_max from the start


def test_choose_action_gating():
    L = _learner(epsilon_max=1.0)
    s = torch.from_numpy(_batch(n=512)[0])
    greedy = torch.argmax(L.q_values(s), 1)
    a0 = L.choose_action(s)  # empty memory: len + 1 > batch_size fails -> random
    assert (a0 != greedy).any() and a0.min() >= 0 and a0.max() < 24
    L.memory.add(s, a0, s, torch.zeros(512, dtype=torch.float64), torch.ones(512, dtype=torch.bool))
    assert torch.equal(L.choose_action(s), greedy)  # epsilon 1: always exploit
    L.mode = "test"
    assert torch.equal(L.choose_action(s), greedy)


def test_replay_ring_compacts_and_wraps():
    R = ddqn.ReplayRing(10, 2, "cpu")
    s = torch.arange(14, dtype=torch.float64).reshape(7, 2)
    a = torch.arange(7)
    r = torch.arange(7, dtype=torch.float64) * 10
    m = torch.tensor([1, 0, 1, 1, 0, 1, 1], dtype=torch.bool)
    assert R.add(s, a, s, r, m) == 5 and len(R) == 5
    assert R.a[:5].tolist() == [0, 2, 3, 5, 6] and R.r[:5].tolist() == [0, 20, 30, 50, 60]
    assert R.add(s, a, s, r, m) == 5 and R.add(s, a + 100, s, r, m) == 5
    assert len(R) == 10 and R.n == 15
    assert R.a[:10].tolist() == [100, 102, 103, 105, 106, 0, 2, 3, 5, 6]  # (row 10: masked-out rows)


def test_actions_and_reward_mapping():
    task = ddqn.ExecutionTask(quantity=100000, n_horizon=27, device="cpu")
    assert task.child == 3846
    obs = torch.zeros((24, 9), dtype=torch.float64)
    obs[:, 0], obs[:, 1] = 10, 80000
    act = task.actions(torch.arange(24), obs).numpy()
    for k, (alloc, scale) in ddqn.ACTIONS.items():
        assert round(act[k, 0] * 100000) == max(0, round(scale * 3846))
        assert tuple(act[k, 1:]) == ddqn.LEVEL_SHARES[alloc]
    obs[:, 0] = 1  # remaining_time == 1: the whole remaining quantity at level 1
    act = task.actions(torch.arange(24), obs).numpy()
    assert np.all(act[:, 0] == 0.8) and np.all(act[:, 1] == 1) and np.all(act[:, 2] == 0)
    # reward: fills (qty, price) of one step, BUY: cash falls by sum q*f
    fills = [(300, 10010), (200, 9990), (1000, 10000)]
    prev = torch.zeros((1, 8), dtype=torch.float64)
    prev[0, 0], prev[0, 2] = -5000000.0, 500
    cur = prev.clone()
    cur[0, 0] -= sum(q * f for q, f in fills)
    cur[0, 2] += sum(q for q, _ in fills)
    got = float(task.reward(prev, cur, torch.tensor([10002.5], dtype=torch.float64), 100000.0)[0])
    assert got == pytest.approx(ddqn_ref.step_reward(fills, 10002.5, 100000.0), rel=1e-12)
    assert float(task.reward(prev, prev, torch.tensor([1.0], dtype=torch.float64), 1e5)[0]) == 0.0


def test_dropout_on_learn_steps_match_reference_with_the_same_masks():
    """train_on_batch in training mode (Dropout 0.1 after layers 2-6, QNets.py:22-26; Keras scales
    kept units by 1 / (1 - rate)): the learner's update with its own drawn masks equals
    ddqn_ref.train_step fed the same masks, over 12 updates and 2 target copies"""
    L = ddqn.DDQNLearner(device="cpu", dropout=0.1, seed=4, dtype=torch.float64)
    ev, tg = _layers(L.eval_model), _layers(L.target_model)
    rms = [(np.zeros_like(W), np.zeros_like(b)) for W, b in ev]
    counter = 0
    dropped = 0
    for it in range(12):
        batch = _batch(seed=40 + it)
        masks = L.dropout_masks(32)
        dropped += sum(int((~m).sum()) for m in masks)
        ev, tg, rms, counter, loss = ddqn_ref.train_step(ev, tg, rms, counter, batch,
                                                         masks=[m.numpy().astype(np.float64) for m in masks])
        cost = L.learn_on(*(torch.from_numpy(x) for x in batch), masks=masks)
        assert abs(float(cost) - loss) <= 1e-9 * max(1.0, loss), it
        for (W, b), (W2, b2) in zip(_layers(L.eval_model), ev):
            np.testing.assert_allclose(W, W2, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(b, b2, rtol=1e-9, atol=1e-9)
    assert dropped > 0.05 * 12 * 32 * (64 + 128 + 128 + 64 + 32)  # about 10 % of the units dropped
    # the masks change the update: the same batches without dropout end elsewhere
    L0 = ddqn.DDQNLearner(device="cpu", dropout=0.0, seed=4, dtype=torch.float64)
    for it in range(12):
        L0.learn_on(*(torch.from_numpy(x) for x in _batch(seed=40 + it)))
    assert not torch.allclose(L0.eflat, L.eflat)


def test_exploration_stream_is_independent_of_masked_updates():
    """choose_action draws from its own stream: masked (no-op) updates between two acting steps
    do not change the actions; the masked updates' losses stay out of cost_hist"""
    s = torch.from_numpy(_batch(n=256)[0])
    acts = []
    for n_masked in (0, 3):
        L = _learner()
        L.memory.add(s, torch.zeros(256, dtype=torch.int64), s, torch.zeros(256, dtype=torch.float64),
                     torch.ones(256, dtype=torch.bool))
        a0 = L.choose_action(s)
        for _ in range(n_masked):
            L.learn(live=torch.tensor(False))
        acts.append((a0, L.choose_action(s)))
        assert L.cost_hist == []
    assert torch.equal(acts[0][1], acts[1][1])
