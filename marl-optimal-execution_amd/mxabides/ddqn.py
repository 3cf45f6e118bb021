"""DDQN optimal-execution learner on PyTorch-ROCm, fed by the MI355X market step.

Restates the reference's DDQLearningExecutionAgent learner (agent/execution/qlearning/
ddqlearning_execution_agent.py, TensorFlow 2.1 / Keras, requirements.txt:17) for thousands of
parallel envs on one device:

* the 24-action table: SIZE_ALLOCATION x SIZE_SCALE (ddqlearning_execution_agent.py:21-37);
* the state: `discretize([time_remaining, qty_remaining, ...], grid)` on a 200 x 200 uniform grid
  over [0, 1]^2 (:129, :301-331; agent/execution/util.py:5-40). `discretize` zips the six
  features with the two grid axes, so the state is the two bin indices of time and quantity;
* the Q-network NNModel_1 (util/model/QNets.py:7-27: Dense 32-64-128-128-64-32 ReLU, Dropout 0.1
  after layers 2-6, linear 24-way head; Keras defaults glorot_uniform / zero bias), EvalModel and
  TargetModel (QNets.py:54-60); NNModel_2 (:30-51) by name;
* epsilon-greedy `choose_action` (:333-362): exploit when U < epsilon and enough experience,
  else `randint(0, n_actions)`; epsilon = epsilon_max unless an increment is given (:100);
* `train_neural_nets` (:448-515): uniform sampling with replacement; q_next AND q_eval4next
  from the target net as it stands, THEN the eval -> target copy every `replace_target_iter`
  learn steps (:508-510), then the update; both from the TARGET net (so the "double" argmax is the target's own: kept as written), no terminal mask,
  one Keras `train_on_batch` (MSE, RMSprop lr 0.01, rho 0.9, eps 1e-7 outside the sqrt,
  TF 2.1 optimizer_v2), then the epsilon update that may overshoot epsilon_max by one step;
* `compute_reward` (:409-446): per fill (1 - (fill - arrival)/arrival) * qty/q0 * 1e4 (BUY).

The environment is the rmsc03 + DummyRL GymKernel composition on the device (BASELINE.json
configs[3]; libmxa MXA_RMSC03_RL), which is a build-defined composition: the reference runs the
DDQN agent only inside a Kernel config (config/execution/marketreplay/execution_marketreplay_ddqn.py)
and never under ABIDESEnv. What the composition changes, and why:

* actions go through DummyRL's action vector [x, level-1 share, level-2 share] (dummy_rl:138-158,
  q/q0 == 1 by the reference's own quirk): `x = qty/q0` places exactly `qty`; allocation 1 ->
  (1, 0), 2 -> (0.5, 0.5), 3 -> (0.34, 0.66) (levels 2-3 merged: order_level is 2); allocation 0
  (a MARKET order in the reference) has no DummyRL counterpart and posts at the level-1 bid.
  The last step (remaining_time == 1) places the whole remaining quantity (:388-390);
* the reward of a step is the SUM of `compute_reward` over the step's fills, from the agent's
  cash and executed-quantity change (sum_i q_i (2 - f_i/A) = 2 dq + dcash/A for a BUY); the
  reference overwrites the experience reward per message (acceptance 0, execution r), an
  artefact of message order that a per-step environment cannot see;
* one learner serves every env (shared replay, one policy); `batch_size`, `train_every` and
  `updates_per_train` default to the reference's 32, 5 and 1.

Across GPUs (bench.py --gpus N, BASELINE configs[3]) the learner is synchronous data-parallel:
with `group` (a torch.distributed process group over RCCL) the eval and target nets start from
rank 0's initialisation (broadcast), every update all-reduces the live-weighted gradient and the
count of live ranks in one message, and every rank applies the same RMSprop step, so ONE policy
serves the whole node. Each rank samples its batch from its own envs' replay; the update equals
one learner's on the union of the LIVE ranks' batches (a rank whose envs are done, or whose replay
is below the batch size, contributes nothing; tests/test_ddqn_multirank.py). Every rank runs the
same collectives on every learn() call, whatever its replay size. The market
results of a given action sequence are world-size invariant (envs shard by global index,
mxabides.shard); the policy trajectory depends on the world size through that batch union.

Random streams: `gen` draws choose_action's exploration, `gen_sample` the batch indices and
`gen_drop` the dropout masks (Keras Dropout 0.1 in train_on_batch). A masked update (learn with
live false) still draws its batch and masks, so those two streams advance on it; the exploration
stream does not.

Everything runs on the device stream the env steps on; the only host read is the stored-transition
count, when the replay ring's host-side bounds cannot decide the batch-size test.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

# ddqlearning_execution_agent.py:21-37
SIZE_ALLOCATION = {1: [1, 0, 0, 0], 2: [0.5, 0.5, 0, 0], 3: [0.34, 0.33, 0.33, 0]}
SIZE_SCALE = [0.1] + [i * 0.5 for i in range(1, 6)]


def _action_table():
    alloc = sorted(list(SIZE_ALLOCATION.keys()) + [0])
    acts, k = {}, 0
    for a in alloc:
        for s in SIZE_SCALE:
            acts[k] = (a, s)
            k += 1
    return acts


ACTIONS = _action_table()
N_ACTIONS = len(ACTIONS)  # 24 (execution_marketreplay_ddqn.py:244)
GRID_BINS = (200, 200)    # create_uniform_grid(low=[0, 0], high=[1, 1], bins=(200, 200)), :129

# DummyRL level shares per allocation type (levels >= 2 merged: order_level 2); 0 = MARKET -> level 1
LEVEL_SHARES = {0: (1.0, 0.0), 1: (1.0, 0.0), 2: (0.5, 0.5), 3: (0.34, 0.66)}


def create_uniform_grid(low, high, bins=(10, 10)):
    """agent/execution/util.py:5-22: interior split points per dimension."""
    return [np.linspace(low[d], high[d], bins[d] + 1)[1:-1] for d in range(len(bins))]


def discretize(sample, grid):
    """agent/execution/util.py:25-40: np.digitize per dimension (zip truncates to the grid)."""
    return list(int(np.digitize(s, g)) for s, g in zip(sample, grid))


class QNet(nn.Module):
    """NNModel_1 / NNModel_2 (util/model/QNets.py:7-51) with Keras Dense defaults."""

    WIDTHS = {"NNModel_1": (32, 64, 128, 128, 64, 32), "NNModel_2": (32, 64, 128, 256, 128, 64, 32)}

    def __init__(self, n_in=2, n_actions=N_ACTIONS, model="NNModel_1", dropout=0.1, generator=None):
        super().__init__()
        w = self.WIDTHS[model]
        dims = (n_in,) + w
        self.hidden = nn.ModuleList(nn.Linear(dims[i], dims[i + 1]) for i in range(len(w)))
        self.logits = nn.Linear(w[-1], n_actions)
        self.p = dropout
        with torch.no_grad():
            for lin in list(self.hidden) + [self.logits]:  # glorot_uniform kernel, zero bias
                lim = math.sqrt(6.0 / (lin.in_features + lin.out_features))
                lin.weight.uniform_(-lim, lim, generator=generator)
                lin.bias.zero_()

    def dropout_widths(self):
        """the widths of the Dropout layers (after hidden layers 2..n, QNets.py:22-26)"""
        return [lin.out_features for lin in list(self.hidden)[1:]]

    def forward(self, x, masks=None):
        """masks: the keep masks (0/1, [batch, width]) of the dropout layers in training mode;
        kept units are scaled by 1 / (1 - rate) as Keras' Dropout does (TF 2.1 nn.dropout)"""
        for i, lin in enumerate(self.hidden):
            x = torch.relu(lin(x))
            if i >= 1 and self.p > 0 and self.training:  # dropout after layers 2..n (QNets.py:22-26)
                if masks is None:
                    x = nn.functional.dropout(x, self.p, True)
                else:
                    x = x * masks[i - 1].to(x.dtype) / (1.0 - self.p)
        return self.logits(x)


class ReplayRing:
    """Device-resident experience (s, a, s', r) of every env (the reference keeps one
    OrderedDict per agent, :115-116). Valid rows are compacted with a prefix sum, no host loop.

    The row count lives on the device (`n_dev`); the host keeps bounds on it (`n_lb`, `n_ub`) and
    reads it only when a size test cannot be decided from them, so the per-step loop does not
    wait for the GPU (in practice one read per training run)."""

    def __init__(self, capacity, n_state, device):
        self.cap = int(capacity)
        # one extra row: masked-out rows of a batched append are written there
        self.s = torch.zeros((self.cap + 1, n_state), dtype=torch.float32, device=device)
        self.s2 = torch.zeros_like(self.s)
        self.a = torch.zeros(self.cap + 1, dtype=torch.int64, device=device)
        self.r = torch.zeros(self.cap + 1, dtype=torch.float32, device=device)
        self.n_dev = torch.zeros((), dtype=torch.int64, device=device)  # rows written so far
        self.n_lb = 0  # host bounds on n_dev
        self.n_ub = 0

    def add_device(self, s, a, s2, r, mask):
        """append rows where mask without a host read; returns the count as a device scalar"""
        m = mask.to(torch.int64)
        c = torch.cumsum(m, 0)
        pos = torch.where(mask, (self.n_dev + c - 1) % self.cap, torch.full_like(c, self.cap))
        self.s[pos] = s.float()
        self.s2[pos] = s2.float()
        self.a[pos] = a
        self.r[pos] = r.float()
        k = c[-1] if len(c) else torch.zeros((), dtype=torch.int64, device=m.device)
        self.n_dev += k
        self.n_ub += len(mask)
        return k

    def add(self, s, a, s2, r, mask):
        """append rows where mask; returns the number appended (one host read)."""
        k = int(self.add_device(s, a, s2, r, mask).item())
        self.n_lb = int(self.n_dev.item())
        return k

    @property
    def n(self):
        return int(self.n_dev.item())

    def more_than(self, x):
        """len(self) > x, reading the device count only when the host bounds cannot decide"""
        if min(self.n_lb, self.cap) > x:
            return True
        if min(self.n_ub, self.cap) <= x:
            return False
        self.n_lb = int(self.n_dev.item())
        self.n_ub = max(self.n_ub, self.n_lb)
        return min(self.n_lb, self.cap) > x

    def __len__(self):
        return min(self.n, self.cap)


class DDQNLearner:
    """DDQLearningExecutionAgent's learner (ddqlearning_execution_agent.py:40-131, 333-362, 448-515).

    Eval and target parameters each live in one flat device buffer (`eflat`, `tflat`; the
    modules' parameters are views of it), so the target copy and the RMSprop step are single
    elementwise passes and every update can be masked on the device: `learn(live=...)` with a
    device bool makes the whole update (target copy, RMSprop step and its state, epsilon,
    `learn_step_counter`) a no-op when it is false, without a host read. The counter and epsilon
    are device scalars for the same reason."""

    def __init__(self, n_state=2, n_actions=N_ACTIONS, replace_target_iter=5, batch_size=32, learning_rate=0.01,
                 epsilon_increment=None, epsilon_max=0.9, reward_decay=0.98, mode="train", model="NNModel_1",
                 dropout=0.1, capacity=1 << 20, device="cuda", seed=0, dtype=torch.float32, group=None):
        self.device = torch.device(device)
        self.dtype = dtype
        self.gen = torch.Generator(device=self.device)  # choose_action's exploration
        self.gen.manual_seed(seed)
        self.gen_sample = torch.Generator(device=self.device)  # train_neural_nets' batch indices
        self.gen_sample.manual_seed(seed + (1 << 20))
        self.gen_drop = torch.Generator(device=self.device)  # train_on_batch's dropout masks
        self.gen_drop.manual_seed(seed + (2 << 20))
        cpu = torch.Generator()
        cpu.manual_seed(seed)
        # EvalModel and TargetModel are two separately initialised Keras models (QNets.py:54-60):
        # two draws from the same generator, not a copy
        self.eval_model, self.eflat = self._flat(QNet(n_state, n_actions, model, dropout, cpu))
        self.target_model, self.tflat = self._flat(QNet(n_state, n_actions, model, dropout, cpu))
        self.n_actions = n_actions
        self.replace_target_iter = replace_target_iter
        self.batch_size = batch_size
        self.learning_rate = learning_rate
        self.epsilon_increment = epsilon_increment
        self.epsilon_max = epsilon_max
        eps0 = 0.0 if epsilon_increment is not None else epsilon_max  # :100
        self._eps = torch.tensor(eps0, dtype=torch.float64, device=self.device)
        self.reward_decay = reward_decay
        self.mode = mode
        self._counter = torch.zeros((), dtype=torch.int64, device=self.device)
        # per learn() call: the loss and whether the update ran (device buffers, grown on the host
        # side: the call count is known without reading the device)
        self._cost = torch.zeros(256, dtype=torch.float64, device=self.device)
        self._cost_live = torch.zeros(256, dtype=torch.bool, device=self.device)
        self._ncost = 0
        # Keras RMSprop (TF 2.1 optimizer_v2, momentum 0, not centered): rho 0.9, epsilon 1e-7
        self.rho, self.rms_eps = 0.9, 1e-7
        self.rms = torch.zeros_like(self.eflat)
        self.memory = ReplayRing(capacity, n_state, self.device)
        # synchronous data parallelism over the ranks of `group` (module docstring)
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if group is not None else 1
        if self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not dist.group.WORLD else 0
            dist.broadcast(self.eflat, src, group=group)
            dist.broadcast(self.tflat, src, group=group)

    def _flat(self, net):
        net = net.to(self.device, self.dtype)
        params = list(net.parameters())
        flat = torch.cat([p.detach().reshape(-1) for p in params]).contiguous()
        off = 0
        for p in params:
            k = p.numel()
            p.data = flat[off:off + k].view_as(p)
            off += k
        return net, flat

    @property
    def learn_step_counter(self):
        return int(self._counter.item())

    @property
    def epsilon(self):
        return float(self._eps.item())

    @property
    def cost_hist(self):
        """the losses of the updates that ran (one host read; not on the step path)"""
        n = self._ncost
        c, live = self._cost[:n].cpu(), self._cost_live[:n].cpu()
        return [float(x) for x, ok in zip(c.tolist(), live.tolist()) if ok]

    def _record_cost(self, loss, live):
        if self._ncost == len(self._cost):
            self._cost = torch.cat([self._cost, torch.zeros_like(self._cost)])
            self._cost_live = torch.cat([self._cost_live, torch.zeros_like(self._cost_live)])
        self._cost[self._ncost] = loss.to(torch.float64)
        self._cost_live[self._ncost] = live
        self._ncost += 1

    def dropout_masks(self, n):
        """train_on_batch's dropout keep masks for a batch of n (Keras: keep where U >= rate)"""
        p = self.eval_model.p
        if p <= 0:
            return None
        return [torch.rand((n, w), generator=self.gen_drop, device=self.device, dtype=torch.float64) >= p
                for w in self.eval_model.dropout_widths()]

    # ---- acting (choose_action, :333-362)
    def q_values(self, s):
        self.eval_model.eval()  # Keras predict(): training=False, no dropout
        with torch.no_grad():
            return self.eval_model(s.to(self.dtype))

    def choose_action(self, s):
        """s [n, n_state] -> actions [n] int64 (epsilon-greedy per env in train mode)."""
        n = s.shape[0]
        greedy = torch.argmax(self.q_values(s), dim=1)
        if self.mode == "test":
            return greedy
        u = torch.rand(n, generator=self.gen, device=self.device, dtype=torch.float64)
        rnd = torch.randint(0, self.n_actions, (n,), generator=self.gen, device=self.device)
        exploit = (u < self._eps) & self.memory.more_than(self.batch_size - 1)  # len + 1 > batch_size
        return torch.where(exploit, greedy, rnd)

    # ---- learning (train_neural_nets, :448-515)
    def q_target(self, s, a, s2, r):
        """the reference's target: both q_next and q_eval4next from the target net (:486-505)."""
        self.target_model.eval()
        self.eval_model.eval()
        with torch.no_grad():
            s, s2, r = s.to(self.dtype), s2.to(self.dtype), r.to(self.dtype)
            q_next = self.target_model(s2)
            q_eval4next = self.target_model(s2)
            q_eval = self.eval_model(s)
            tgt = q_eval.clone()
            idx = torch.arange(s.shape[0], device=s.device)
            best = torch.argmax(q_eval4next, dim=1)
            tgt[idx, a] = r + self.reward_decay * q_next[idx, best]
        return tgt

    def learn_on(self, s, a, s2, r, live=None, masks=None):
        """one train_neural_nets update on a given batch, in the reference's order: the target
        from the target net as it stands (:486-505), THEN the eval -> target copy when
        learn_step_counter % replace_target_iter == 0 (:508-510), then train_on_batch (:513).
        `live` (device bool, default true) masks the whole update; `masks` are the dropout keep
        masks (default: drawn from gen_drop). With a process group the update is one learner's on
        the union of the LIVE ranks' batches: each rank's gradient is weighted by its own live
        flag and the sum is divided by the number of live ranks (one all-reduce carries both), so a
        rank whose envs are all done adds nothing from its stale replay; the update runs when any
        rank is live. Every rank issues the same collectives on every call. Returns the (local)
        loss."""
        if live is None:
            live = torch.ones((), dtype=torch.bool, device=self.device)
        local_live = live
        if masks is None:
            masks = self.dropout_masks(s.shape[0])
        tgt = self.q_target(s, a, s2, r)
        self.eval_model.train()  # train_on_batch: training=True (dropout active)
        for p in self.eval_model.parameters():
            p.grad = None
        loss = torch.mean((self.eval_model(s.to(self.dtype), masks) - tgt) ** 2)
        loss.backward()
        with torch.no_grad():
            g = torch.cat([p.grad.reshape(-1) for p in self.eval_model.parameters()])
            if self.world > 1:  # one policy for the node: the mean gradient over the live ranks
                import torch.distributed as dist
                w = local_live.to(g.dtype).reshape(1)
                gl = torch.cat([g * w, w])
                dist.all_reduce(gl, group=self.group)
                n_live = gl[-1]
                live = n_live > 0
                g = gl[:-1] / torch.clamp(n_live, min=1)
            # the target copy comes after the target (:508-510), before the RMSprop step; the
            # gradient above is the eval net's and does not read the target parameters after
            # q_target, so the copy can follow the all-reduce
            do_copy = live & (self._counter % self.replace_target_iter == 0)
            self.tflat.copy_(torch.where(do_copy, self.eflat, self.tflat))
            rms = self.rho * self.rms + (1 - self.rho) * g * g
            self.rms.copy_(torch.where(live, rms, self.rms))
            step = self.learning_rate * g / (torch.sqrt(self.rms) + self.rms_eps)
            self.eflat.sub_(torch.where(live, step, torch.zeros_like(step)))
            if self.epsilon_increment is not None:  # :515, may overshoot epsilon_max by one step
                e = torch.where(self._eps < self.epsilon_max, self._eps + self.epsilon_increment,
                                torch.full_like(self._eps, self.epsilon_max))
                self._eps.copy_(torch.where(live, e, self._eps))
            self._counter += live.to(torch.int64)
        for p in self.eval_model.parameters():
            p.grad = None
        loss = loss.detach()
        self._record_cost(loss, live)
        return loss

    def learn(self, live=None):
        """sample a batch with replacement (np.random.choice(current_size, batch)) and update."""
        m = self.memory
        if self.world > 1:
            # the size test is per rank (its own envs' outcomes fill its replay), but the
            # collectives of learn_on must pair up on every rank: a rank below the batch size
            # still takes part, with its own update masked off (an empty replay samples row 0)
            ok = torch.clamp(m.n_dev, max=m.cap) > self.batch_size
            live = ok if live is None else (live & ok)
        elif not m.more_than(self.batch_size):
            return None
        size = torch.clamp(m.n_dev, max=m.cap).to(torch.float64)  # the current size, on the device
        u = torch.rand(self.batch_size, generator=self.gen_sample, device=self.device, dtype=torch.float64)
        idx = torch.clamp((u * size).to(torch.int64), max=m.cap - 1)
        return self.learn_on(m.s[idx], m.a[idx], m.s2[idx], m.r[idx], live=live)


class ExecutionTask:
    """Maps the rmsc03 + DummyRL env (obs float64[9], agent state) to the DDQN's state, action
    and reward (ddqlearning_execution_agent.py:301-331, 364-407, 409-446).

    obs[0] = remaining horizon steps, obs[1] = remaining quantity (dummy_rl:294-315); the
    horizon has `n_horizon` points; the parent order is `quantity` shares BUY."""

    def __init__(self, quantity=100000, n_horizon=27, device="cuda"):
        self.q0 = float(quantity)
        self.nh = int(n_horizon)
        self.child = int(self.q0 / (self.nh - 1))  # generate_schedule: int(quantity / (len - 1))
        g = create_uniform_grid([0, 0], [1.0, 1.0], GRID_BINS)
        self.grid = [torch.tensor(x, dtype=torch.float64, device=device) for x in g]
        tab = np.zeros((N_ACTIONS, 3))
        for k, (alloc, scale) in ACTIONS.items():
            tab[k] = (max(0, round(scale * self.child)) / self.q0,) + LEVEL_SHARES[alloc]
        self.table = torch.tensor(tab, dtype=torch.float64, device=device)

    def state(self, obs):
        """discretize([2*rem_t/len - 1, 2*rem_q/q0 - 1]) -> float [n, 2] bin indices."""
        tr = 2 * (obs[:, 0] / self.nh) - 1
        qr = 2 * (obs[:, 1] / self.q0) - 1
        # np.digitize(x, increasing bins) == torch.bucketize(x, bins, right=True)
        return torch.stack([torch.bucketize(tr, self.grid[0], right=True),
                            torch.bucketize(qr, self.grid[1], right=True)], 1).to(torch.float32)

    def actions(self, a, obs):
        """DDQN action index -> DummyRL action vector [n, 3] float64 (take_action, :364-407)."""
        act = self.table[a].clone()
        last = obs[:, 0] == 1  # remaining_time == 1: the whole remaining quantity, allocation 0
        act[:, 0] = torch.where(last, obs[:, 1] / self.q0, act[:, 0])
        act[:, 1] = torch.where(last, torch.ones_like(act[:, 1]), act[:, 1])
        act[:, 2] = torch.where(last, torch.zeros_like(act[:, 2]), act[:, 2])
        return act

    @staticmethod
    def reward(prev, cur, arrival, q0):
        """sum over the step's fills of compute_reward (BUY): 1e4/q0 * (2 dq + dcash / A);
        prev/cur are mxa_write_rl_state rows (CASH, holdings, executed, ...)."""
        dq = cur[:, 2] - prev[:, 2]
        dcash = cur[:, 0] - prev[:, 0]
        return torch.where(dq > 0, 1e4 / q0 * (2 * dq + dcash / arrival), torch.zeros_like(dq))


_PERIOD_LIB = None


def period_lib():
    """libmxa_ddqn.so (include/mxa_ddqn.h): the per-period bookkeeping kernel of run_episode;
    None when it is not built"""
    global _PERIOD_LIB
    if _PERIOD_LIB is None:
        import ctypes
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libmxa_ddqn.so")
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        P, I, I64, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
        L.mxa_ddqn_period.argtypes = [P, I, I, I, I] + [P] * 13 + [P, I, P, I, D, D, D, P, P, P, P, I64, P, P]
        L.mxa_ddqn_state.argtypes = [P, I, I, P, P, I, P, I, D, D, P]
        L.mxa_ddqn_actions.argtypes = [P, I, I, P, P, P, D, P]
        _PERIOD_LIB = L
    return _PERIOD_LIB


def _state_device(L, task, obs, out):
    rc = L.mxa_ddqn_state(torch.cuda.current_stream().cuda_stream, obs.shape[0], obs.shape[1], obs.data_ptr(),
                          task.grid[0].data_ptr(), task.grid[0].numel(), task.grid[1].data_ptr(), task.grid[1].numel(),
                          float(task.nh), task.q0, out.data_ptr())
    if rc:
        raise RuntimeError("mxa_ddqn_state: hip error %d" % rc)
    return out


def run_episode(env, learner, task, seeds=None, train_every=5, updates_per_train=1, record=None, timing=None,
                fused=None):
    """fused (default: a learner on the GPU with libmxa_ddqn.so built): the bookkeeping after each
    step in one kernel (include/mxa_ddqn.h), bitwise the same as the PyTorch ops that fused=False
    runs (tests/test_gpu_ddqn.py; 59.9 -> 55.8 ms per rmsc03_ddqn x4096 episode on one box)."""
    L = period_lib() if fused is not False and learner.device.type == "cuda" else None
    if fused and L is None:
        raise RuntimeError("run_episode(fused=True): libmxa_ddqn.so is not built (build_lib.build_ddqn)")
    if L is not None:
        return _run_episode_fused(L, env, learner, task, seeds, train_every, updates_per_train, record, timing)
    return _run_episode_torch(env, learner, task, seeds, train_every, updates_per_train, record, timing)


def _run_episode_fused(L, env, learner, task, seeds, train_every, updates_per_train, record, timing):
    """run_episode with the per-period bookkeeping in one launch; same order of RNG draws, replay
    appends and updates as _run_episode_torch"""
    from .gym import OBS_SIZE, RL_STATE_WORDS
    dev = learner.device
    n = env.n_envs
    nh = task.nh
    env.reset(seeds=seeds)
    obs = torch.zeros((n, OBS_SIZE), dtype=torch.float64, device=dev)
    flags = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros((n, RL_STATE_WORDS), dtype=torch.float64, device=dev)
    prev = torch.zeros_like(st)
    act0 = torch.zeros((n, 3), dtype=torch.float64, device=dev)
    env.step_device(act0.data_ptr(), obs.data_ptr(), flags.data_ptr())
    env.write_rl_state(st.data_ptr())
    if record is not None:
        record.append(act0.clone())
    alive = ((flags & 2) != 0) & ((flags & 5) == 0)
    alive_next = torch.zeros_like(alive)
    live = torch.zeros((), dtype=torch.bool, device=dev)
    lob_ok = (st[:, 7] == 3)
    arrival = torch.where(lob_ok, (st[:, 3] + st[:, 4]) / 2, torch.ones_like(st[:, 3])).contiguous()
    rw = torch.zeros((nh, n), dtype=torch.float64, device=dev)
    actions = []
    stored = torch.zeros((), dtype=torch.int64, device=dev)
    env_steps = alive.to(torch.int64)
    s = _state_device(L, task, obs, torch.empty((n, 2), dtype=torch.float32, device=dev))
    s2 = torch.empty_like(s)
    m = learner.memory
    train = learner.mode == "train"
    g0, g1 = task.grid
    table = task.table.contiguous()
    act = torch.empty((n, 3), dtype=torch.float64, device=dev)
    for step_counter in range(nh):
        a = learner.choose_action(s).contiguous()
        rc = L.mxa_ddqn_actions(torch.cuda.current_stream().cuda_stream, n, obs.shape[1], obs.data_ptr(), a.data_ptr(),
                                table.data_ptr(), task.q0, act.data_ptr())
        if rc:
            raise RuntimeError("mxa_ddqn_actions: hip error %d" % rc)
        if record is not None:
            record.append(act.clone())
        st, prev = prev, st  # write_rl_state fills the other buffer: prev keeps the state before the step
        if timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        env.step_device(act.data_ptr(), obs.data_ptr(), flags.data_ptr())
        if timing is not None:
            e1.record()
            timing.append((e0, e1))
        env.write_rl_state(st.data_ptr())
        rc = L.mxa_ddqn_period(torch.cuda.current_stream().cuda_stream, n, obs.shape[1], st.shape[1], int(train),
                               obs.data_ptr(), st.data_ptr(), prev.data_ptr(), arrival.data_ptr(), flags.data_ptr(),
                               alive.data_ptr(), alive_next.data_ptr(), live.data_ptr(), s.data_ptr(), a.data_ptr(),
                               s2.data_ptr(), rw[step_counter].data_ptr(), env_steps.data_ptr(), g0.data_ptr(),
                               g0.numel(), g1.data_ptr(), g1.numel(), float(nh), task.q0, 1e4 / task.q0,
                               m.s.data_ptr(), m.s2.data_ptr(), m.a.data_ptr(), m.r.data_ptr(), m.cap,
                               m.n_dev.data_ptr(), stored.data_ptr())
        if rc:
            raise RuntimeError("mxa_ddqn_period: hip error %d" % rc)
        if train:
            m.n_ub += n
            if step_counter % train_every == 0:
                for _ in range(updates_per_train):
                    learner.learn(live=live)
        actions.append(a)
        alive, alive_next = alive_next, alive
        s, s2 = s2, s
    return {"rewards": rw if nh else None, "actions": torch.stack(actions) if actions else None,
            "returns": rw.sum(0), "flags": flags, "arrival": arrival, "stored": stored, "env_steps": env_steps,
            "steps": nh + 1}


def _run_episode_torch(env, learner, task, seeds=None, train_every=5, updates_per_train=1, record=None, timing=None):
    """One episode of every env of a VecABIDESEnv (rmsc03 + DummyRL) driven by the learner, all on
    the current torch stream (the env must step on it: env.set_stream). Mirrors the agent's
    per-period loop (place_order, :275-299): observe, choose, act, then store the completed
    transition and train every `train_every` periods (train_step_counter % 5 == 0, :286-293).

    Returns a dict of device tensors (rewards [steps, n], actions [steps, n], flags) and the
    number of stored transitions. `record` (a list) receives the per-step action vectors;
    `timing` (a list) receives a (start, end) torch.cuda.Event pair around every step launch."""
    from .gym import OBS_SIZE, RL_STATE_WORDS
    dev = learner.device
    n = env.n_envs
    nh = task.nh
    env.reset(seeds=seeds)
    obs = torch.zeros((n, OBS_SIZE), dtype=torch.float64, device=dev)
    flags = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros((n, RL_STATE_WORDS), dtype=torch.float64, device=dev)
    act0 = torch.zeros((n, 3), dtype=torch.float64, device=dev)  # first step: no cached LOB, nothing placed
    env.step_device(act0.data_ptr(), obs.data_ptr(), flags.data_ptr())
    env.write_rl_state(st.data_ptr())
    if record is not None:
        record.append(act0.clone())
    alive = ((flags & 2) != 0) & ((flags & 5) == 0)
    lob_ok = (st[:, 7] == 3)
    arrival = torch.where(lob_ok, (st[:, 3] + st[:, 4]) / 2, torch.ones_like(st[:, 3]))  # mid at start_time
    rewards, actions = [], []
    stored = torch.zeros((), dtype=torch.int64, device=dev)
    env_steps = alive.to(torch.int64)  # per env: ABIDESEnv.step calls taken while alive (the first one included)
    step_counter = 0
    # every horizon step is enqueued without waiting for the GPU (no host read of `alive` except
    # on training steps): envs that are done stay done in the step kernel, and their rows are
    # masked out below
    for _ in range(nh):
        s = task.state(obs)
        a = learner.choose_action(s)
        act = task.actions(a, obs)
        if record is not None:
            record.append(act.clone())
        prev = st.clone()
        if timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        env.step_device(act.data_ptr(), obs.data_ptr(), flags.data_ptr())
        if timing is not None:
            e1.record()
            timing.append((e0, e1))
        env.write_rl_state(st.data_ptr())
        ok = alive & ((flags & 2) != 0) & ((flags & 4) == 0)
        r = task.reward(prev, st, arrival, task.q0)
        s2 = task.state(obs)
        env_steps += alive.to(torch.int64)
        if learner.mode == "train":
            stored += learner.memory.add_device(s, a, s2, r, ok)
            # the reference's agents stop training with their episode: no update on stale replay
            # once every env is done; decided on the device (a masked no-op), no host read
            if step_counter % train_every == 0:
                live = alive.any()
                for _ in range(updates_per_train):
                    learner.learn(live=live)
        rewards.append(torch.where(ok, r, torch.zeros_like(r)))
        actions.append(a)
        step_counter += 1
        alive = ok & ((flags & 1) == 0)
    rw = torch.stack(rewards) if rewards else None
    return {"rewards": rw, "actions": torch.stack(actions) if actions else None,
            "returns": rw.sum(0) if rw is not None else torch.zeros(n, dtype=torch.float64, device=dev),
            "flags": flags, "arrival": arrival, "stored": stored, "env_steps": env_steps,
            "steps": step_counter + 1}
