"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): a float64 numpy restatement
of the reference DDQN learner's arithmetic, for the parity tests of mxabides.ddqn.

Follows agent/execution/qlearning/ddqlearning_execution_agent.py and util/model/QNets.py; the
Keras 2 (TensorFlow 2.1, requirements.txt:17) pieces are restated from their published
algorithm because TensorFlow is not installed here: Dense = x @ W + b with W
[in, out]; `mse` = mean over all elements; RMSprop optimizer_v2 with momentum 0, not centered:
rms = rho*rms + (1-rho)*g^2, w -= lr * g / (sqrt(rms) + eps). Parity with Keras itself is
therefore unpinned; what is pinned is the reference's own algorithm around it (the target of
train_neural_nets, the action table, the state discretization)."""
import numpy as np


def action_table(size_allocation, size_scale):
    """ddqlearning_execution_agent.py:27-37"""
    alloc = list(size_allocation.keys())
    alloc.append(0)
    alloc.sort()
    acts, k = {}, 0
    for i in range(len(alloc)):
        for j in range(len(size_scale)):
            acts[k] = (alloc[i], size_scale[j])
            k += 1
    return acts


def forward(layers, x, masks=None, rate=0.1):
    """layers: [(W [in,out], b)], ReLU on all but the last (QNets.py:19-27).  masks: the keep
    masks of the Dropout(rate) layers after hidden layers 2..n in training mode (QNets.py:22-26;
    Keras scales kept units by 1 / (1 - rate)); None = predict(), no dropout."""
    acts = [x]
    for i, (W, b) in enumerate(layers):
        z = acts[-1] @ W + b
        if i == len(layers) - 1:
            acts.append(z)
            continue
        h = np.maximum(z, 0.0)
        if masks is not None and i >= 1:
            h = h * masks[i - 1] / (1.0 - rate)
        acts.append(h)
    return acts


def q_target(eval_layers, target_layers, s, a, s2, r, gamma):
    """train_neural_nets, ddqlearning_execution_agent.py:475-490"""
    q_next = forward(target_layers, s2)[-1]
    q_eval4next = forward(target_layers, s2)[-1]
    q_eval = forward(eval_layers, s)[-1]
    tgt = q_eval.copy()
    bi = np.arange(len(s))
    tgt[bi, a.astype(int)] = r + gamma * q_next[bi, np.argmax(q_eval4next, axis=1)]
    return tgt


def mse_grads(layers, x, tgt, masks=None, rate=0.1):
    """loss = mean((f(x) - tgt)^2) and d loss / d (W, b) for every layer (train_on_batch: the
    dropout masks of training mode, if given)."""
    acts = forward(layers, x, masks, rate)
    out = acts[-1]
    loss = np.mean((out - tgt) ** 2)
    d = 2.0 * (out - tgt) / out.size
    grads = [None] * len(layers)
    for i in range(len(layers) - 1, -1, -1):
        W, _ = layers[i]
        grads[i] = (acts[i].T @ d, d.sum(0))
        if i:
            # acts[i] = relu(z) (* mask / (1 - rate) after a dropout layer): > 0 exactly where
            # both the ReLU and the mask pass
            scale = 1.0 / (1.0 - rate) if (masks is not None and i - 1 >= 1) else 1.0
            d = (d @ W.T) * (acts[i] > 0) * scale
    return loss, grads


def rmsprop_step(layers, grads, rms, lr, rho=0.9, eps=1e-7):
    """Keras optimizer_v2 RMSprop, momentum 0, not centered (TF 2.1 rmsprop.py)."""
    new, new_rms = [], []
    for (W, b), (gW, gb), (rW, rb) in zip(layers, grads, rms):
        rW = rho * rW + (1 - rho) * gW * gW
        rb = rho * rb + (1 - rho) * gb * gb
        new.append((W - lr * gW / (np.sqrt(rW) + eps), b - lr * gb / (np.sqrt(rb) + eps)))
        new_rms.append((rW, rb))
    return new, new_rms


def step_reward(fills, arrival, q0):
    """compute_reward summed over fills [(qty, fill_price)] for a BUY (ddqlearning_execution_agent.py:425-432)"""
    return sum((1 - ((f - arrival) / arrival)) * q / q0 * 10000 for q, f in fills)


def train_step(eval_layers, target_layers, rms, counter, batch, lr=0.01, gamma=0.98, replace_target_iter=5, masks=None,
               rate=0.1):
    """One whole `train_neural_nets` update (ddqlearning_execution_agent.py:448-515) after the
    batch is sampled, in the reference's order:
      1. q_next, q_eval4next from the target net AS IT STANDS, q_eval from eval (:486-505);
      2. then, if learn_step_counter % replace_target_iter == 0, eval -> target (:508-510);
      3. then train_on_batch on the eval net (:513): MSE, one RMSprop step;
      4. epsilon, then learn_step_counter += 1 (:526-530).
    batch = (s, a, s2, r); masks: train_on_batch's dropout keep masks (None: dropout off).
    Returns (eval', target', rms', counter', loss)."""
    s, a, s2, r = batch
    tgt = q_target(eval_layers, target_layers, s, a, s2, r, gamma)
    if counter % replace_target_iter == 0:
        target_layers = [(W.copy(), b.copy()) for W, b in eval_layers]
    loss, grads = mse_grads(eval_layers, s, tgt, masks, rate)
    eval_layers, rms = rmsprop_step(eval_layers, grads, rms, lr)
    return eval_layers, target_layers, rms, counter + 1, loss
