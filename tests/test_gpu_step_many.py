"""k ABIDESEnv.step calls in one launch (include/mxa.h mxa_step_many, bench.py's GymKernel lines):
step i of every env equals the i-th of k one-step launches (mxa_step_device) — observation bits,
flags, events and the per-pop parity hash — on the IBM replay and on rmsc03 + DummyRL, including
envs that end (done, or the reference's ValueError) inside the launch, and a launch that picks
up where one-step launches left off."""
import os

import numpy as np
import pytest
import torch

from mxabides import tape
from mxabides.gym import ACTION_SIZE, OBS_SIZE, VecABIDESEnv

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _actions(k, n, seed, scale):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = torch.rand((k, n, ACTION_SIZE), generator=g, dtype=torch.float64, device="cuda")
    a[:, :, 0] *= scale
    return a


def _one_by_one(v, act, k0, k1, obs, flags):
    for i in range(k0, k1):
        v.step_device(act[i].data_ptr(), obs[i].data_ptr(), flags[i].data_ptr())


def _make(kind, n):
    if kind == "replay":
        return VecABIDESEnv(tape.Tape.load(os.path.join(GOLD, "tape_IBM_2003-01-14.npz")), n)
    return VecABIDESEnv(seeds=(123456789 + np.arange(n)) & 0xFFFFFFFF)


@pytest.mark.parametrize("kind,n,k,scale", [("replay", 16, 120, 0.01), ("rmsc03_rl", 64, 27, 0.05)])
def test_gpu_step_many_equals_one_step_launches(kind, n, k, scale):
    act = _actions(k, n, 5, scale)
    obs_a = torch.zeros((k, n, OBS_SIZE), dtype=torch.float64, device="cuda")
    flg_a = torch.zeros((k, n), dtype=torch.int32, device="cuda")
    obs_b, flg_b = torch.zeros_like(obs_a), torch.zeros_like(flg_a)
    a, b = _make(kind, n), _make(kind, n)
    for v in (a, b):
        v.set_parity_hash(True)
        v.reset()
    torch.cuda.synchronize()  # the handles run on streams of their own
    _one_by_one(a, act, 0, k, obs_a, flg_a)
    b.step_many_device(k, act.data_ptr(), obs_b.data_ptr(), flg_b.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(flg_a, flg_b)
    assert torch.equal(obs_a.view(torch.int64), obs_b.view(torch.int64))  # bit for bit
    sa, sb = a.summary(), b.summary()
    for key in ("events", "hash", "status", "err", "current_time"):
        assert (sa[key] == sb[key]).all(), key
    if kind == "rmsc03_rl":  # some envs end inside the launch (done or the reference's ValueError)
        assert (flg_b[-1] & 1).any()


def test_gpu_step_many_continues_one_step_launches():
    n, k0, k1 = 16, 7, 40
    act = _actions(k1, n, 9, 0.01)
    obs_a = torch.zeros((k1, n, OBS_SIZE), dtype=torch.float64, device="cuda")
    flg_a = torch.zeros((k1, n), dtype=torch.int32, device="cuda")
    obs_b, flg_b = torch.zeros_like(obs_a), torch.zeros_like(flg_a)
    a, b = _make("replay", n), _make("replay", n)
    for v in (a, b):
        v.set_parity_hash(True)
        v.reset()
    torch.cuda.synchronize()
    _one_by_one(a, act, 0, k1, obs_a, flg_a)
    _one_by_one(b, act, 0, k0, obs_b, flg_b)
    b.step_many_device(k1 - k0, act[k0:].data_ptr(), obs_b[k0:].data_ptr(), flg_b[k0:].data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(flg_a, flg_b)
    assert torch.equal(obs_a.view(torch.int64), obs_b.view(torch.int64))
    assert (a.summary()["hash"] == b.summary()["hash"]).all()
