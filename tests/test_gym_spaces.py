"""ABIDESEnv.action_space / observation_space are Box-like (ABIDESEnv.py:22-26): a learner's
.shape, .low/.high, .sample() and .contains() work without gym installed."""
import numpy as np

from mxabides.gym import ACTION_SIZE, Box


def test_box_surface():
    a = Box([0.0] * ACTION_SIZE, [1.0] * ACTION_SIZE)
    assert a.shape == (ACTION_SIZE,) and a.dtype == np.float32
    a.seed(3)
    x = a.sample()
    assert x.shape == a.shape and x.dtype == np.float32 and a.contains(x) and x in a
    assert not a.contains(np.full(ACTION_SIZE, 2.0)) and not a.contains(np.zeros(ACTION_SIZE + 1))
    a.seed(3)
    assert (a.sample() == x).all()
    o = Box([0] * 10, [0] * 10)  # the reference declares a degenerate observation box
    assert o.shape == (10,) and (o.sample() == 0).all()
