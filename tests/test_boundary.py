"""C-ABI argument validation (include/mxa.h): every entry point rejects bad arguments with
MXA_EINVAL before it touches a device, so these run without a GPU.  The tape rules restate
the reference's LOBSTEROrdersProcessor/Order invariants the device path relies on."""
import ctypes

import numpy as np
import pytest

from mxabides import _lib, tape

EINVAL = -1


@pytest.fixture(scope="module")
def L():
    return _lib.load()


def _replay(L, t, oid, price, size, buy, n_envs=1):
    h = ctypes.c_void_p()
    arr = [np.ascontiguousarray(x, dtype=np.int64) for x in (t, oid, price, size)]
    b = np.ascontiguousarray(buy, dtype=np.int8)
    rc = L.mxa_create_replay(arr[0].ctypes.data, arr[1].ctypes.data, arr[2].ctypes.data, arr[3].ctypes.data,
                             b.ctypes.data, len(arr[0]), n_envs, 0, 0, ctypes.byref(h))
    return rc


def test_create_rejects_bad_arguments(L):
    h = ctypes.c_void_p()
    seeds = np.arange(4, dtype=np.uint32)
    assert L.mxa_create(_lib.MXA_RMSC03, 0, seeds.ctypes.data, 0, 0, ctypes.byref(h)) == EINVAL
    assert L.mxa_create(_lib.MXA_RMSC03, 4, None, 0, 0, ctypes.byref(h)) == EINVAL
    assert L.mxa_create(_lib.MXA_RMSC03, 4, seeds.ctypes.data, 0, -1, ctypes.byref(h)) == EINVAL
    assert L.mxa_create(_lib.MXA_RMSC03, 4, seeds.ctypes.data, 0, 0, None) == EINVAL
    assert L.mxa_create(99, 4, seeds.ctypes.data, 0, 0, ctypes.byref(h)) == EINVAL
    # the replay composition is built by mxa_create_replay, not by a config id
    assert L.mxa_create(_lib.MXA_MARKETREPLAY, 4, seeds.ctypes.data, 0, 0, ctypes.byref(h)) == EINVAL
    assert not h


def test_null_handle_calls_are_rejected(L):
    assert L.mxa_reset(None, None) == EINVAL
    assert L.mxa_launch(None, 10) == EINVAL
    assert L.mxa_run(None, 10, 0, None) == EINVAL
    assert L.mxa_step(None, None, None, None) == EINVAL
    assert L.mxa_n_agents(None) == 0


def test_replay_rejects_malformed_tapes(L):
    t = np.array([10, 20, 30]) * 10 ** 9 + 34200 * 10 ** 9
    ok = dict(oid=[100000, 100001, 100000], price=[5000, 5001, 5000], size=[100, 50, 0], buy=[1, 0, 1])
    assert _replay(L, t[::-1], **ok) == EINVAL                                  # not time-sorted
    assert _replay(L, t, **dict(ok, oid=[100000, -5, 100000])) == EINVAL        # negative id
    assert _replay(L, t, **dict(ok, size=[100, -1, 0])) == EINVAL               # negative size
    assert _replay(L, t, **dict(ok, price=[5000, 1 << 21, 5000])) == EINVAL     # beyond the price ladder
    # auto ids (DummyRL's and ORDER_ID 0 records') could reach an explicit tape id: the
    # reference's Order._order_ids skip rule would then apply, so the tape is refused
    assert _replay(L, t, **dict(ok, oid=[0, 4000, 4000])) == EINVAL
    assert _replay(L, t[:0], **{k: v[:0] for k, v in ok.items()}) == EINVAL    # empty tape
    assert _replay(L, t, n_envs=0, **ok) == EINVAL


def test_tape_container_validation():
    with pytest.raises(ValueError):
        tape.Tape([], [], [], [], [])
    with pytest.raises(ValueError):
        tape.Tape([2, 1], [1, 2], [5, 5], [1, 1], [1, 0])
    with pytest.raises(ValueError):
        tape.Tape([1, 2], [1, -2], [5, 5], [1, 1], [1, 0])
    t = tape.Tape([1, 2, 3], [0, 7, 0], [5, 5, 6], [1, 1, 2], [1, 0, 1])
    assert t.n_auto == 2 and len(t) == 3


def test_mm_params_abi_layout_and_defaults():
    """mxa_mm_params (include/mxa.h): the host record, the oracle's ora_mm_params and the library's
    mxa_mm_defaults() (config/rmsc03.py:39-43 defaults) agree; no GPU call"""
    import ctypes

    import numpy as np

    import pyoracle
    from mxabides import configs
    assert configs.MM_PARAMS_DTYPE.itemsize == 32 and configs.MM_PARAMS_DTYPE == pyoracle.MM_DTYPE
    p = configs.mm_params(3, pov=[0.05, 0.1, 0.2], num_ticks=50, wake_up_freq=["10S", "1min", 5 * 10 ** 9])
    assert p["mm_wake_up_freq_ns"].tolist() == [10 ** 10, 6 * 10 ** 10, 5 * 10 ** 9]
    assert p["mm_num_ticks"].tolist() == [50] * 3 and p["mm_min_order_size"].tolist() == [20] * 3
    import mxabides
    L = mxabides.load()

    class MM(ctypes.Structure):
        _fields_ = [(n, {"<f8": ctypes.c_double, "<i4": ctypes.c_int32, "<i8": ctypes.c_int64}[configs.MM_PARAMS_DTYPE[n].str])
                    for n in configs.MM_PARAMS_DTYPE.names]
    L.mxa_mm_defaults.restype = MM
    d = L.mxa_mm_defaults()
    ref = configs.mm_params(1)[0]
    assert (d.mm_pov, d.mm_min_order_size, d.mm_window_size, d.mm_num_ticks, d.mm_wake_up_freq_ns) == \
        (ref["mm_pov"], ref["mm_min_order_size"], ref["mm_window_size"], ref["mm_num_ticks"], ref["mm_wake_up_freq_ns"])
    assert (configs.mm_params(1)[["mm_pov", "mm_min_order_size", "mm_window_size", "mm_num_ticks"]].tolist()[0] ==
            (0.05, 20, 5, 20))
