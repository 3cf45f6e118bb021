"""The C oracle's config/rmsc03.py with market-maker options (ora_create_mm) against reference runs
of the script with scripts/rmsc03.sh's options on its seeds 30-35 (tests/golden/
rmsc03_mm_0.05_25_5_50_10S_*): every trace record kept, the whole-run hash, books, holdings."""
import numpy as np
import pytest

import pyoracle
from golden_util import first_mismatch, load_named


@pytest.mark.parametrize("seed", range(30, 36))
def test_oracle_mm_options_match_reference(seed):
    d, ref, summ = load_named("rmsc03_mm_0.05_25_5_50_10S_%d" % seed)
    mm = np.zeros(1, dtype=pyoracle.MM_DTYPE)
    mm["mm_pov"], mm["mm_min_order_size"], mm["mm_window_size"] = 0.05, 25, 5
    mm["mm_num_ticks"], mm["mm_wake_up_freq_ns"] = 50, 10 ** 10
    o = pyoracle.OracleEnv("rmsc03", seed, trace_cap=len(ref), mm=mm[0])
    o.run()
    assert o.error[0] == 0
    assert first_mismatch(o.trace(), ref) == -1
    assert o.events == d["events"] and "%016x" % o.hash == d["hash"]
    assert o.book(0) == d["bids"] and o.book(1) == d["asks"]


def test_oracle_default_options_equal_rmsc03():
    seeds = np.arange(100, 132, dtype=np.uint32)
    mm = np.zeros(len(seeds), dtype=pyoracle.MM_DTYPE)
    mm["mm_pov"], mm["mm_min_order_size"], mm["mm_window_size"], mm["mm_num_ticks"] = 0.05, 20, 5, 20
    mm["mm_wake_up_freq_ns"] = 10 ** 9
    ev, hs, er, _ = pyoracle.run_batch_mm(seeds, mm, 4)
    ev0, hs0, _ = pyoracle.run_batch("rmsc03", seeds, 4)
    assert (ev == ev0).all() and (hs == hs0).all() and (er == 0).all()
