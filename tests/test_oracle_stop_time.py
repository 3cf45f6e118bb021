"""Kernel.runner(startTime, stopTime) with a caller's stopTime (Kernel.py:50-64, 190-196): the loop
stops at its first pop past stopTime, after handling that event.  The C oracle (ora_set_stop)
against reference runs of the config scripts with kernelStopTime replaced
(tests/golden/gen_fixtures.py "CFG@HH:MM:SS")."""
import pytest

import pyoracle
from golden_util import STOP_FIXTURES, first_mismatch, load_named


@pytest.mark.parametrize("cfg,seed,stop,name", STOP_FIXTURES)
def test_oracle_stop_time_matches_reference(cfg, seed, stop, name):
    d, ref, summ = load_named(name)
    e = pyoracle.OracleEnv(cfg, seed, trace_cap=len(ref) + 1)
    e.set_stop(stop)
    e.run()
    assert e.error[0] == 0
    assert first_mismatch(e.trace(), ref) == -1
    assert e.events == d["events"] and "%016x" % e.hash == d["hash"]
    assert ref[-2][0] <= stop < ref[-1][0] and d["final_time"] == ref[-1][0]  # one pop past stopTime
    assert e.book(0) == d["bids"] and e.book(1) == d["asks"]
    e.finish()
    rep = e.report()
    assert [l for l in rep if l.startswith("Final holdings")] == d["final_holdings_lines"]
    assert [l for l in rep if not l.startswith("Final holdings")] == d["mean_lines"]
    got = e.summary_log()
    assert got == summ and all(type(a["Event"]) is type(b["Event"]) for a, b in zip(got, summ))
