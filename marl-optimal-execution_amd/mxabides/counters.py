"""Algorithmic HBM bytes of the market step, counted per event class.

The device counts, in instrumented runs (parity hash on), every pop by message kind, the busy
requeues, the events pushed, the RNG words drawn, the agent-record round trips and the pops
handled inside batched event runs (include/mxa.h mxa_read_counters).  The algorithmic bytes are
what those events must move in the structure-of-arrays design, with the per-unit sizes of
SURVEY.md §8(d):

* 48 B per pop (the event record read) and per push (the event written), 48 B more per busy
  requeue (Kernel.py:224-230 re-inserts the event);
* 2 x 64 B per agent-record round trip (the record read and written back): counted where an
  event really needs the recipient's state, not per pop (the exchange reads nothing of its own
  record but a zero computation delay, an acknowledgement only sets agentCurrentTimes, and a
  batched run of acknowledgements loads its agent once);
* 8 B per RNG word drawn (the 4-byte MT19937 output plus its amortised twist rewrite);
* 2 x (16 B level header + 32 B order slot) per book touch: every LIMIT / CANCEL / MODIFY order
  the exchange handles touches one level, and every fill one more resting order (a fill sends
  two ORDER_EXECUTED messages, OrderBook.py:88-91).

SURVEY.md §8(d) also lists 16 B x log2(Q) of binary-heap sift per queue operation; this design
has no heap (each pop is a wave-min over per-lane slot minima in LDS), so that term is reported
separately (`heap_sift_model`) and not part of the count.

The per-event figure is the total over every env divided by the total pops.  It is a property
of the workload (the same seeds give the same counts), so bench.py counts one batch of the timed
workload with the instrumentation on and applies the figure to the timed, uninstrumented run.
"""
import numpy as np

K_LIMIT, K_CANCEL, K_MODIFY, K_EXECUTED = 11, 12, 13, 15  # mxa_layout.h MK_*
C_REQUEUE, C_PUSH, C_RNG, C_POPS, C_MAXQ, C_MAXBOOK, C_REC, C_RUN = 25, 26, 27, 28, 29, 30, 31, 32

EVENT_BYTES = 48
RECORD_BYTES = 64
RNG_WORD_BYTES = 8
BOOK_TOUCH_BYTES = 2 * (16 + 32)
SIFT_BYTES = 16


def algorithmic_bytes(c):
    """c: [n_envs][COUNTER_WORDS] counters -> (total bytes, total pops, breakdown dict)"""
    c = np.asarray(c, dtype=np.int64)
    pops, push, req, rng = c[:, C_POPS], c[:, C_PUSH], c[:, C_REQUEUE], c[:, C_RNG]
    book = c[:, K_LIMIT] + c[:, K_CANCEL] + c[:, K_MODIFY] + c[:, K_EXECUTED] // 2
    parts = {
        "events": int((EVENT_BYTES * (pops + push + req)).sum()),
        "agent_records": int((2 * RECORD_BYTES * c[:, C_REC]).sum()),
        "rng": int((RNG_WORD_BYTES * rng).sum()),
        "book": int((BOOK_TOUCH_BYTES * book).sum()),
    }
    return sum(parts.values()), int(pops.sum()), parts


def bytes_per_event(c):
    """(bytes per event, breakdown per event, per-event unit counts) of a counter block"""
    total, pops, parts = algorithmic_bytes(c)
    c = np.asarray(c, dtype=np.int64)
    n = max(1, pops)
    per = {k: v / n for k, v in parts.items()}
    sift = np.ceil(np.log2(np.maximum(2, c[:, C_MAXQ]))).astype(np.int64)
    units = {"pushes": float(c[:, C_PUSH].sum()) / n, "rng_words": float(c[:, C_RNG].sum()) / n,
             "requeues": float(c[:, C_REQUEUE].sum()) / n, "fills": float((c[:, K_EXECUTED] // 2).sum()) / n,
             "record_round_trips": float(c[:, C_REC].sum()) / n, "run_members": float(c[:, C_RUN].sum()) / n,
             "heap_sift_model": float((SIFT_BYTES * sift * (c[:, C_POPS] + c[:, C_PUSH])).sum()) / n}
    return total / n, per, units


def strict_bytes_per_event(c):
    """SURVEY.md §8(d) read literally: the 2 x 64 B agent-record round trip charged on EVERY pop
    (not only where an event loads the recipient's state), the other terms as counted.  Reported
    beside the counted figure (bytes_per_event), which is the conservative one."""
    total, pops, parts = algorithmic_bytes(c)
    c = np.asarray(c, dtype=np.int64)
    n = max(1, pops)
    strict = total - parts["agent_records"] + 2 * RECORD_BYTES * int(c[:, C_POPS].sum())
    return strict / n
