"""Algorithmic HBM bytes of the market step, counted per event class.

The device counts, in instrumented runs (parity hash on), every pop by message kind, the busy
requeues, the events pushed and the RNG words drawn (include/mxa.h mxa_read_counters).  The
algorithmic bytes are the bytes those events must move in a structure-of-arrays design, with the
per-unit sizes of SURVEY.md §8(d):

* 48 B per pop (the event record read) and per push (the event written), 48 B more per busy
  requeue (Kernel.py:224-230 re-inserts the event);
* 2 x 64 B per pop: the recipient's agent record, read and written back;
* 8 B per RNG word drawn (the 4-byte MT19937 output plus its amortised twist rewrite);
* 2 x (16 B level header + 32 B order slot) per book touch: every LIMIT / CANCEL / MODIFY order
  the exchange handles touches one level, and every fill one more resting order (a fill sends
  two ORDER_EXECUTED messages, OrderBook.py:88-91);
* 16 B x log2(max pending events) per pop and per push: the sift of a binary heap over the
  event queue (queue.PriorityQueue, Kernel.py:24, 192).

The per-event figure is the total over every env divided by the total pops.  It is a property
of the workload (the same seeds give the same counts), so bench.py counts one batch of the timed
workload with the instrumentation on and applies the figure to the timed, uninstrumented run.
"""
import numpy as np

K_LIMIT, K_CANCEL, K_MODIFY, K_EXECUTED = 11, 12, 13, 15  # mxa_layout.h MK_*
C_REQUEUE, C_PUSH, C_RNG, C_POPS, C_MAXQ = 25, 26, 27, 28, 29

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
    sift = np.ceil(np.log2(np.maximum(2, c[:, C_MAXQ]))).astype(np.int64)
    parts = {
        "events": int((EVENT_BYTES * (pops + push + req)).sum()),
        "agent_records": int((2 * RECORD_BYTES * pops).sum()),
        "rng": int((RNG_WORD_BYTES * rng).sum()),
        "book": int((BOOK_TOUCH_BYTES * book).sum()),
        "heap_sift": int((SIFT_BYTES * sift * (pops + push)).sum()),
    }
    return sum(parts.values()), int(pops.sum()), parts


def bytes_per_event(c):
    """(bytes per event, breakdown per event, per-event unit counts) of a counter block"""
    total, pops, parts = algorithmic_bytes(c)
    c = np.asarray(c, dtype=np.int64)
    per = {k: v / max(1, pops) for k, v in parts.items()}
    units = {"pushes": float(c[:, C_PUSH].sum()) / max(1, pops), "rng_words": float(c[:, C_RNG].sum()) / max(1, pops),
             "requeues": float(c[:, C_REQUEUE].sum()) / max(1, pops),
             "fills": float((c[:, K_EXECUTED] // 2).sum()) / max(1, pops)}
    return total / max(1, pops), per, units
