"""Helpers to read the committed reference fixtures (tests/golden/)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = [("sparse_zi_100", 123456789), ("rmsc03", 123456789), ("rmsc03", 1008), ("rmsc03", 7),
            ("sparse_zi_1000", 123456789), ("value_noise", 123456789), ("value_noise", 7),
            ("rmsc02", 7), ("rmsc02", 123456789), ("rmsc01", 7), ("rmsc01", 99),
            ("obi_rmsc02", 7), ("obi_rmsc02", 123456789), ("obi_rmsc02", 30), ("obi_rmsc02", 107),
            ("random_fund_value", 7), ("random_fund_value", 123456789),
            ("random_fund_diverse", 7), ("random_fund_diverse", 123456789),
            ("hist_fund_value", 7), ("hist_fund_value", 123456789),
            ("hist_fund_diverse", 7), ("hist_fund_diverse", 123456789),
            ("rmsc03_sbmm", 123456789), ("rmsc03_sbmm", 7), ("rmsc03_sbmm_poll", 123456789), ("rmsc03_sbmm_poll", 7)]
HIST_CONFIGS = ("hist_fund_value", "hist_fund_diverse")
FUND = os.path.join(GOLDEN, "fund_JPM_20190628.npz")  # gen_fixtures.py fund_series()


def market_kw(cfg):
    """VecMarket keyword arguments a configuration needs: the ExternalFileOracle series of the
    hist_fund_* fixtures"""
    if cfg in HIST_CONFIGS:
        from mxabides.fundamental import FundamentalSeries
        return {"fundamental": FundamentalSeries.load(FUND)}
    return {}


def load(cfg, seed):
    with open(os.path.join(GOLDEN, "%s_%d.json" % (cfg, seed))) as f:
        d = json.load(f)
    tr = np.load(os.path.join(GOLDEN, "%s_%d.npz" % (cfg, seed)))["trace"]
    return d, tr


def first_mismatch(a, b):
    n = min(len(a), len(b))
    bad = np.nonzero((a[:n] != b[:n]).any(1))[0]
    return int(bad[0]) if len(bad) else (-1 if len(a) == len(b) else n)


def kat_lines():
    lines = open(os.path.join(GOLDEN, "sparse_zi_1000_kat.txt")).read().splitlines()
    holdings = [l.strip() for l in lines if l.startswith("Final holdings")]
    means, take = [], False
    for l in lines:
        if l.startswith("Mean ending value"):
            take = True
            continue
        if take:
            if not l.startswith("\t"):
                break
            means.append(l.strip())
    return holdings, means


# Kernel.runner with a caller's stopTime (gen_fixtures.py "CFG@HH:MM:SS"): (config, seed, stop
# as ns since midnight, fixture name)
NS_S = 1_000_000_000
STOP_FIXTURES = [("rmsc03", 123456789, 11 * 3600 * NS_S, "rmsc03_stop110000_123456789"),
                 ("value_noise", 7, (10 * 3600 + 15 * 60) * NS_S, "value_noise_stop101500_7"),
                 ("sparse_zi_100", 123456789, (9 * 3600 + 45 * 60 + 30) * NS_S, "sparse_zi_100_stop094530_123456789")]


def load_named(name):
    """(fixture dict, trace, summary rows) of tests/golden/<name>.*"""
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, name + "_summary.json")) as f:
        summ = json.load(f)
    tr = np.load(os.path.join(GOLDEN, name + ".npz"))["trace"]
    return d, tr, summ


FNV_OFF, FNV_PRIME, M64 = 0xCBF29CE484222325, 0x100000001B3, (1 << 64) - 1


def fnv_words(h, words):
    """gen_fixtures.fnv_words: FNV-1a-64 over int64 words"""
    for w in words:
        h = ((h ^ (int(w) & M64)) * FNV_PRIME) & M64
    return h


def book_row_digests(flat):
    """per book_log row: FNV-1a-64 over (t, n, price, volume, ...) without the executed-quantity
    words, the digest gen_fixtures.save_booklog stores for every row"""
    from mxabides import booklog as bl
    return [fnv_words(FNV_OFF, [t, len(p)] + np.stack([p, v], axis=1).ravel().tolist())
            for t, _, _, p, v in bl.iter_rows(flat)]


def event_digest(events):
    """gen_fixtures.save_booklog's digest of the exchange's BEST_BID / BEST_ASK / LAST_TRADE rows
    (time, kind 0/1/2, Event bytes)"""
    kinds = {"BEST_BID": 0, "BEST_ASK": 1, "LAST_TRADE": 2}
    h = FNV_OFF
    for t, k, s in events:
        h = fnv_words(h, [t, kinds[k]] + list(s.encode()))
    return h


# ExchangeAgent.log rows (gen_fixtures.py save_exlog, mxabides.booklog.exchange_log): the words
# of one row's digest -- time, Event kind (0 int, 1 str, 2 order dict), the EventType's bytes
# (length-prefixed), then the int, the string's bytes, or the order's seven fields
def exlog_row_words(t, etype, ekind, eint, estr, order):
    b = etype.encode()
    w = [t, ekind, len(b)] + list(b)
    if ekind == 0:
        return w + [eint]
    if ekind == 1:
        s = estr.encode()
        return w + [len(s)] + list(s)
    return w + list(order)


def exlog_row_tuple(row):
    """one mxabides.booklog.exchange_log row as the fixture's (t, EventType, kind, int, str, order)"""
    t, et, ev = row
    t = -1 if t is None else int(t)
    if isinstance(ev, dict):
        f = ev["fill_price"]
        return (t, et, 2, 0, "", (int(ev["agent_id"]), int(ev["time_placed"]), int(ev["quantity"]),
                                  int(ev["is_buy_order"]), int(ev["order_id"]), -(1 << 63) if f is None else int(f),
                                  int(ev["limit_price"])))
    if isinstance(ev, str):
        return (t, et, 1, 0, ev, (0,) * 7)
    return (t, et, 0, int(ev), "", (0,) * 7)


def exlog_fixture(name):
    """tests/golden/<name>_exlog.npz (gen_fixtures.py exlog): (row count, digest, verbatim rows as
    exlog_row_tuple tuples, the npz)"""
    z = np.load(os.path.join(GOLDEN, "%s_exlog.npz" % name))
    types = [str(x) for x in z["types"]]
    rows = [(int(t), types[int(k)], int(ek), int(ei), str(es), tuple(int(x) for x in o))
            for t, k, ek, ei, es, o in zip(z["t"], z["type_idx"], z["ekind"], z["eint"], z["estr"], z["order"])]
    return int(z["n_rows"]), int(z["digest"]), rows, z


def exlog_digest(rows):
    """FNV-1a-64 over every row's exlog_row_words (the fixture's digest)"""
    h = 0xCBF29CE484222325
    for row in rows:
        for w in exlog_row_words(*exlog_row_tuple(row)):
            h = ((h ^ (int(w) & 0xFFFFFFFFFFFFFFFF)) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


# runtime compositions (tests/golden/gen_config_fixtures.py): (name, seed) of cfg_<name>_<seed>.*
COMPOSITION_FIXTURES = [("rmsc03_n100_v20", 123456789), ("rmsc03_n100_v20", 7), ("rmsc03_alt", 123456789),
                        ("rmsc03_alt", 11), ("sparse_zi_alt", 123456789), ("sparse_zi_alt", 7),
                        ("sparse_zi_matrix_200", 123456789), ("value_noise_alt", 123456789), ("value_noise_alt", 7)]


def load_composition(name, seed):
    """(fixture dict with its "composition" fields, trace, summary rows) of cfg_<name>_<seed>"""
    return load_named("cfg_%s_%d" % (name, seed))


def composition_names():
    return sorted({n for n, _ in COMPOSITION_FIXTURES})
