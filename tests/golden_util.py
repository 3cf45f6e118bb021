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
