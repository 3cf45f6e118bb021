#!/usr/bin/env python3
"""Golden-fixture generator: runs the *reference* ABIDES (read-only, /root/reference)
in this build container and records what the product must reproduce.

CONTAINER-ONLY TEST INFRASTRUCTURE.  Nothing under tests/, bench.py or the product
imports this module; it is committed so the fixtures under tests/golden/ can be
regenerated.  /root/reference does not exist on the GPU box.

What is recorded per (config, seed):
  * the kernel event trace: one int64 record per priority-queue pop
      [t_ns_since_midnight, recipient, msg_type, kind, f0, f1, f2, f3, f4, f5]
    (field meaning per kind: see KIND_* below and DESIGN.md §"Trace records")
    The record is the parity unit of the whole project: the same record is produced
    by the C oracle (oracle/) and by the HIP kernels (trace ring / rolling hash).
  * a word-wise FNV-1a rolling hash over those records (checkpoint every 1000 pops),
  * the final state: per-agent holdings + cash + open orders, the exchange book
    (levels, FIFO order ids/qty), global order-id counter, message count, stdout
    "Final holdings ..." and "Mean ending value" lines.

Third-party modules the reference imports but this image lacks are replaced by
logging-only stubs: `jsons.dump` (used only to log orders),
pandas 2 API renames (`pandas.io.json.json_normalize`, `SparseDataFrame`, `Timedelta.delta` =
the ns count of the pinned pandas 0.24, read by ExchangeAgent.publishOrderBookData), and the
bz2 log writers are no-ops.  None of them touches the simulated arithmetic.

Usage:  python tests/golden/gen_fixtures.py all          (writes tests/golden/*.npz/json)
        python tests/golden/gen_fixtures.py summaries    (only the *_summary.json summary logs)
        python tests/golden/gen_fixtures.py booklog      (*_booklog.npz: book snapshot outputs)
        python tests/golden/gen_fixtures.py exlog        (*_exlog.npz: the exchange's agent log)
        python tests/golden/gen_fixtures.py run CFG SEED OUT [--full] [--booklog]
"""
import importlib
import io
import json
import os
import subprocess
import sys
import tempfile
import types
import zlib

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

# ---- message kinds (shared with oracle/abides_oracle.h and csrc/mxa_trace.h) ----
KIND = {
    "WAKEUP": 0,
    "WHEN_MKT_OPEN_REQ": 1, "WHEN_MKT_CLOSE_REQ": 2,
    "WHEN_MKT_OPEN": 3, "WHEN_MKT_CLOSE": 4,
    "QUERY_SPREAD_REQ": 5, "QUERY_SPREAD": 6,
    "QUERY_LAST_TRADE_REQ": 7, "QUERY_LAST_TRADE": 8,
    "QUERY_TRANSACTED_VOLUME_REQ": 9, "QUERY_TRANSACTED_VOLUME": 10,
    "LIMIT_ORDER": 11, "CANCEL_ORDER": 12, "MODIFY_ORDER": 13,
    "ORDER_ACCEPTED": 14, "ORDER_EXECUTED": 15, "ORDER_CANCELLED": 16,
    "MKT_CLOSED": 17, "ORDER_MODIFIED": 18, "KERNEL_CANCEL_ORDER": 19,
    "MARKET_DATA": 20,
    "QUERY_ORDER_STREAM_REQ": 21, "QUERY_ORDER_STREAM": 22,
    "MARKET_DATA_SUBSCRIPTION_REQUEST": 23, "MARKET_DATA_SUBSCRIPTION_CANCELLATION": 24,
}

FNV_OFF = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
M64 = (1 << 64) - 1


def fnv_words(h, words):
    for w in words:
        h = ((h ^ (int(w) & M64)) * FNV_PRIME) & M64
    return h


def _price(p):
    """Integer cents (the simulated configs); marketreplay dollars -> 1e-4 units."""
    if p is None:
        return -1
    if isinstance(p, (float, np.floating)):
        return int(round(p * 10000))
    return int(p)


SB_ID_BASE = 0x40000000  # SpreadBasedMarketMakerAgent's string ids "<name>_<id>_<n>" -> SB_ID_BASE + n


def _oid(x):
    """order id as the device carries it: ints as they are; SpreadBasedMarketMakerAgent's string
    ids (generateNewOrderId, SpreadBasedMarketMakerAgent.py:279-288) by their counter"""
    if isinstance(x, str):
        return SB_ID_BASE + int(x.rsplit("_", 1)[1])
    return int(x)


def _order_fields(o, with_qty=True):
    return [_oid(o.order_id), int(o.agent_id), 1 if o.is_buy_order else 0,
            int(o.quantity) if with_qty else 0, _price(o.limit_price)]


def encode(t_rel, recipient, mtype, msg):
    """Map one popped event to the fixed 10-word parity record."""
    f = [0, 0, 0, 0, 0, 0]
    if msg is None:
        kind = KIND["WAKEUP"] if mtype == 2 else KIND["KERNEL_CANCEL_ORDER"]
        return [t_rel, recipient, mtype, kind] + f
    b = msg.body
    m = b["msg"]
    req = "sender" in b and m not in ("LIMIT_ORDER", "CANCEL_ORDER", "MODIFY_ORDER")
    if m in ("WHEN_MKT_OPEN", "WHEN_MKT_CLOSE"):
        if req:
            kind = KIND[m + "_REQ"]
            f[0] = b["sender"]
        else:
            kind = KIND[m]
            f[0] = int(b["data"].value) - MIDNIGHT
    elif m == "QUERY_SPREAD":
        if req:
            kind = KIND["QUERY_SPREAD_REQ"]
            f[0], f[1] = b["sender"], int(b["depth"])
        else:
            kind = KIND["QUERY_SPREAD"]
            bids, asks = b["bids"], b["asks"]
            f[0] = _price(bids[0][0]) if bids else -1
            f[1] = int(bids[0][1]) if bids else 0
            f[2] = _price(asks[0][0]) if asks else -1
            f[3] = int(asks[0][1]) if asks else 0
            f[4] = _price(b["data"])
            f[5] = (1 if b["mkt_closed"] else 0) + 2 * len(bids) + (1 << 20) * len(asks)
    elif m == "QUERY_LAST_TRADE":
        if req:
            kind = KIND["QUERY_LAST_TRADE_REQ"]
            f[0] = b["sender"]
        else:
            kind = KIND["QUERY_LAST_TRADE"]
            f[0] = _price(b["data"])
            f[5] = 1 if b["mkt_closed"] else 0
    elif m == "QUERY_TRANSACTED_VOLUME":
        if req:
            kind = KIND["QUERY_TRANSACTED_VOLUME_REQ"]
            import pandas as pd
            f[0], f[1] = b["sender"], int(pd.to_timedelta(b["lookback_period"]).value)
        else:
            kind = KIND["QUERY_TRANSACTED_VOLUME"]
            f[0] = int(b["transacted_volume"])
            f[5] = 1 if b["mkt_closed"] else 0
    elif m == "LIMIT_ORDER":
        kind = KIND[m]
        f[:5] = _order_fields(b["order"])
    elif m == "CANCEL_ORDER":
        kind = KIND[m]
        # the agent's own order object travels by reference and may be partially
        # executed before delivery; the exchange only uses id/side/price.
        f[:5] = _order_fields(b["order"], with_qty=False)
    elif m == "MODIFY_ORDER":
        kind = KIND[m]
        f[:5] = _order_fields(b["new_order"])
    elif m in ("ORDER_ACCEPTED", "ORDER_CANCELLED"):
        kind = KIND[m]
        f[:5] = _order_fields(b["order"])
    elif m == "ORDER_EXECUTED":
        kind = KIND[m]
        f[:5] = _order_fields(b["order"])
        f[5] = _price(b["order"].fill_price)
    elif m == "MKT_CLOSED":
        kind = KIND[m]
    elif m == "ORDER_MODIFIED":
        kind = KIND[m]
        # the message aliases the order object now resting in the book (OrderBook.py:366),
        # whose quantity can change before delivery; the replay agent ignores the message
        f[:5] = _order_fields(b["new_order"], with_qty=False)
    elif m == "MARKET_DATA":
        # ExchangeAgent.publishOrderBookData: fresh level lists (not aliased)
        kind = KIND[m]
        bids, asks = b["bids"], b["asks"]
        f[0] = _price(bids[0][0]) if bids else -1
        f[1] = int(bids[0][1]) if bids else 0
        f[2] = _price(asks[0][0]) if asks else -1
        f[3] = int(asks[0][1]) if asks else 0
        f[4] = _price(b["last_transaction"])
        f[5] = len(bids) + (len(asks) << 8)
    elif m == "MARKET_DATA_SUBSCRIPTION_REQUEST":
        kind = KIND[m]
        f[0], f[1], f[2] = b["sender"], int(b["levels"]), int(b["freq"])
    elif m == "MARKET_DATA_SUBSCRIPTION_CANCELLATION":
        kind = KIND[m]
        f[0] = b["sender"]
    elif m == "QUERY_ORDER_STREAM":
        if req:
            kind = KIND["QUERY_ORDER_STREAM_REQ"]
            f[0], f[1] = b["sender"], int(b["length"])
        else:
            # the reply carries live references to the exchange's history epochs; the record
            # keeps how many epochs it returned
            kind = KIND["QUERY_ORDER_STREAM"]
            f[0] = len(b["orders"])
            f[5] = 1 if b["mkt_closed"] else 0
    else:
        raise RuntimeError("unknown message " + m)
    return [t_rel, recipient, mtype, kind] + [int(x) for x in f]


MIDNIGHT = 0
TRACE = []
BOOK_LOG = False  # book_freq 0 with a compact OrderBook.book_log (booklog fixtures only)
FLOG = False      # only the oracle's f_log (flog fixtures: the ExternalFileOracle's)
EXLOG = False     # only the exchange's own log (ExchangeAgent.log: EXCHANGE_AGENT.bz2)
EXLOG_ROWS = 40000  # exlog fixtures keep this many rows verbatim and every row as a digest
DIGEST_ROWS = 2000  # booklog fixtures above this many rows keep these verbatim and the rest as digests
BOOKLOG_FULL_ROWS = 300  # rows kept verbatim to run the reference's logOrderBookSnapshots on


class CompactBookLog(list):
    """OrderBook.book_log whose rows drop the quotes_seen zeros (a row holds every quote seen so
    far, which for a whole session is gigabytes); the first BOOKLOG_FULL_ROWS rows are also kept
    verbatim.  Row (t, [(price, volume) of the levels, bids negative])."""

    def __init__(self):
        super().__init__()
        self.full = []

    def append(self, row):
        if len(self.full) < BOOKLOG_FULL_ROWS:
            self.full.append(dict(row))
        t = int(row["QuoteTime"].value)
        super().append((t, [(int(q), int(v)) for q, v in row.items() if q != "QuoteTime" and v != 0]))
SUMMARY_ONLY = False


def install_stubs():
    jsons = types.ModuleType("jsons")
    jsons.dump = lambda obj, **kw: dict(vars(obj))
    sys.modules["jsons"] = jsons
    import pandas
    import pandas.io.json
    pandas.io.json.json_normalize = pandas.json_normalize
    pandas.SparseDataFrame = pandas.DataFrame
    if not hasattr(pandas.Timedelta, "delta"):  # pandas 0.24 (requirements.txt): ns as an int
        pandas.Timedelta.delta = property(lambda self: self.value)
    sys.path.insert(0, REF)


def run_config(cfg, seed, out, full, composition=None):
    """composition: {"date": "YYYY-MM-DD", "script": callable} of gen_config_fixtures.py, which builds
    its agent list from the reference's classes and calls Kernel.runner itself"""
    global MIDNIGHT
    install_stubs()
    import queue

    import pandas as pd

    class RecPQ(queue.PriorityQueue):
        def get(self, *a, **k):
            item = super().get(*a, **k)
            t, (rcp, mtype, msg) = item
            TRACE.append(encode(int(t.value) - MIDNIGHT, int(rcp), int(mtype.value), msg))
            return item

    import Kernel as K
    orig_init = K.Kernel.__init__

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.messages = RecPQ()
        CAPTURE["kernel"] = self

    K.Kernel.__init__ = init
    K.Kernel.writeLog = lambda *a, **k: None
    K.Kernel.writeSummaryLog = lambda *a, **k: None
    from agent.ExchangeAgent import ExchangeAgent
    orig_snapshots = ExchangeAgent.logOrderBookSnapshots
    ExchangeAgent.logOrderBookSnapshots = lambda *a, **k: None
    # the book snapshot log (OrderBook.book_log, appended after every limit order whenever
    # book_freq is not None) only feeds logOrderBookSnapshots at termination; rmsc01's
    # book_freq="M" would hold every snapshot row of a 6.5 h session in memory (the config's own
    # comment: "should be 0 but MemoryError").  It never touches the simulated arithmetic.
    _ex_init = ExchangeAgent.__init__

    def ex_init(self, *a, **k):
        _ex_init(self, *a, **k)
        if not BOOK_LOG:
            self.book_freq = None
        else:  # the full-depth snapshot log (rmsc03's own setting; -b 0 for the others)
            self.book_freq = 0
            for ob in self.order_books.values():
                ob.book_log = CompactBookLog()
    ExchangeAgent.__init__ = ex_init
    from agent.TradingAgent import TradingAgent
    TradingAgent.getTransactedVolume = TradingAgent.get_transacted_volume  # SURVEY.md key finding 3

    if cfg.startswith("rmsc03_sbmm"):
        # rmsc03 with its market maker slot (config/rmsc03.py:158-177) a SpreadBasedMarketMakerAgent
        # (agent/market_makers/SpreadBasedMarketMakerAgent.py; no reference config uses it): the
        # script's own arguments (window 5, 20 ticks, wake-up 1 s, random_state drawn in place),
        # order_size = --mm-min-order-size (20); subscribe=True (the agent's default) or, for
        # rmsc03_sbmm_poll, False
        from agent.market_makers.SpreadBasedMarketMakerAgent import SpreadBasedMarketMakerAgent
        sub = cfg == "rmsc03_sbmm"

        def factory(id, name, type, symbol, starting_cash, pov, min_order_size, window_size, num_ticks,
                    wake_up_freq, log_orders, random_state):
            return SpreadBasedMarketMakerAgent(
                id, "SPREAD_BASED_MARKET_MAKER_AGENT_{}".format(id), "SpreadBasedMarketMakerAgent", symbol,
                starting_cash, order_size=min_order_size, window_size=window_size, num_ticks=num_ticks,
                wake_up_freq=wake_up_freq, subscribe=sub, log_orders=log_orders, random_state=random_state)
        stub = types.ModuleType("agent.market_makers.POVMarketMakerAgent")
        stub.POVMarketMakerAgent = factory
        sys.modules["agent.market_makers.POVMarketMakerAgent"] = stub
        cfg_script = "rmsc03"
    else:
        cfg_script = cfg
    mm_args = None
    if cfg.startswith("rmsc03%"):
        # config/rmsc03.py with its market-maker options (config/rmsc03.py:39-43), the parameters
        # scripts/rmsc03.sh sweeps: rmsc03%POV,MIN_ORDER_SIZE,WINDOW_SIZE,NUM_TICKS,WAKE_UP_FREQ
        pov, mos, ws, nt, wf = cfg.split("%", 1)[1].split(",")
        mm_args = ["--mm-pov", pov, "--mm-min-order-size", mos, "--mm-window-size", ws, "--mm-num-ticks", nt,
                   "--mm-wake-up-freq", wf]
        cfg = cfg_script = "rmsc03"
    stop_at = None
    if "@" in cfg:  # CFG@HH:MM:SS: Kernel.runner(stopTime=that time of the day) instead of the script's
        cfg, stop_at = cfg.split("@")
        orig_runner = K.Kernel.runner

        def runner(self, *a, **k):
            k["stopTime"] = k["startTime"].normalize() + pd.Timedelta(stop_at)
            return orig_runner(self, *a, **k)
        K.Kernel.runner = runner
    replay = None
    twap = None
    if cfg.startswith(("twap:", "twap_e:")):
        # config/execution/marketreplay/execution_marketreplay.py TICKER DATE: the replay plus a
        # TWAPExecutionAgent; twap_e adds -e (execution_agents: the agent trades)
        twap = cfg.startswith("twap_e:")
        cfg = "marketreplay:" + cfg.split(":", 1)[1]
    if cfg.startswith("marketreplay:"):  # config/marketreplay.py TICKER DATE (Kernel.runner replay)
        _, ticker, rdate = cfg.split(":")
        replay = (ticker, rdate)
        cfg = cfg_script = "marketreplay"
        # the script's relative paths: the LOBSTER message file under data/lobster/ (linked to the
        # one the reference ships) and an empty processed-orders folder (the processor parses the
        # CSV; the committed pickles are never loaded)
        d = os.path.join("data", "lobster", "LOBSTER_SampleFile_%s_%s_1" % (ticker, rdate))
        os.makedirs(d, exist_ok=True)
        os.makedirs(os.path.join("data", "marketreplay", "level_1"), exist_ok=True)
        fn = "%s_%s_34200000_57600000_message_1.csv" % (ticker, rdate)
        src = os.path.join(REF, "data", "lobster", "LOBSTER_SampleFile_%s_1" % ticker, fn)
        if not os.path.exists(os.path.join(d, fn)):
            os.symlink(src, os.path.join(d, fn))
    date = {"sparse_zi_100": "2019-06-28", "sparse_zi_1000": "2019-06-28", "rmsc03": "2019-06-28",
            "value_noise": "2019-06-28", "rmsc01": "2019-06-28", "rmsc02": "2019-06-28",
            "obi_rmsc02": "2019-06-28", "random_fund_value": "2019-06-28",
            "random_fund_diverse": "2019-06-28", "hist_fund_value": "2019-06-28",
            "hist_fund_diverse": "2019-06-28", "marketreplay": replay[1] if replay else None,
            "rmsc03_sbmm": "2019-06-28", "rmsc03_sbmm_poll": "2019-06-28"}[cfg] if composition is None \
        else composition["date"]
    MIDNIGHT = int(pd.Timestamp(date).value)
    argv = ["abides.py", "-c", cfg_script, "-s", str(seed)]
    if cfg_script in ("rmsc03", "random_fund_value", "random_fund_diverse"):
        argv += ["-t", "ABM", "-d", "20190628"]
    if mm_args:
        argv += mm_args
    if replay:
        argv += ["-t", replay[0], "-d", replay[1]]
    module = "config." + cfg_script
    if twap is not None:
        module = "config.execution.marketreplay.execution_marketreplay"
        argv[2] = "execution_marketreplay"
        if twap:
            argv.append("-e")
    if cfg in ("hist_fund_value", "hist_fund_diverse"):  # ExternalFileOracle on the JPM mid-price series
        fp = os.path.abspath("fund_JPM_20190628.pkl")
        write_fund_files(fp)
        argv += ["-t", "JPM", "-d", "20190628", "-f", fp]
    sys.argv = argv
    buf = io.StringIO()
    real_stdout = sys.stdout
    sys.stdout = buf
    stop_error = None
    try:
        if composition is None:
            importlib.import_module(module)
        else:
            composition["script"]()
    except Exception as ex:  # e.g. ZeroIntelligenceAgent.kernelStopping's IndexError (rmsc01)
        if "kernel" not in CAPTURE:
            raise
        stop_error = "%s: %s" % (type(ex).__name__, ex)
    finally:
        sys.stdout = real_stdout
    kern = CAPTURE["kernel"]
    stdout = buf.getvalue().splitlines()

    from util.order.Order import Order
    agents = kern.agents
    ex = agents[0]
    sym = list(ex.order_books)[0]
    ob = ex.order_books[sym]

    def lvl(side):
        return [[[_oid(o.order_id), int(o.agent_id), int(o.quantity), _price(o.limit_price)] for o in level] for level in side]

    final = {
        "config": cfg, "seed": seed, "events": len(TRACE),
        "order_id_counter": int(Order.order_id),
        "n_order_ids": len(Order._order_ids),
        "bids": lvl(ob.bids), "asks": lvl(ob.asks),
        "last_trade": _price(ob.last_trade),
        "agents": [],
        "final_holdings_lines": [s for s in stdout if s.startswith("Final holdings")],
        "mean_lines": [],
        "final_time": int(kern.currentTime.value) - MIDNIGHT,
        "stop_error": stop_error,
    }
    take = False
    for s in stdout:
        if s.startswith("Mean ending value"):
            take = True
            continue
        if take:
            if s.startswith("Simulation ending"):
                break
            final["mean_lines"].append(s.strip())
    for a in agents[1:]:
        h = {k: int(v) for k, v in a.holdings.items()}
        final["agents"].append({
            "id": a.id, "cash": h.get("CASH"), "shares": h.get(sym, 0),
            "open_orders": [[_oid(o.order_id), 1 if o.is_buy_order else 0, int(o.quantity), _price(o.limit_price)]
                            for o in a.orders.values()],
        })
    tr = np.asarray(TRACE, dtype=np.int64)
    hs, h = [], FNV_OFF
    for i, rec in enumerate(TRACE):
        h = fnv_words(h, rec)
        if (i + 1) % 1000 == 0:
            hs.append(h)
    final["hash"] = "%016x" % h
    final["hash_checkpoints"] = ["%016x" % x for x in hs]
    # Kernel.summaryLog (Kernel.py:549-554): what writeSummaryLog pickles to summary_log.bz2
    summary = [{"AgentID": int(r["AgentID"]), "AgentStrategy": r["AgentStrategy"], "EventType": r["EventType"],
                "Event": r["Event"] if isinstance(r["Event"], (int, float)) else str(r["Event"])}
               for r in kern.summaryLog]
    with open(out + "_summary.json", "w") as f:
        json.dump(summary, f, indent=0)
    if FLOG:  # the oracle's f_log[sym] after kernelStopping (ExchangeAgent.kernelTerminating's frame)
        fl = ex.oracle.f_log[sym]
        np.savez_compressed(
            out + "_flog.npz",
            fund_time=np.asarray([int(pd.Timestamp(r["FundamentalTime"]).value) - MIDNIGHT for r in fl], dtype=np.int64),
            fund_value=np.asarray([r["FundamentalValue"] for r in fl], dtype=np.float64),
            fund_types=np.asarray(sorted({type(r["FundamentalValue"]).__name__ for r in fl})),
            fund_dtype=np.asarray(str(pd.DataFrame(fl).set_index("FundamentalTime")["FundamentalValue"].dtype)))
        return
    if BOOK_LOG:
        save_booklog(ex, ob, sym, orig_snapshots, out)
        return
    if EXLOG:
        save_exlog(ex, sym, out)
        return
    if SUMMARY_ONLY:
        return
    with open(out + ".json", "w") as f:
        json.dump(final, f, indent=0)
    keep = tr if full else tr[:20000]
    np.savez_compressed(out + ".npz", trace=keep)


CAPTURE = {}

FUND_CSV = os.path.join(REF, "data", "JPM_2019-06-28_34200_57571_orderbook_1.csv")


def fund_series():
    """The ExternalFileOracle input of the hist_fund_* fixtures: a mid-price series built the way
    util/formatting/mid_price_from_orderbook.py builds one ((ask_price_1 + bid_price_1) / 2 per
    book timestamp), from the level-1 book the reference ships (data/JPM_2019-06-28_..._orderbook_1.csv;
    the series its scripts name, scripts/hist_fund_value.sh, is not in the repository).  Rows
    with an empty side have no mid and are dropped."""
    import pandas as pd
    df = pd.read_csv(FUND_CSV)
    mid = (df["ask_price_1"] + df["bid_price_1"]) / 2
    s = pd.Series(mid.to_numpy(dtype=np.float64), index=pd.DatetimeIndex(pd.to_datetime(df["time"])))
    return s.dropna()


def write_fund_files(pickle_path):
    """our own series file for the reference's ExternalFileOracle (read_pickle of a file this
    script wrote) and the committed arrays the device and the oracle read"""
    import pandas as pd
    s = fund_series()
    s.to_pickle(pickle_path)
    mid0 = int(pd.Timestamp("2019-06-28").value)
    np.savez_compressed(os.path.join(HERE, "fund_JPM_20190628.npz"), t=s.index.asi8 - mid0, v=s.to_numpy())


def save_booklog(ex, ob, sym, orig_snapshots, out):
    """<out>_booklog.npz: every book_log row (flat int64: t - midnight, n, then n (price, volume)
    pairs, bids best-first then asks best-first), the exchange's BEST_BID / BEST_ASK / LAST_TRADE
    events (ExchangeAgent log: time, type 0/1/2, then the Event string), and
    logOrderBookSnapshots' DataFrames (book_freq 0; wide_book False and True) over the first
    BOOKLOG_FULL_ROWS rows, as the reference writes them."""
    import pandas as pd
    flat, digests = [], []
    for k, (t, lv) in enumerate(ob.book_log):
        bids = sorted((p, v) for p, v in lv if v < 0)[::-1]
        asks = sorted((p, v) for p, v in lv if v > 0)
        row = [t - MIDNIGHT, len(bids) + len(asks)]
        for p, v in bids + asks:
            row += [p, v]
        digests.append(fnv_words(FNV_OFF, row))  # every row: FNV-1a-64 over its int64 words
        if k < DIGEST_ROWS:
            flat += row
    types_ = {"BEST_BID": 0, "BEST_ASK": 1, "LAST_TRADE": 2}
    ev = [(int(r["EventTime"].value) - MIDNIGHT, types_[r["EventType"]], r["Event"]) for r in ex.log
          if r["EventType"] in types_]
    ev_digest = FNV_OFF
    for e_t, e_k, e_s in ev:  # every event: time, kind and the Event string's bytes
        ev_digest = fnv_words(ev_digest, [e_t, e_k] + list(e_s.encode()))
    rows_complete = len(ob.book_log) <= DIGEST_ROWS
    ev = ev if rows_complete else ev[:3 * DIGEST_ROWS]
    frames = {}
    full_rows = ob.book_log.full
    for wide in (False, True):
        got = {}
        ob.book_log = list(full_rows)
        ex.wide_book = wide
        ex.writeLog = lambda df, filename=None: got.update(df=df, filename=filename)
        orig_snapshots(ex, sym)
        df = got["df"]
        frames[wide] = df
    narrow, wide = frames[False], frames[True]
    has_oracle = getattr(ex, "oracle", None) is not None  # config/marketreplay.py: oracle=None
    flog = ex.oracle.f_log[sym] if has_oracle else []
    np.savez_compressed(
        out + "_booklog.npz",
        rows=np.asarray(flat, dtype=np.int64),
        rows_complete=np.asarray(rows_complete),
        row_digests=np.asarray(digests, dtype=np.uint64),
        ev_digest=np.asarray(ev_digest, dtype=np.uint64),
        n_events=np.asarray(len([r for r in ex.log if r["EventType"] in types_])),
        ev_t=np.asarray([e[0] for e in ev], dtype=np.int64),
        ev_type=np.asarray([e[1] for e in ev], dtype=np.int8),
        ev_text=np.asarray([e[2] for e in ev]),
        full_time=narrow.index.get_level_values(0).asi8 - MIDNIGHT,
        full_quote=np.asarray(narrow.index.get_level_values(1), dtype=np.int64),
        full_volume=narrow["Volume"].to_numpy(dtype=np.float64),
        full_dtype=np.asarray(str(narrow["Volume"].dtype)),
        full_filename=np.asarray(got["filename"]),
        wide_time=wide.index.asi8 - MIDNIGHT,
        wide_cols=np.asarray(wide.columns, dtype=np.int64),
        wide_values=wide.to_numpy(dtype=np.float64),
        wide_dtypes=np.asarray([str(d) for d in wide.dtypes]),
        # SparseMeanRevertingOracle.f_log[sym] after kernelStopping, the frame ExchangeAgent.
        # kernelTerminating writes as fundamental_<sym> (ExchangeAgent.py:111-117)
        fund_time=np.asarray([int(r["FundamentalTime"].value) - MIDNIGHT for r in flog], dtype=np.int64),
        fund_value=np.asarray([r["FundamentalValue"] for r in flog], dtype=np.float64),
        fund_types=np.asarray([type(r["FundamentalValue"]).__name__ for r in flog]),
        fund_dtype=np.asarray(str(pd.DataFrame(flog).set_index("FundamentalTime")["FundamentalValue"].dtype)
                              if flog else ""),
        full_rows=np.asarray(BOOKLOG_FULL_ROWS))


def save_exlog(ex, sym, out):
    """<out>_exlog.npz: ExchangeAgent.log, the frame Agent.kernelTerminating writes as
    EXCHANGE_AGENT.bz2 (agent/Agent.py:86-95; log_events=True, ExchangeAgent.py:39).  One row per
    logEvent call (Agent.py:97-110): EventTime (ns since midnight, -1 for AGENT_TYPE's None),
    EventType, and the Event as the log holds it -- an int (the sender of a non-order message,
    ExchangeAgent.py:167), a string (AGENT_TYPE, BEST_BID / BEST_ASK / LAST_TRADE,
    util/OrderBook.py:112-141) or, with log_orders, the order's attribute dict (the jsons.dump
    stub returns vars(order); ExchangeAgent.py:163-165, 477-482).  The first EXLOG_ROWS rows
    verbatim, every row in an FNV-1a digest (tests/golden_util.exlog_row_words)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from golden_util import exlog_row_words
    rows = []
    keys = set()
    for r in ex.log:
        t = -1 if r["EventTime"] is None else int(r["EventTime"].value) - MIDNIGHT
        ev = r["Event"]
        if isinstance(ev, dict):
            keys.add(",".join(ev))
            if ev["symbol"] != sym:
                raise ValueError("order of another symbol in the exchange log")
            fill = ev["fill_price"]
            rows.append((t, r["EventType"], 2, 0, "", (
                int(ev["agent_id"]), int(ev["time_placed"].value) - MIDNIGHT, int(ev["quantity"]),
                1 if ev["is_buy_order"] else 0, _oid(ev["order_id"]), -(1 << 63) if fill is None else _price(fill),
                _price(ev["limit_price"]))))
        elif isinstance(ev, str):
            rows.append((t, r["EventType"], 1, 0, ev, (0,) * 7))
        else:
            rows.append((t, r["EventType"], 0, int(ev), "", (0,) * 7))
    digest = FNV_OFF
    for row in rows:
        digest = fnv_words(digest, exlog_row_words(*row))
    keep = rows[:EXLOG_ROWS]
    types_ = sorted({r[1] for r in rows})
    o = np.asarray([r[5] for r in keep], dtype=np.int64).reshape(-1, 7)
    np.savez_compressed(
        out + "_exlog.npz",
        n_rows=np.asarray(len(rows)), digest=np.asarray(digest, dtype=np.uint64),
        t=np.asarray([r[0] for r in keep], dtype=np.int64),
        types=np.asarray(types_), type_idx=np.asarray([types_.index(r[1]) for r in keep], dtype=np.int16),
        ekind=np.asarray([r[2] for r in keep], dtype=np.int8),
        eint=np.asarray([r[3] for r in keep], dtype=np.int64),
        estr=np.asarray([r[4] for r in keep]),
        order=o,  # agent_id, time_placed, quantity, is_buy_order, order_id, fill_price, limit_price
        order_keys=np.asarray(sorted(keys)), symbol=np.asarray(sym),
        name=np.asarray(ex.name), log_orders=np.asarray(bool(ex.log_orders)))


def rng_kats(path):
    """numpy legacy RandomState known answers (MT19937 + legacy distributions)."""
    out = {}
    for seed in (0, 1, 5489, 123456789, 2 ** 32 - 1):
        rs = np.random.RandomState(seed)
        d = {"u32": rs.randint(0, 2 ** 32, size=700, dtype=np.uint64).astype(np.int64).tolist()}
        rs = np.random.RandomState(seed)
        d["double"] = [float(rs.rand()) for _ in range(300)]
        rs = np.random.RandomState(seed)
        seq = []
        for i in range(400):
            k = i % 8
            if k == 0:
                seq.append(["randint", 0, 100, int(rs.randint(0, 100))])
            elif k == 1:
                seq.append(["normal", 1e5, 100.0, float(rs.normal(1e5, 100.0))])
            elif k == 2:
                seq.append(["exponential", 1e12, 0, float(rs.exponential(1e12))])
            elif k == 3:
                seq.append(["uniform", 21000.0, 100000.0, float(rs.uniform(21000, 100000))])
            elif k == 4:
                seq.append(["randint", 20, 50, int(rs.randint(20, 50))])
            elif k == 5:
                seq.append(["randint", 0, 2, int(rs.randint(0, 2))])
            elif k == 6:
                seq.append(["rand", 0, 0, float(rs.rand())])
            else:
                seq.append(["randint", 0, 1, int(rs.randint(0, 1))])
        d["mixed"] = seq
        out[str(seed)] = d
    with open(path, "w") as f:
        json.dump(out, f)


def main():
    global SUMMARY_ONLY
    global BOOK_LOG
    global FLOG
    global EXLOG
    if sys.argv[1] == "run":
        SUMMARY_ONLY = "--summary-only" in sys.argv
        BOOK_LOG = "--booklog" in sys.argv
        FLOG = "--flog" in sys.argv
        EXLOG = "--exlog" in sys.argv
        run_config(sys.argv[2], int(sys.argv[3]), sys.argv[4], "--full" in sys.argv)
        return
    if sys.argv[1] in ("booklog", "flog", "exlog"):  # <cfg>_<seed>_booklog.npz / _flog.npz / _exlog.npz
        if sys.argv[1] == "exlog":  # the exchange's agent log, EXCHANGE_AGENT.bz2 (log_orders on / off)
            jobs = [("sparse_zi_100", 123456789), ("sparse_zi_1000", 123456789), ("rmsc03", 123456789),
                    ("value_noise", 7), ("marketreplay:IBM:2003-01-14", 1)]
        elif sys.argv[1] == "booklog":  # order-book snapshot outputs (the replays: config/marketreplay.py's book_freq 0)
            jobs = [("rmsc03", 123456789), ("value_noise", 7), ("marketreplay:IBM:2003-01-14", 1),
                    ("marketreplay:GOOG:2012-06-21", 1)]
        else:  # the ExternalFileOracle's f_log (fundamental_JPM)
            jobs = [("hist_fund_value", 7), ("hist_fund_diverse", 7)]
        if len(sys.argv) > 2:
            jobs = [j for j in jobs if j[0].startswith(sys.argv[2])]
        procs = []
        for cfg, seed in jobs:
            out = os.path.join(HERE, "%s_%d" % (cfg.replace(":", "_"), seed))
            cmd = [sys.executable, os.path.abspath(__file__), "run", cfg, str(seed), out, "--" + sys.argv[1]]
            procs.append(subprocess.Popen(cmd, cwd=tempfile.mkdtemp(prefix="gf_"),
                                          env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1")))
        for (cfg, seed), p in zip(jobs, procs):
            print(cfg, seed, "rc", p.wait())
        return
    if sys.argv[1] == "summaries":  # only the summary logs (<cfg>_<seed>_summary.json)
        sys.argv[1] = "all"
        extra = ["--summary-only"]
    else:
        extra = []
    assert sys.argv[1] == "all"
    if not extra:
        rng_kats(os.path.join(HERE, "rng_kats.json"))
    jobs = [("sparse_zi_100", 123456789, True), ("rmsc03", 123456789, False),
            ("rmsc03", 1008, True), ("rmsc03", 7, False), ("sparse_zi_1000", 123456789, False),
            ("value_noise", 123456789, True), ("value_noise", 7, False),
            # rmsc01 (2M pops each; ~25 min of the reference): 123456789 ends in the reference's
            # IndexError in ZeroIntelligenceAgent.kernelStopping (recorded as stop_error)
            ("rmsc01", 7, False), ("rmsc01", 99, False), ("rmsc01", 123456789, False),
            # rmsc02: rmsc01 with market-data subscriptions (market maker, momentum agents) and a
            # latency matrix with noise, from midnight to 17:00
            ("rmsc02", 7, False), ("rmsc02", 123456789, False),
            # obi_rmsc02: rmsc02's market with 89 ZI, 5 OrderBookImbalanceAgent, 5 momentum agents
            ("obi_rmsc02", 7, False), ("obi_rmsc02", 123456789, False),
            # seeds on which the OBI agents trade (found with the oracle; 7 and 123456789 stay flat)
            ("obi_rmsc02", 30, False), ("obi_rmsc02", 107, False),
            # random_fund_value: rmsc03's agent classes at 5,100 agents (5000 noise, 100 value) over
            # the whole 09:30-16:00 session; ~5,100 pending events in the queue
            ("random_fund_value", 7, False), ("random_fund_value", 123456789, False),
            # random_fund_diverse: random_fund_value plus a MarketMakerAgent and 25 momentum agents
            ("random_fund_diverse", 7, False), ("random_fund_diverse", 123456789, False),
            # hist_fund_value / hist_fund_diverse: the same markets on an ExternalFileOracle (the
            # fundamental is the JPM level-1 mid-price series, interpolated; fund_series())
            ("hist_fund_value", 7, False), ("hist_fund_value", 123456789, False),
            ("hist_fund_diverse", 7, False), ("hist_fund_diverse", 123456789, False),
            # config/marketreplay.py: the exchange and the MarketReplayAgent under Kernel.runner
            ("marketreplay:IBM:2003-01-14", 1, False), ("marketreplay:GOOG:2012-06-21", 1, False),
            # Kernel.runner with a caller's stopTime (the scripts' own kernelStopTime replaced)
            ("rmsc03@11:00:00", 123456789, True), ("value_noise@10:15:00", 7, True),
            ("sparse_zi_100@09:45:30", 123456789, True),
            # config/execution/marketreplay/execution_marketreplay.py: the replay plus the TWAP
            # execution agent, passive (no -e) and trading (-e)
            ("twap:IBM:2003-01-14", 1, False), ("twap_e:IBM:2003-01-14", 1, True),
            ("twap:GOOG:2012-06-21", 1, False), ("twap_e:GOOG:2012-06-21", 1, True),
            # rmsc03 with a SpreadBasedMarketMakerAgent in the market maker's slot: subscribe=True
            # (MARKET_DATA every 10 s) and polling (QUERY_SPREAD every second)
            ("rmsc03_sbmm", 123456789, True), ("rmsc03_sbmm", 7, False),
            ("rmsc03_sbmm_poll", 123456789, True), ("rmsc03_sbmm_poll", 7, False),
            # a polling seed whose first QUERY_SPREAD finds a side empty before any mid was known:
            # receiveMessage's UnboundLocalError ends the reference's run after 649 pops
            ("rmsc03_sbmm_poll", 123456798, True),
            # config/rmsc03.py with the market-maker options of scripts/rmsc03.sh (pov 0.05, min
            # order size 25, window 5, 50 ticks, wake-up "10S"), on the script's seeds 30-35
            ] + [("rmsc03%0.05,25,5,50,10S", s, s == 30) for s in range(30, 36)]
    if len(sys.argv) > 2:
        jobs = [j for j in jobs if j[0] == sys.argv[2] or j[0].startswith(sys.argv[2] + ":")]
    procs = []
    for cfg, seed, full in jobs:
        out = os.path.join(HERE, "%s_%d" % (cfg.replace("@", "_stop").replace(":", ""), seed) if "@" in cfg
                           else "%s_%d" % (cfg.replace(":", "_").replace("%", "_mm_").replace(",", "_"), seed))
        cmd = [sys.executable, os.path.abspath(__file__), "run", cfg, str(seed), out] + (["--full"] if full else []) + extra
        wd = tempfile.mkdtemp(prefix="gf_")
        procs.append((cfg, seed, subprocess.Popen(cmd, cwd=wd, env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))))
    for cfg, seed, p in procs:
        rc = p.wait()
        print(cfg, seed, "rc", rc)


if __name__ == "__main__":
    main()
