"""Order-book outputs of the reference's exchange, rebuilt from libmxa's book-update log.

The device writes one 16-byte record per handled limit order and per cancellation
(include/mxa.h mxa_book_rec).  This module replays the price-level volumes from them into what
the reference produces at the end of OrderBook.handleLimitOrder (util/OrderBook.py:112-168):

  * the OrderBook.book_log rows (one per handled limit order: every level, bids negative),
    archived by ExchangeAgent.logOrderBookSnapshots (agent/ExchangeAgent.py:389-469) as
    ORDERBOOK_<symbol>_FULL.bz2 with book_freq 0 (rmsc03's setting), narrow or wide_book;
  * the exchange's BEST_BID / BEST_ASK / LAST_TRADE events (Agent.logEvent rows EventTime,
    EventType, Event), the series cli/event_midpoint.py and cli/event_ticker.py read.

Matching at level granularity is exact: executeOrder (OrderBook.py:172-240) fills an incoming
order from the best opposite level while its price crosses, each level giving min(remaining,
level volume) at the level's price, so the level volumes, the executed quantity and the
LAST_TRADE average int(round(sum p*q / sum q)) follow from the records alone.

The same stream carries SparseMeanRevertingOracle.f_log (util/oracle/SparseMeanRevertingOracle.py:
63, 122): one record per fundamental value computed (price BL_FUNDAMENTAL, qty the value), the
series ExchangeAgent.kernelTerminating writes as fundamental_<symbol>.bz2 (ExchangeAgent.py:111-117).

With mxa_set_exchange_log the stream also carries the exchange's own log, ExchangeAgent.log
(agent/Agent.py:97-110), written by Agent.kernelTerminating as EXCHANGE_AGENT.bz2 (Agent.py:86-95):
a record per message the exchange logs on receipt (ExchangeAgent.py:162-167), per ORDER_*
notification it sends with log_orders (:477-482), and per order created (its time_placed);
exchange_log rebuilds the rows with the BEST_BID / BEST_ASK / LAST_TRADE rows in their place.

Rows are kept in one flat int64 array, the format the CPU oracle writes too:
    t, n, executed quantity, average trade price (0 without an execution),
    then n (price, volume) pairs: bids best-first (negative volumes), then asks best-first.
"""
import bisect

import numpy as np

REC_DTYPE = np.dtype([("t", "<i8"), ("price", "<i4"), ("qty", "<i4")])
BL_FUNDAMENTAL = -(1 << 31)
BL_FUND_LO, BL_FUND_HI = -(1 << 31) + 1, -(1 << 31) + 2  # ExternalFileOracle f_log value words
BL_MODIFY = 1 << 30  # modifyOrder on the replay book: price -(p | BL_MODIFY | side << 29), qty the volume change
# the exchange's own log (include/mxa.h MXA_BL_EV_*): price = code + message kind
BL_EV_RX = -(1 << 31) + 256
BL_EV_NT = BL_EV_RX + 256
BL_EV_PLACE = BL_EV_RX + 512
BL_EV_END = BL_EV_RX + 768
FILL_NONE = -(1 << 31)
# message kinds (the trace's, tests/golden/gen_fixtures.py KIND) by the msg names the log holds
KIND_NAMES = {1: "WHEN_MKT_OPEN", 2: "WHEN_MKT_CLOSE", 5: "QUERY_SPREAD", 7: "QUERY_LAST_TRADE",
              9: "QUERY_TRANSACTED_VOLUME", 11: "LIMIT_ORDER", 12: "CANCEL_ORDER", 13: "MODIFY_ORDER",
              14: "ORDER_ACCEPTED", 15: "ORDER_EXECUTED", 16: "ORDER_CANCELLED", 21: "QUERY_ORDER_STREAM",
              23: "MARKET_DATA_SUBSCRIPTION_REQUEST", 24: "MARKET_DATA_SUBSCRIPTION_CANCELLATION"}
K_LIMIT, K_CANCEL = 11, 12
R_BAR = 100000.0           # SparseMeanRevertingOracle r_bar of every plain config (a float)
MKT_OPEN_NS = (9 * 60 + 30) * 60 * 10**9
SESSION_DATE = "2019-06-28"  # the plain configs' simulated date (abides.py -d / config defaults)
# get_quote_range_iterator's excluded quotes (ExchangeAgent.py:399)
FORBIDDEN_QUOTES = (0, 19999900)


def exlog_mask(rec):
    """the exchange log's records (include/mxa.h MXA_BL_EV_*) and the order records after them"""
    p = np.asarray(rec, dtype=REC_DTYPE)["price"].astype(np.int64)
    code = (p >= BL_EV_RX) & (p < BL_EV_END)
    has_order = ((p >= BL_EV_RX + K_LIMIT) & (p <= BL_EV_RX + K_CANCEL)) | ((p >= BL_EV_NT) & (p < BL_EV_PLACE))
    follows = np.zeros(len(p), dtype=bool)
    follows[1:] = has_order[:-1]
    return code | follows


def book_mask(rec):
    """the records that change the book (limit orders, cancellations, modifyOrder): not f_log
    records, not the exchange log's records nor the order records that follow them"""
    p = np.asarray(rec, dtype=REC_DTYPE)["price"].astype(np.int64)
    f_log = (p >= -(1 << 31)) & (p <= BL_FUND_HI)
    return ~f_log & ~exlog_mask(rec)


def rows_from_records(rec):
    """Replay device records into flat book_log rows (format above)."""
    rec = np.asarray(rec, dtype=REC_DTYPE)
    rec = rec[book_mask(rec)]  # f_log and exchange-log records carry no book change
    vol = ({}, {})       # bids, asks: price -> resting volume
    px = ([], [])        # their prices, ascending
    out = []
    for t, p, q in zip(rec["t"].tolist(), rec["price"].tolist(), rec["qty"].tolist()):
        if p < 0 and (-p) & BL_MODIFY:  # modifyOrder (replay): the level's head takes the new quantity
            s = ((-p) >> 29) & 1
            p = (-p) & ((1 << 29) - 1)
            vol[s][p] += q
            continue
        if p < 0:  # cancelOrder: the level loses the cancelled quantity
            s = 0 if q > 0 else 1
            p = -p
            v = vol[s][p] - abs(q)
            if v:
                vol[s][p] = v
            else:
                del vol[s][p]
                px[s].pop(bisect.bisect_left(px[s], p))
            continue
        own = 0 if q > 0 else 1  # the side the order rests on
        opp = 1 - own
        q = abs(q)
        xq = tp = 0
        ov, op = vol[opp], px[opp]
        while q and op and (op[0] <= p if own == 0 else op[-1] >= p):
            best = op[0] if own == 0 else op[-1]
            v = ov[best]
            c = v if q >= v else q
            q -= c
            xq += c
            tp += best * c
            if c == v:
                del ov[best]
                op.pop(0 if own == 0 else -1)
            else:
                ov[best] = v - c
        if q:
            if p in vol[own]:
                vol[own][p] += q
            else:
                vol[own][p] = q
                bisect.insort(px[own], p)
        out += [t, len(px[0]) + len(px[1]), xq, int(round(tp / xq)) if xq else 0]
        for b in reversed(px[0]):
            out += [b, -vol[0][b]]
        for a in px[1]:
            out += [a, vol[1][a]]
    return np.asarray(out, dtype=np.int64)


def iter_rows(flat):
    """(t, executed qty, average price, prices, volumes) per row."""
    flat = np.asarray(flat, dtype=np.int64)
    i, n = 0, len(flat)
    while i < n:
        t, m, xq, avg = (int(x) for x in flat[i:i + 4])
        pv = flat[i + 4:i + 4 + 2 * m]
        yield t, xq, avg, pv[0::2], pv[1::2]
        i += 4 + 2 * m


def strip_executions(flat):
    """the rows without the executed-quantity / average-price words (t, n, pairs)"""
    out = []
    for t, _, _, p, v in iter_rows(flat):
        out += [t, len(p)]
        out += np.stack([p, v], axis=1).ravel().tolist()
    return np.asarray(out, dtype=np.int64)


def exchange_events(flat, symbol):
    """The exchange log rows handleLimitOrder appends (OrderBook.py:114-141), in order:
    (t, EventType, Event) with Event exactly the reference's strings."""
    ev = []
    for t, xq, avg, p, v in iter_rows(flat):
        bid = np.flatnonzero(v < 0)
        ask = np.flatnonzero(v > 0)
        if len(bid):
            ev.append((t, "BEST_BID", "%s,%d,%d" % (symbol, p[bid[0]], -v[bid[0]])))
        if len(ask):
            ev.append((t, "BEST_ASK", "%s,%d,%d" % (symbol, p[ask[0]], v[ask[0]])))
        if xq:
            ev.append((t, "LAST_TRADE", "{},${:0.4f}".format(xq, avg)))
    return ev


def _order(r, agent, placed, symbol, date):
    """the order a log row carries, as the jsons.dump stub of the fixtures sees it (vars(order):
    util/order/LimitOrder.py:14-19, Order.py:11-33): time_placed in ns since midnight here"""
    t, p, q = int(r["t"]), int(r["price"]), int(r["qty"])
    oid = t & 0xFFFFFFFF
    oid = oid - (1 << 32) if oid >= 1 << 31 else oid
    fill = t >> 32
    if oid not in placed:
        raise ValueError("order %d of the exchange log was never placed in this log" % oid)
    return {"agent_id": agent, "time_placed": placed[oid], "symbol": symbol, "quantity": abs(q),
            "is_buy_order": q > 0, "order_id": oid, "fill_price": None if fill == FILL_NONE else fill,
            "limit_price": p}


def exchange_log(rec, symbol, agent_type="ExchangeAgent"):
    """ExchangeAgent.log (Agent.logEvent rows, Agent.py:97-110) from a book-update stream written
    with the exchange log on: [(EventTime ns since midnight or None, EventType, Event)].

    Row order is the reference's: AGENT_TYPE (Agent.__init__, currentTime None); per received
    message its row (ExchangeAgent.py:162-167: the sender, or with log_orders the order of a
    LIMIT_ORDER / CANCEL_ORDER); within handleLimitOrder the ORDER_EXECUTED pairs and the
    ORDER_ACCEPTED rows (sendMessage, :477-482) and then BEST_BID / BEST_ASK / LAST_TRADE
    (OrderBook.py:112-141); cancelOrder's ORDER_CANCELLED.  Order Events are dicts in
    vars(order) key order with time_placed in ns (jsons_dump_order serializes them)."""
    rec = np.asarray(rec, dtype=REC_DTYPE)
    p = rec["price"].astype(np.int64)
    bm = book_mask(rec)
    per_limit = [[]]
    for t, xq, avg, pr, v in iter_rows(rows_from_records(rec)):
        ev = []
        bid = np.flatnonzero(v < 0)
        ask = np.flatnonzero(v > 0)
        if len(bid):
            ev.append((t, "BEST_BID", "%s,%d,%d" % (symbol, pr[bid[0]], -v[bid[0]])))
        if len(ask):
            ev.append((t, "BEST_ASK", "%s,%d,%d" % (symbol, pr[ask[0]], v[ask[0]])))
        if xq:
            ev.append((t, "LAST_TRADE", "{},${:0.4f}".format(xq, avg)))
        per_limit.append(ev)
    per_limit = per_limit[1:]
    rows = [(None, "AGENT_TYPE", agent_type)]
    placed, pending, li, i, n = {}, [], 0, 0, len(rec)
    while i < n:
        pi, ti, qi = int(p[i]), int(rec["t"][i]), int(rec["qty"][i])
        if (BL_EV_NT <= pi < BL_EV_PLACE or pi in (BL_EV_RX + K_LIMIT, BL_EV_RX + K_CANCEL)) and i + 1 >= n:
            # an order row's second record is missing: the stream was cut (a full log, env error
            # ERR_BOOK_LOG_FULL, or a partial read)
            raise ValueError("exchange log truncated after record %d (order row without its order record; "
                             "a full book-update log ends the env with ERR_BOOK_LOG_FULL)" % i)
        if BL_EV_NT <= pi < BL_EV_PLACE:  # a notification of the order being handled
            rows.append((ti, KIND_NAMES[pi - BL_EV_NT], _order(rec[i + 1], qi, placed, symbol, None)))
            i += 2
            continue
        rows += pending  # anything else: the last limit order's handling is over
        pending = []
        if BL_EV_RX <= pi < BL_EV_NT:
            k = pi - BL_EV_RX
            if k in (K_LIMIT, K_CANCEL):
                rows.append((ti, KIND_NAMES[k], _order(rec[i + 1], qi, placed, symbol, None)))
                i += 2
                continue
            rows.append((ti, KIND_NAMES[k], qi))
        elif pi == BL_EV_PLACE:
            placed[qi] = ti
        elif bm[i] and pi > 0:  # a limit order: its BEST rows follow its notifications
            pending = per_limit[li]
            li += 1
        i += 1
    return rows + pending


def jsons_dump_order(d, date=SESSION_DATE):
    """js.dump(order, strip_privates=True) of jsons 0.8.8 (requirements.txt), restated from its
    published serializers: the object's public attributes in __dict__ order, ints and bools as
    they are, None kept, and time_placed (a pandas Timestamp, a datetime) as RFC 3339
    '%Y-%m-%dT%H:%M:%S' with '.%f' when it has microseconds and the local UTC offset of a naive
    datetime ('Z' on a UTC host).  PARITY UNPINNED: jsons is not importable here, so only the
    fields (exchange_log's dicts) are checked against the reference, not this string form."""
    import pandas as pd
    out = dict(d)
    ts = pd.Timestamp(date) + pd.Timedelta(int(d["time_placed"]), unit="ns")
    pat = "%Y-%m-%dT%H:%M:%S" + (".%f" if ts.microsecond else "")
    out["time_placed"] = ts.strftime(pat) + "Z"
    return out


def exchange_log_frame(rows, date=SESSION_DATE):
    """pd.DataFrame(ExchangeAgent.log).set_index("EventTime") as Agent.kernelTerminating writes it
    to EXCHANGE_AGENT.bz2 (Agent.py:86-95): EventTime NaT for AGENT_TYPE, order Events through
    jsons_dump_order"""
    import pandas as pd
    base = pd.Timestamp(date)
    ev = [jsons_dump_order(e, date) if isinstance(e, dict) else e for _, _, e in rows]
    df = pd.DataFrame({"EventTime": [None if t is None else base + pd.Timedelta(t, unit="ns") for t, _, _ in rows],
                       "EventType": [r[1] for r in rows], "Event": ev})
    return df.set_index("EventTime")


def exchange_events_frame(flat, symbol, date=SESSION_DATE):
    """exchange_events as the exchange's log DataFrame (Agent.kernelTerminating,
    Agent.py:92-95): index EventTime, columns EventType, Event."""
    import pandas as pd
    ev = exchange_events(flat, symbol)
    base = pd.Timestamp(date)
    df = pd.DataFrame({"EventTime": base + pd.to_timedelta([e[0] for e in ev], unit="ns"),
                       "EventType": [e[1] for e in ev], "Event": [e[2] for e in ev]})
    return df.set_index("EventTime")


def book_log_frame(flat, date=SESSION_DATE):
    """pd.DataFrame(book.book_log).set_index("QuoteTime") (ExchangeAgent.py:413-414): a column
    per quote in first-appearance order; a row holds the quote's level volume, 0 once the quote
    has been seen (OrderBook.quotes_seen) and NaN before; columns without a NaN stay int64."""
    import pandas as pd
    times, cols, first, cells = [], {}, [], []
    for r, (t, _, _, p, v) in enumerate(iter_rows(flat)):
        times.append(t)
        for q, vol in zip(p.tolist(), v.tolist()):
            j = cols.get(q)
            if j is None:
                j = cols[q] = len(first)
                first.append(r)
            cells.append((r, j, vol))
    nr, nc = len(times), len(first)
    m = np.where(np.arange(nr)[:, None] >= np.asarray(first, dtype=np.int64)[None, :], 0.0, np.nan)
    if cells:
        c = np.asarray(cells, dtype=np.int64)
        m[c[:, 0], c[:, 1]] = c[:, 2]
    index = pd.DatetimeIndex(pd.Timestamp(date) + pd.to_timedelta(np.asarray(times, dtype=np.int64), unit="ns"),
                             name="QuoteTime")
    data = {}
    for q, j in cols.items():
        col = m[:, j]
        data[q] = col.astype(np.int64) if first[j] == 0 else col
    return pd.DataFrame(data, index=index, columns=list(cols))


def orderbook_full(flat, date=SESSION_DATE, wide_book=False):
    """ExchangeAgent.logOrderBookSnapshots with book_freq 0 (ExchangeAgent.py:410-432, 457-464):
    the last row per timestamp, sorted by time; narrow: a (time, quote) MultiIndex over every
    time and every quote seen (except 0 and 19999900) with one column Volume; wide_book: the
    quote columns sorted."""
    import warnings

    import pandas as pd
    df = book_log_frame(flat, date)
    df = df[~df.index.duplicated(keep="last")]
    df = df.sort_index()
    if wide_book:
        return df.reindex(sorted(df.columns), axis=1)
    quotes = sorted(q for q in df.columns.unique() if q not in FORBIDDEN_QUOTES)
    filled = pd.MultiIndex.from_product([df.index, quotes], names=["time", "quote"])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        s = df.stack()
    s = s.reindex(filled)
    out = pd.DataFrame(index=s.index)
    out["Volume"] = s
    return out


def fundamental_log(rec, mkt_open=MKT_OPEN_NS, r_bar=R_BAR, external=False):
    """the oracle's f_log[symbol] as (times ns, values) arrays:
    * SparseMeanRevertingOracle (SMRO:63, 122): the opening entry (mkt_open, r_bar) and one
      (FundamentalTime, FundamentalValue) per computed value (BL_FUNDAMENTAL records);
    * ExternalFileOracle (ExternalFileOracle.py:19, 97): one entry per getPriceAtTime inside the
      series, the opening lookup included (BL_FUND_LO / BL_FUND_HI record pairs: the double)."""
    rec = np.asarray(rec, dtype=REC_DTYPE)
    lo = rec[rec["price"] == BL_FUND_LO]
    if external:
        hi = rec[rec["price"] == BL_FUND_HI]
        if len(hi) != len(lo) or (hi["t"] != lo["t"]).any():
            raise ValueError("ExternalFileOracle f_log records must come in (low, high) pairs")
        bits = (lo["qty"].astype(np.int64) & 0xFFFFFFFF) | ((hi["qty"].astype(np.int64) & 0xFFFFFFFF) << 32)
        return lo["t"].astype(np.int64), bits.astype(np.uint64).view(np.float64)
    f = rec[rec["price"] == BL_FUNDAMENTAL]
    t = np.concatenate([[mkt_open], f["t"]]).astype(np.int64)
    v = np.concatenate([[r_bar], f["qty"].astype(np.float64)])
    return t, v


def fundamental_frame(rec, date=SESSION_DATE, mkt_open=MKT_OPEN_NS, r_bar=R_BAR, external=False):
    """pd.DataFrame(f_log[symbol]).set_index("FundamentalTime") as ExchangeAgent.kernelTerminating
    writes it (ExchangeAgent.py:111-117): FundamentalValue float64 (the opening r_bar is a float;
    the ExternalFileOracle's values are interpolated floats).  Empty for an ExternalFileOracle that
    was never asked inside its series (the reference then writes no file)."""
    import pandas as pd
    t, v = fundamental_log(rec, mkt_open, r_bar, external)
    idx = pd.DatetimeIndex(pd.Timestamp(date) + pd.to_timedelta(t, unit="ns"), name="FundamentalTime")
    return pd.DataFrame({"FundamentalValue": v}, index=idx)
