"""Replay-tape ingestion: LOBSTER message files -> the packed per-record arrays the replay
agent consumes.

`load_lobster` restates LOBSTEROrdersProcessor.processOrders (MarketReplayAgent.py:178-220)
on the CSV path (the reference's processed-pickle cache is never read): columns
TIMESTAMP (seconds after midnight), EVENT_TYPE (ignored, as in the reference), ORDER_ID,
SIZE, PRICE (1e-4 $), BUY_SELL_FLAG (1 buy / -1 sell); time = date + 09:30 + (s - 09:30)
via pandas Timedelta; PRICE / 100 truncated to int (cents); keep 09:30 <= time < 16:00;
records grouped by time in file order (`groupby(level=0)`).
"""
import os

import numpy as np

OPEN = "09:30:00"
CLOSE = "16:00:00"


class Tape:
    """Time-sorted replay records: t (ns since midnight), oid, price (cents), size, buy, and the
    ticker they belong to (`symbol`: the MarketReplayAgent's symbol, config/marketreplay.py -t)."""

    def __init__(self, t, oid, price, size, buy, symbol=None, date=None):
        self.symbol = symbol
        self.date = date  # the simulated date (YYYY-MM-DD): the outputs' timestamps
        self.t = np.ascontiguousarray(t, dtype=np.int64)
        self.oid = np.ascontiguousarray(oid, dtype=np.int64)
        self.price = np.ascontiguousarray(price, dtype=np.int64)
        self.size = np.ascontiguousarray(size, dtype=np.int64)
        self.buy = np.ascontiguousarray(buy, dtype=np.int8)
        n = len(self.t)
        if not (len(self.oid) == len(self.price) == len(self.size) == len(self.buy) == n) or n == 0:
            raise ValueError("tape arrays must be non-empty and of equal length")
        if (np.diff(self.t) < 0).any():
            raise ValueError("tape must be time-sorted")
        if (self.oid < 0).any():
            raise ValueError("negative ORDER_ID")
        # ORDER_ID 0 records (LOBSTER hidden executions) take auto ids from the global
        # Order.order_id counter (Order.py:26) that DummyRL's orders also use
        self.n_auto = int((self.oid == 0).sum())

    def __len__(self):
        return len(self.t)

    def save(self, path):
        extra = {"symbol": np.array(self.symbol)} if self.symbol else {}
        if self.date:
            extra["date"] = np.array(self.date)
        np.savez_compressed(path, t=self.t, oid=self.oid, price=self.price, size=self.size, buy=self.buy, **extra)

    @classmethod
    def load(cls, path, symbol=None, date=None):
        """symbol / date: the ticker and the simulated date; default the ones saved with the tape,
        else those of a tape_<SYM>_<YYYY-MM-DD>.npz file name"""
        z = np.load(path, allow_pickle=False)
        base = os.path.basename(path)
        parts = base[:-4].split("_") if base.startswith("tape_") and base.endswith(".npz") else []
        if symbol is None:
            symbol = str(z["symbol"]) if "symbol" in z.files else (parts[1] if len(parts) >= 3 else None)
        if date is None:
            date = str(z["date"]) if "date" in z.files else (parts[2] if len(parts) >= 3 else None)
        return cls(z["t"], z["oid"], z["price"], z["size"], z["buy"], symbol=symbol, date=date)


def load_lobster(path, date, symbol=None):
    """symbol: the ticker (default the <SYM> of LOBSTER's <SYM>_<date>_..._message_<k>.csv name)"""
    import pandas as pd

    df = pd.read_csv(path, names=["TIMESTAMP", "EVENT_TYPE", "ORDER_ID", "SIZE", "PRICE", "BUY_SELL_FLAG"])
    day = pd.Timestamp(date)
    start, end = day + pd.to_timedelta(OPEN), day + pd.to_timedelta(CLOSE)
    ts = start + pd.to_timedelta(df["TIMESTAMP"], "s") - pd.to_timedelta(OPEN)
    keep = ((ts >= start) & (ts < end)).to_numpy()
    t = (ts - day).to_numpy().astype("timedelta64[ns]").astype(np.int64)[keep]
    oid = df["ORDER_ID"].to_numpy().astype(np.int64)[keep]
    size = df["SIZE"].astype(int).to_numpy().astype(np.int64)[keep]
    price = (df["PRICE"].astype(float) / 100).astype(int).to_numpy().astype(np.int64)[keep]
    buy = (df["BUY_SELL_FLAG"].astype(int) == 1).to_numpy()[keep]
    order = np.argsort(t, kind="stable")
    if symbol is None:
        symbol = os.path.basename(path).split("_")[0] or None
    return Tape(t[order], oid[order], price[order], size[order], buy[order], symbol=symbol,
                date=str(day.date()))
