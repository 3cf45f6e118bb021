"""The ExternalFileOracle's fundamental series for the hist_fund_* configurations.

util/oracle/ExternalFileOracle.py:21-35 loads, per symbol, a pandas Series of fundamental values
indexed by timestamp: the mid prices util/formatting/mid_price_from_orderbook.py writes
((ask_price_1 + bid_price_1) / 2 per order-book timestamp).  libmxa takes the series as two
arrays (mxa_create_hist): ns since midnight of the simulated date, and the float values.
"""
import numpy as np


class FundamentalSeries:
    def __init__(self, t_ns, values):
        self.t = np.ascontiguousarray(t_ns, dtype=np.int64)
        self.v = np.ascontiguousarray(values, dtype=np.float64)
        if self.t.ndim != 1 or self.t.shape != self.v.shape or not len(self.t):
            raise ValueError("a fundamental series needs matching non-empty time and value arrays")
        if (np.diff(self.t) < 0).any():
            raise ValueError("fundamental series times must be sorted")

    def __len__(self):
        return len(self.t)

    @property
    def r_bar(self):
        """oracle.fundamentals[symbol].values[0] (config/hist_fund_value.py:80)"""
        return float(self.v[0])

    @classmethod
    def from_pandas(cls, series, date):
        """a pandas Series indexed by Timestamps (what the reference's oracle reads)"""
        import pandas as pd
        mid = int(pd.Timestamp(date).value)
        return cls(series.index.asi8 - mid, series.to_numpy(dtype=np.float64))

    @classmethod
    def from_level1_csv(cls, path, date):
        """mid prices of a level-1 order-book CSV with columns time, ask_price_1, bid_price_1 (the
        reference ships data/JPM_2019-06-28_34200_57571_orderbook_1.csv); timestamps with an empty
        side have no mid and are dropped"""
        import pandas as pd
        df = pd.read_csv(path)
        mid = (df["ask_price_1"] + df["bid_price_1"]) / 2
        s = pd.Series(mid.to_numpy(dtype=np.float64), index=pd.DatetimeIndex(pd.to_datetime(df["time"]))).dropna()
        return cls.from_pandas(s, date)

    @classmethod
    def load(cls, path):
        """an npz with arrays t (ns since midnight) and v"""
        z = np.load(path, allow_pickle=False)
        return cls(z["t"], z["v"])
