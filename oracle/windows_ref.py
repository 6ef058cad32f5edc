"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does). Pure-Python
restatement (event loop, small cases) of the Flink window aggregates computed on the device by
realtime-fraud-detection_amd/csrc/windows.hip.

Reference (fl/ = services/flink-jobs/src/main/java/com/frauddetection/):
  processUserVelocity: keyBy(userId), SlidingEventTimeWindows(5 min, 1 min)     fl/windows/WindowProcessor.java:36-48
  processMerchantPatterns: keyBy(merchantId), TumblingEventTimeWindows(1 h)     :54-66
  forBoundedOutOfOrderness(10 s) watermarks                                      :40-43, 58-61
  UserVelocityAggregateFunction.add / getResult / calculateVelocityScore         :256-352
  MerchantAggregateFunction.add / getResult / std-dev / calculateMerchantRiskScore :365-484
Flink semantics restated (flink-streaming-java 1.18, the job's pinned Flink; not vendored here):
  SlidingEventTimeWindows.assignWindows: starts = last start <= ts, stepping back by the slide while
    start > ts - size; TumblingEventTimeWindows: start = ts - ts mod size (offset 0);
  BoundedOutOfOrdernessWatermarks: watermark = max timestamp - lag - 1;
  EventTimeTrigger: a window fires when watermark >= end - 1; allowed lateness 0: an element whose
    windows are all past the watermark is dropped, windows receive only elements that arrive before
    they fire; a window with no elements never fires.
Micro-batch restatement (declared, DESIGN.md "Windows"): the watermark advances once per batch after the
batch's elements are assigned; flush = end of input (Flink emits MAX_WATERMARK: everything fires).
Declared deviations from the Java arithmetic: amounts are exact integer cents (totalAmount = cents/100),
the merchant std-dev is the exact-moment formula sqrt((n S2 - S1^2) / n^2) / 100 (Java: two-pass f64
mean / average of squared deviations; agrees to ~1e-15 relative, see java_stddev below). Transactions
with an unknown merchant (-1) are not aggregated by merchant.
PARITY UNPINNED: no JDK / Flink here and the reference has no tests or fixtures for these functions.
"""
from __future__ import annotations

import math

USER_SIZE, USER_SLIDE, MERCH_SIZE = 300_000, 60_000, 3_600_000


def velocity_score(cnt: int, cents: int, fraud: int, uniq_m: int) -> float:
    """calculateVelocityScore (WindowProcessor.java:327-351), amount thresholds on exact cents."""
    score = 0.0
    if cnt > 20:
        score += 0.4
    elif cnt > 10:
        score += 0.2
    elif cnt > 5:
        score += 0.1
    if cents > 1_000_000:
        score += 0.3
    elif cents > 500_000:
        score += 0.2
    elif cents > 100_000:
        score += 0.1
    rate = fraud / cnt if cnt > 0 else 0.0
    score += rate * 0.4
    div = uniq_m / cnt if cnt > 0 else 0.0
    if div < 0.2:
        score += 0.2
    return min(1.0, score)


def exact_stddev(cents_list) -> float:
    n = len(cents_list)
    if n < 2:
        return 0.0
    s1 = sum(cents_list)
    s2 = sum(c * c for c in cents_list)
    num = n * s2 - s1 * s1
    return math.sqrt(float(num) / (float(n) * float(n))) / 100.0


def java_stddev(amounts) -> float:
    """calculateStandardDeviation (WindowProcessor.java:447-457) as written (two-pass f64)."""
    if len(amounts) < 2:
        return 0.0
    mean = sum(amounts) / len(amounts)
    return math.sqrt(sum((a - mean) ** 2 for a in amounts) / len(amounts))


def merchant_risk(cnt: int, fraud_rate: float, avg: float, sd: float, uniq_u: int) -> float:
    """calculateMerchantRiskScore (WindowProcessor.java:459-483)."""
    score = 0.0
    score += fraud_rate * 0.5
    if cnt > 1000:
        score += 0.2
    elif cnt > 500:
        score += 0.1
    if avg > 0 and sd / avg > 2.0:
        score += 0.2
    div = uniq_u / cnt if cnt > 0 else 0.0
    if div < 0.1:
        score += 0.3
    return min(1.0, score)


class WindowOracle:
    """Events: dicts with key, ts, cents, merchant (-1 unknown), pm (255 null), fraud (bool),
    score (float, NaN null)."""

    def __init__(self, max_out_of_orderness_ms: int = 10_000):
        self.ooo = max_out_of_orderness_ms
        self.wm = None          # None = no watermark yet (Long.MIN_VALUE)
        self.max_seen = None
        self.events = []        # retained events, arrival order
        self.observed = False   # observe() since the last step (sharded: advance on the node-wide max)

    def observe(self, max_event_ts: int):
        """fd_windows_observe: the node-wide batch's largest event time (sharded runs)."""
        self.max_seen = max_event_ts if self.max_seen is None else max(self.max_seen, max_event_ts)
        self.observed = True

    def _fires(self, end: int, w_prev, w_new) -> bool:
        return (w_prev is None or end - 1 > w_prev) and end - 1 <= w_new

    def step(self, batch, flush: bool = False):
        """Add one micro-batch; returns (user windows, merchant windows) fired by it (lists of dicts)."""
        for e in batch:
            self.events.append(e)
            self.max_seen = e["ts"] if self.max_seen is None else max(self.max_seen, e["ts"])
        w_prev = self.wm
        w_new = w_prev
        if (batch or self.observed) and self.max_seen is not None:
            cand = self.max_seen - self.ooo - 1
            w_new = cand if w_new is None else max(w_new, cand)
        self.observed = False
        if flush and self.max_seen is not None:
            cand = self.max_seen + MERCH_SIZE
            w_new = cand if w_new is None else max(w_new, cand)
        if w_new == w_prev:
            return [], []
        self.wm = w_new
        uwin, mwin = {}, {}
        for e in self.events:                       # arrival order = Java add() order
            last = e["ts"] // USER_SLIDE
            for j in range(USER_SIZE // USER_SLIDE):
                m = last - j
                if self._fires(m * USER_SLIDE + USER_SIZE, w_prev, w_new):
                    uwin.setdefault((e["key"], m), []).append(e)
            if e["merchant"] >= 0:
                h = e["ts"] // MERCH_SIZE
                if self._fires(h * MERCH_SIZE + MERCH_SIZE, w_prev, w_new):
                    mwin.setdefault((e["merchant"], h), []).append(e)
        users = [self._user(k, m, evs) for (k, m), evs in uwin.items()]
        merchants = [self._merchant(mm, h, evs) for (mm, h), evs in mwin.items()]
        keep = w_new + 2 - USER_SIZE, w_new + 2 - MERCH_SIZE
        self.events = [e for e in self.events if e["ts"] >= min(keep)]  # retention (no-op semantically)
        return users, merchants

    @staticmethod
    def _common(evs):
        cnt = len(evs)
        cents = sum(e["cents"] for e in evs)
        fraud = sum(1 for e in evs if e["fraud"])
        high = sum(1 for e in evs if not math.isnan(e["score"]) and e["score"] > 0.7)
        pms = {e["pm"] for e in evs if e["pm"] != 255}
        first = last = 0
        for e in evs:                                # accumulator windowStart / windowEnd rule
            if first == 0 or e["ts"] < first:
                first = e["ts"]
            if e["ts"] > last:
                last = e["ts"]
        return cnt, cents, fraud, high, len(pms), first, last

    def _user(self, key, m, evs):
        cnt, cents, fraud, high, npm, first, last = self._common(evs)
        uniq_m = len({e["merchant"] for e in evs})
        total = cents / 100.0
        return dict(user_key=key, window_start=m * USER_SLIDE, window_end=m * USER_SLIDE + USER_SIZE,
                    first_ts=first, last_ts=last, count=cnt, fraud_count=fraud, high_risk_count=high,
                    unique_merchants=uniq_m, unique_payment_methods=npm, total_amount=total,
                    avg_amount=total / cnt, fraud_rate=fraud / cnt,
                    velocity_score=velocity_score(cnt, cents, fraud, uniq_m))

    def _merchant(self, merchant, h, evs):
        cnt, cents, fraud, high, npm, first, last = self._common(evs)
        uniq_u = len({e["key"] for e in evs})
        fcents = sum(e["cents"] for e in evs if e["fraud"])
        total = cents / 100.0
        avg = total / cnt
        rate = fraud / cnt
        sd = exact_stddev([e["cents"] for e in evs])
        return dict(merchant=merchant, window_start=h * MERCH_SIZE, window_end=h * MERCH_SIZE + MERCH_SIZE,
                    first_ts=first, last_ts=last, count=cnt, fraud_count=fraud, high_risk_count=high,
                    unique_users=uniq_u, unique_payment_methods=npm, total_amount=total,
                    fraud_amount=fcents / 100.0, avg_amount=avg, fraud_rate=rate, amount_stddev=sd,
                    risk_score=merchant_risk(cnt, rate, avg, sd, uniq_u),
                    # the exact moments (fd_merchant_window's merge fields)
                    cents=cents, fraud_cents=fcents, s2=sum(e["cents"] * e["cents"] for e in evs),
                    pm_set={e["pm"] for e in evs if e["pm"] != 255})
