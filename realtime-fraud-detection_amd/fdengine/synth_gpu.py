"""Seeded transaction streams generated on the GPU, for benches and tests at 10^8 cards (no network, no dataset).

SURVEY §8(d)'s stream: each card transacts txn_frequency ~ floor(Gamma(2, 2)) + 1 times a day
(services/data-simulator/src/main/python/simulator.py:229), so the node's arrivals are a Poisson process of rate
sum(txn_frequency) / 86 400 s and each arrival's card is drawn with probability proportional to its frequency
(the simulator's per-user draw, simulator.py:302, weighted by activity). The per-transaction fields follow
synth._txn_stream_indexed (simulator.py:298-374): amount = max(1, avg * N(1, .3) * N(1, .2)) in cents, the
card-testing / account-takeover / synthetic fraud patterns (:107-152), 1 % unknown users, 0.5 % unknown merchants,
5 % private IPs.

Warm state: `warm_history` runs `hours` of that stream (about 4.5 transactions per card per day, 450 M at 10^8
cards over 24 h) through the engine's own feature path before a benchmark or test, so the 5 min / 1 h / 24 h
windows hold the events the reference's per-user state would (RedisService.java:178-207), and optionally returns
the history rows of a given set of cards, so a CPU oracle can rebuild exactly those cards' state (per-card state is
independent of other cards).

Everything here is test / bench input generation (torch on the GPU); the scoring path never imports it.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ._native import TXN_FIELDS

DAY_S = 86400.0
_SIGN = -(1 << 63)  # the high bit of a u64 card key (synth._nonzero_u64 / card_keys set it)


class CardPopulation:
    """Device copies of a card population (synth.card_attrs fields + txn_frequency) and a frequency-weighted
    sampler over it: cards are grouped by frequency (a stable sort), a draw picks a group with probability
    f * |group f| / sum(freq), then a card of the group uniformly."""

    def __init__(self, attrs: dict, device):
        import torch
        self.torch, self.device = torch, device
        self.n = len(attrs["key"])
        self.key = torch.from_numpy(np.ascontiguousarray(attrs["key"]).view(np.int64)).to(device)
        self.fp = torch.from_numpy(np.ascontiguousarray(attrs["device_fp"]).view(np.int64)).to(device)
        self.avg = torch.from_numpy(np.ascontiguousarray(attrs["avg_amount"], np.float64)).to(device)
        freq = np.asarray(attrs["txn_frequency"], np.int32)
        self.txns_per_day = float(freq.sum(dtype=np.int64))
        f = torch.from_numpy(freq).to(device)
        self.order = torch.sort(f, stable=True).indices
        vals, counts = torch.unique_consecutive(f[self.order], return_counts=True)
        w = vals.double() * counts.double()
        self.cum = torch.cumsum(w, 0) / w.sum()
        self.counts = counts
        self.offsets = torch.cumsum(counts, 0) - counts
        del f

    @property
    def rate_per_s(self) -> float:
        return self.txns_per_day / DAY_S

    def draw(self, n: int, gen):
        t = self.torch
        u = t.rand(n, dtype=t.float64, device=self.device, generator=gen)
        g = t.searchsorted(self.cum, u, right=True).clamp_(max=len(self.cum) - 1)
        cnt = self.counts[g]
        v = t.rand(n, dtype=t.float64, device=self.device, generator=gen)
        k = t.minimum((v * cnt.double()).long(), cnt - 1)
        return self.order[self.offsets[g] + k]


class StreamGen:
    """Arrival-ordered transactions over a CardPopulation: Poisson arrivals at `rate_per_s` from `t0_ms`."""

    def __init__(self, pop: CardPopulation, n_merchants: int, seed: int, t0_ms: int, rate_per_s: float,
                 unknown_user_frac: float = 0.01, unknown_merchant_frac: float = 0.005):
        import torch
        self.torch, self.pop = torch, pop
        self.dev = pop.device
        self.gen = torch.Generator(device=self.dev)
        self.gen.manual_seed(int(seed))
        self.nm = int(n_merchants)
        self.mean_gap_ms = 1000.0 / float(rate_per_s)
        self.clock = torch.full((1,), float(t0_ms), dtype=torch.float64, device=self.dev)  # continuous time (ms)
        self.uu, self.um = unknown_user_frac, unknown_merchant_frac

    def _u(self, n):
        t = self.torch
        return t.rand(n, dtype=t.float64, device=self.dev, generator=self.gen)

    def _keys(self, n):
        t = self.torch
        return t.randint(1, (1 << 62), (n,), dtype=t.int64, device=self.dev, generator=self.gen) | _SIGN

    def next(self, n: int) -> dict:
        """n transactions (device tensors of the TXN_FIELDS dtypes, plus card_idx: the population index, -1 for an
        unknown user, and is_fraud)."""
        t, p, g = self.torch, self.pop, self.gen
        gaps = t.empty(n, dtype=t.float64, device=self.dev).exponential_(1.0 / self.mean_gap_ms, generator=g)
        clock = self.clock + t.cumsum(gaps, 0)
        self.clock = clock[-1:].clone()
        ts = t.floor(clock).long()
        c = p.draw(n, g)
        unknown = self._u(n) < self.uu
        key = t.where(unknown, self._keys(n), p.key[c])
        merchant = t.randint(0, self.nm, (n,), dtype=t.int32, device=self.dev, generator=g)
        merchant = t.where(self._u(n) < self.um, t.full_like(merchant, -1), merchant)
        base = p.avg[c] * (1.0 + 0.3 * t.randn(n, dtype=t.float64, device=self.dev, generator=g)) \
            * (1.0 + 0.2 * t.randn(n, dtype=t.float64, device=self.dev, generator=g))
        cents = t.clamp(t.round(base * 100.0), min=100.0)
        roll = self._u(n)
        testing = roll < 0.02
        takeover = (roll >= 0.02) & (roll < 0.03)
        synthetic = (roll >= 0.03) & (roll < 0.035)
        cents = t.where(testing, t.round((1.0 + 4.0 * self._u(n)) * 100.0), cents)
        cents = t.where(synthetic, t.round((1000.0 + 4000.0 * self._u(n)) * 100.0), cents)
        pick = t.randint(0, 3, (n,), device=self.dev, generator=g)
        fps = p.fp[c]
        dfp = fps.gather(1, pick[:, None]).squeeze(1)
        dfp = t.where(dfp == 0, fps[:, 0], dfp)
        dfp = t.where(takeover, self._keys(n), dfp)
        ip = t.where(self._u(n) < 0.05, 1, 2).to(t.uint8)
        ff = t.full((n,), 255, dtype=t.uint8, device=self.dev)
        return {"card_key": key, "ts_ms": ts, "amount_cents": cents.long(), "merchant": merchant, "device_fp": dfp,
                "ip_class": ip, "hour": ff, "weekend": ff.clone(), "card_idx": t.where(unknown, -1, c),
                "is_fraud": roll < 0.055}


def warm_history(eng, pop: CardPopulation, n_merchants: int, seed: int, t_start_ms: int, t_end_ms: int,
                 chunk: int = 1 << 20, keep_keys=None, vec_scratch=None) -> dict:
    """Drive the stream of `pop` over event time [t_start_ms, t_end_ms) through the engine's feature path
    (fd_features_device: card state read and updated, vectors discarded), in micro-batches of `chunk`.
    keep_keys: optional device tensor (int64 view of u64 card keys): the rows of those cards are returned
    (host arrays, arrival order) for an oracle to replay. -> {"transactions": count, "rows": dict or None,
    "batches": count}"""
    import torch
    gen = StreamGen(pop, n_merchants, seed, t_start_ms, pop.rate_per_s)
    vec = vec_scratch if vec_scratch is not None else torch.empty((chunk, 64), dtype=torch.float32,
                                                                  device=pop.device)
    kept, total, batches = [], 0, 0
    sorted_keep = torch.unique(keep_keys) if keep_keys is not None else None
    while True:
        b = gen.next(chunk)
        last = int(b["ts_ms"][-1].item())  # one sync per micro-batch of history (~1 M transactions)
        m = chunk
        if last >= t_end_ms:
            m = int(torch.searchsorted(b["ts_ms"], torch.tensor([t_end_ms], device=pop.device)).item())
        if m:
            cols = {f: b[f][:m].contiguous() for f in TXN_FIELDS}
            eng.features_device({f: cols[f].data_ptr() for f in TXN_FIELDS}, m, vec.data_ptr())
            if sorted_keep is not None:
                hit = torch.isin(cols["card_key"], sorted_keep)
                kept.append({f: cols[f][hit] for f in TXN_FIELDS})
            total += m
            batches += 1
        if m < chunk:
            break
    rows = None
    if sorted_keep is not None:
        rows = {f: torch.cat([k[f] for k in kept]).cpu().numpy() if kept else np.zeros(0) for f in TXN_FIELDS}
        rows = host_columns(rows)
    return {"transactions": total, "rows": rows, "batches": batches}


_HOST_DTYPES = {"card_key": np.uint64, "ts_ms": np.int64, "amount_cents": np.int64, "merchant": np.int32,
                "device_fp": np.uint64, "ip_class": np.uint8, "hour": np.uint8, "weekend": np.uint8}


def host_columns(cols: dict) -> dict:
    """Device or int64-viewed columns -> host arrays in the engine's / oracle's dtypes (keys as u64)."""
    out = {}
    for f in TXN_FIELDS:
        a = cols[f]
        if hasattr(a, "cpu"):
            a = a.cpu().numpy()
        a = np.ascontiguousarray(a)
        dt = _HOST_DTYPES[f]
        out[f] = a.view(dt) if a.dtype.itemsize == np.dtype(dt).itemsize and a.dtype != dt else a.astype(dt)
    return out


def occupancy(raw: np.ndarray) -> dict:
    """Mean prior events in the 5 min / 1 h / 24 h windows per scored transaction, from the raw bridged features
    (oracle.velocity_ref.RAW_COLUMNS 9-11: velocity_5min / 1hour / 24hour counts)."""
    r = np.asarray(raw)
    return {"mean_events_5m": round(float(r[:, 9].mean()), 4), "mean_events_1h": round(float(r[:, 10].mean()), 4),
            "mean_events_24h": round(float(r[:, 11].mean()), 4),
            "frac_with_24h_history": round(float((r[:, 11] > 0).mean()), 4)}


def population_attrs(n_cards: int, seed: int = 42, chunk: int = 1 << 23, threads: int = 8) -> dict:
    """synth.card_attrs of cards 0..n_cards-1 (with txn_frequency), computed in chunks on a thread pool."""
    from concurrent.futures import ThreadPoolExecutor

    from . import synth
    bounds = [(a, min(n_cards, a + chunk)) for a in range(0, n_cards, chunk)]
    with ThreadPoolExecutor(max(1, threads)) as ex:
        parts = list(ex.map(lambda ab: synth.card_attrs(np.arange(ab[0], ab[1], dtype=np.int64), seed), bounds))
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def subset(attrs: dict, mask: Optional[np.ndarray]) -> dict:
    return attrs if mask is None else {k: v[mask] for k, v in attrs.items()}


_DEV_DTYPES = {"card_key": "int64", "ts_ms": "int64", "amount_cents": "int64", "merchant": "int32",
               "device_fp": "int64", "ip_class": "uint8", "hour": "uint8", "weekend": "uint8"}
T_HISTORY_MS = 1_757_030_400_000  # 2025-09-05 00:00 UTC: where the synthetic history starts


def warm_workload(eng, device, n_cards: int, rank: int, world: int, n_batches: int, batch: int, hours: float = 24.0,
                  keep_batches: int = 2, host_batches: int = 0, n_merchants: int = 5000, seed: int = 42,
                  t_history_ms: int = T_HISTORY_MS, log=None, gather_keys=None) -> dict:
    """The warm-state workload of BASELINE config 4 (and its GPU test) on one rank of `world`:

    1. the population of n_cards (synth.card_attrs, hash-derived from the card id) — this rank's owned cards are
       loaded into the engine (fd_state_load_users); the merchant table must be loaded already;
    2. the rank's ingest stream, resident in HBM: n_batches micro-batches of `batch` transactions drawn over ALL
       cards, starting at t_history + hours, at the node's rate / world (the ranks' streams superpose to the
       node's Poisson stream);
    3. `hours` of history over the owned cards, [t_history, t_history + hours), through the engine's feature path
       (warm_history), so the first resident batch meets populated windows;
    4. host copies of the first keep_batches resident batches, the history rows of the cards they touch and those
       cards' profiles (an oracle replays exactly that: per-card state is independent), and host_batches more
       micro-batches after the resident ones (host memory only: the PCIe-inclusive latency line).
    gather_keys (world > 1): a collective mapping this rank's kept card keys (int64 device tensor) to every rank's
    (concatenated): the history rows kept are then those of the OWNED cards any rank's kept batches touch — the
    rows an oracle of the whole node needs (a card's history lives on its owner only).
    -> dict of the above plus counts and timings."""
    import time

    import torch

    from .engine import shard_of
    say = log or (lambda *a: None)
    t = time.time()
    attrs = population_attrs(n_cards, seed)
    own_mask = None if world == 1 else shard_of(attrs["key"], world) == rank
    own = subset(attrs, own_mask)
    eng.load_users(own["key"], own["avg_amount"], own["account_age_days"], own["device_fp"])
    n_owned = len(own["key"])
    t_pop = time.time() - t
    pop_all = CardPopulation(attrs, device)
    pop_own = pop_all if own_mask is None else CardPopulation(own, device)
    del own
    T0 = t_history_ms + int(round(hours * 3_600_000))
    gen = StreamGen(pop_all, n_merchants, seed=200 + rank, t0_ms=T0, rate_per_s=pop_all.rate_per_s / world)
    total = n_batches * batch
    resident = {f: torch.empty(total, dtype=getattr(torch, _DEV_DTYPES[f]), device=device) for f in TXN_FIELDS}
    card_idx = torch.empty(total, dtype=torch.int64, device=device)
    step = 1 << 20
    for a in range(0, total, step):
        m = min(step, total - a)
        b = gen.next(m)
        for f in TXN_FIELDS:
            resident[f][a:a + m] = b[f]
        card_idx[a:a + m] = b["card_idx"]
    extra = []
    for _ in range(host_batches):
        b = gen.next(batch)
        extra.append({f: b[f].cpu() for f in TXN_FIELDS})
    kr = min(total, keep_batches * batch)
    keep_keys = resident["card_key"][:kr] if kr else None
    if keep_keys is not None and gather_keys is not None:
        keep_keys = gather_keys(keep_keys.contiguous())
    t = time.time()
    hist = warm_history(eng, pop_own, n_merchants, seed=900 + rank, t_start_ms=t_history_ms, t_end_ms=T0,
                        keep_keys=keep_keys)
    torch.cuda.synchronize(device) if device.type == "cuda" else None
    t_hist = time.time() - t
    head = host_columns({f: resident[f][:kr] for f in TXN_FIELDS})
    idx = card_idx[:kr].cpu().numpy()
    known = np.unique(idx[idx >= 0])
    profiles = {k: v[known] for k, v in attrs.items()}
    say(f"[warm] population {n_cards} ({n_owned} owned) {t_pop:.1f}s; history {hours:g} h = {hist['transactions']} "
        f"transactions in {hist['batches']} micro-batches {t_hist:.1f}s; resident {n_batches} x {batch}")
    return {"resident": resident, "head": head, "head_card_idx": idx, "history_rows": hist["rows"],
            "profiles": profiles, "n_owned": n_owned, "history_transactions": hist["transactions"],
            "history_hours": hours, "history_seconds": round(t_hist, 2), "population_seconds": round(t_pop, 2),
            "rate_per_s_node": pop_all.rate_per_s, "t_stream_ms": T0, "host_batches": extra}
