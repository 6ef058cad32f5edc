"""The seeded stream generator of the benches' warm-state workload (fdengine/synth_gpu.py), run on the CPU device:
SURVEY §8(d)'s shape — cards drawn in proportion to txn_frequency = floor(Gamma(2, 2)) + 1 per day
(simulator.py:229), Poisson arrivals at sum(freq) / 86 400 s, the simulator's per-transaction distributions — and the
warm-history driver (event-time bounds, the kept rows of a card subset)."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "realtime-fraud-detection_amd"))

torch = pytest.importorskip("torch")

from fdengine import synth_gpu as SG  # noqa: E402
from fdengine._native import TXN_FIELDS  # noqa: E402


@pytest.fixture(scope="module")
def pop():
    attrs = SG.population_attrs(200_000, seed=42, chunk=1 << 16, threads=4)
    return attrs, SG.CardPopulation(attrs, torch.device("cpu"))


def test_frequency_distribution(pop):
    attrs, _ = pop
    f = attrs["txn_frequency"].astype(np.float64)
    assert f.min() >= 1
    # floor(Gamma(2, 2)) + 1: mean E[floor(X)] + 1 ~ 4.5, P(freq == 1) = P(X < 1) = 1 - 1.5 e^-0.5
    assert abs(f.mean() - 4.5) < 0.05
    assert abs((f == 1).mean() - (1 - 1.5 * np.exp(-0.5))) < 0.01


def test_draw_is_frequency_weighted(pop):
    attrs, p = pop
    g = torch.Generator().manual_seed(1)
    c = p.draw(400_000, g).numpy()
    f = attrs["txn_frequency"].astype(np.float64)
    want = (f * f).sum() / f.sum()  # a transaction's card frequency: size-biased
    assert abs(f[c].mean() - want) / want < 0.01
    assert abs(p.rate_per_s - f.sum() / 86400.0) < 1e-9


def test_stream_fields(pop):
    attrs, p = pop
    gen = SG.StreamGen(p, 5000, seed=3, t0_ms=1_000_000, rate_per_s=p.rate_per_s)
    a = gen.next(100_000)
    b = gen.next(100_000)
    ts = torch.cat([a["ts_ms"], b["ts_ms"]]).numpy()
    assert (np.diff(ts) >= 0).all() and ts[0] >= 1_000_000
    gap = (ts[-1] - ts[0]) / (len(ts) - 1)
    assert abs(gap - 1000.0 / p.rate_per_s) / (1000.0 / p.rate_per_s) < 0.02
    unknown = (a["card_idx"] < 0).numpy()
    assert abs(unknown.mean() - 0.01) < 0.002
    keys = a["card_key"].numpy().view(np.uint64)
    known = ~unknown
    assert (keys[known] == attrs["key"][a["card_idx"].numpy()[known]]).all()
    assert (keys >> np.uint64(63) == 1).all()
    cents = a["amount_cents"].numpy()
    assert cents.min() >= 100 and (a["merchant"].numpy() == -1).mean() < 0.01
    assert abs(a["is_fraud"].numpy().mean() - 0.055) < 0.005
    assert set(np.unique(a["ip_class"].numpy())) == {1, 2}
    assert (a["device_fp"].numpy() != 0).all()


class _Recorder:
    """stands in for FraudEngine.features_device: records the micro-batches it is given"""

    def __init__(self):
        self.batches = []

    def features_device(self, ptrs, n, vec_ptr, raw_ptr=0):
        self.batches.append(n)


def test_warm_history_bounds_and_kept_rows(pop, monkeypatch):
    attrs, p = pop
    seen = []
    orig = SG.StreamGen.next

    def spy(self, n):
        b = orig(self, n)
        seen.append({f: b[f].clone() for f in TXN_FIELDS})
        return b

    monkeypatch.setattr(SG.StreamGen, "next", spy)
    keep = torch.from_numpy(attrs["key"][:5000].view(np.int64))
    rec = _Recorder()
    t0, t1 = 5_000_000, 5_000_000 + 3_600_000 * 6
    out = SG.warm_history(rec, p, 5000, seed=9, t_start_ms=t0, t_end_ms=t1, chunk=1 << 16, keep_keys=keep)
    allts = torch.cat([s["ts_ms"] for s in seen]).numpy()
    m = int((allts < t1).sum())
    assert out["transactions"] == m == sum(rec.batches)
    assert abs(m - p.rate_per_s * 6 * 3600) < 5 * np.sqrt(p.rate_per_s * 6 * 3600)
    allk = torch.cat([s["card_key"] for s in seen]).numpy()[:m]
    hit = np.isin(allk, attrs["key"][:5000].view(np.int64))
    rows = out["rows"]
    assert len(rows["card_key"]) == hit.sum() > 0
    assert (rows["card_key"] == allk[hit].view(np.uint64)).all()
    assert (rows["ts_ms"] == allts[:m][hit]).all() and rows["card_key"].dtype == np.uint64
