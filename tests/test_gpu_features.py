"""GPU parity of the feature kernels (fd_features_*) against the CPU oracle on the same seeded stream:
bridged raw features bit-exact (counts are integers, sums integer cents / 100.0), scoring vectors
bit-exact except transcendental slots, which may differ by at most 1 f32 ulp (device log1p vs libm),
state carried across micro-batches, both window modes, repeat cards inside a batch (arrival order),
unknown users / merchants."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from oracle import velocity_ref as VR
from oracle.features_c import OracleFeatureState

pytestmark = pytest.mark.gpu


def _pair(engine, mode, n_users, n_merch=200, K=8, cap=None):
    pop = synth.population(n_users, n_merch, seed=n_users)
    U, M = pop["users"], pop["merchants"]
    cap = cap or 4 * n_users + 4096
    engine.state_init(cap, mode, K)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    orc = OracleFeatureState(cap, mode, K)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    return pop, orc


def _slice(tx, a, b):
    return {k: v[a:b] for k, v in tx.items()}


def _check_vectors(vec, rvec):
    same = vec == rvec
    if not same.all():
        bad = np.argwhere(~same)
        assert set(bad[:, 1].tolist()) <= {1}, f"non-transcendental slots differ: {sorted(set(bad[:, 1].tolist()))}"
        ulps = np.abs(vec.view(np.int32)[~same].astype(np.int64) - rvec.view(np.int32)[~same].astype(np.int64))
        assert ulps.max() <= 1


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n_users,rate", [(200, 0.5), (20000, 50.0)])  # dense repeats / mostly distinct
def test_features_match_oracle_across_batches(engine, mode, n_users, rate):
    pop, orc = _pair(engine, mode, n_users)
    tx = synth.txn_stream(pop, 24000, seed=3, rate_per_s=rate, unknown_user_frac=0.03, unknown_merchant_frac=0.03)
    for a, b in [(0, 1), (1, 257), (257, 8000), (8000, 24000)]:  # ragged micro-batches, state carried
        part = _slice(tx, a, b)
        vec, raw = engine.features(part, want_raw=True)
        rraw, rvec = orc.run(part)
        np.testing.assert_array_equal(raw, rraw)
        _check_vectors(vec, rvec)
    info = engine.state_info()
    assert info["cards"] >= n_users


def test_small_stream_against_python_chain(engine):
    """The pinned chain itself (Java restatement -> FeatureProcessor restatement) on a small stream."""
    pop = synth.population(60, 20, seed=9)
    U, M = pop["users"], pop["merchants"]
    engine.state_init(1024, 0, 1)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    py = VR.FeatureState(0)
    py.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    py.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    tx = synth.txn_stream(pop, 600, seed=10, rate_per_s=0.2)
    vec, raw = engine.features(tx, want_raw=True)
    rraw = py.run(tx)
    np.testing.assert_array_equal(raw, rraw)
    _check_vectors(vec, VR.vectors(rraw).astype(np.float32))


def test_table_full_is_reported(engine):
    engine.state_init(8, 0, 1)
    pop = synth.population(4, 2, seed=1)
    tx = synth.txn_stream(pop, 64, seed=2, unknown_user_frac=1.0)  # 64 distinct unknown cards > 8 slots
    with pytest.raises(Exception) as ei:
        engine.features(tx)
    assert "card table full" in str(ei.value)
