"""CPU: the feature-half oracle. The C restatement (oracle_features.c, used at scale) must equal the
pure-Python chain (velocity_ref.py -> features_ref.py, whose FeatureProcessor half is pinned to the
reference by golden vectors) on the same seeded stream, in both window modes, including unknown
users / merchants, repeat cards inside a batch and TTL expiry."""
import numpy as np
import pytest

from fdengine import synth
from oracle import velocity_ref as VR
from oracle.features_c import OracleFeatureState, vector_from_raw


def _setup(mode, n_users=300, n_txn=3000, rate=0.5, seed=5):
    pop = synth.population(n_users, 50, seed=seed)
    tx = synth.txn_stream(pop, n_txn, seed=seed + 1, rate_per_s=rate, unknown_user_frac=0.05,
                          unknown_merchant_frac=0.05)
    U, M = pop["users"], pop["merchants"]
    py = VR.FeatureState(window_mode=mode, ring_k=8)
    py.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    py.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    c = OracleFeatureState(4096, window_mode=mode, ring_k=8)
    c.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    c.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    return tx, py, c


@pytest.mark.parametrize("mode", [0, 1])
def test_c_oracle_equals_python_chain(mode):
    tx, py, c = _setup(mode)
    raw_py = py.run(tx)
    raw_c, vec_c = c.run(tx)
    np.testing.assert_array_equal(raw_c, raw_py)
    vec_py = VR.vectors(raw_py)
    np.testing.assert_array_equal(vec_c, vec_py.astype(np.float32))
    # the stream exercises what it should
    assert (raw_py[:, 10] > 0).mean() > 0.2         # cards with live velocity state
    assert np.isnan(raw_py[:, 8]).any()             # unknown users
    assert (raw_py[:, 5] == 0.1).any()              # unknown merchants
    assert (raw_py[:, 6] == 0).any() and (raw_py[:, 6] == 1).any()


def test_redis_compat_windows_are_identical_and_expire():
    tx, py, c = _setup(0, n_users=50, n_txn=2000, rate=0.02)  # sparse: many > 1 h gaps
    raw, _ = c.run(tx)
    assert (raw[:, 9] == raw[:, 10]).all() and (raw[:, 10] == raw[:, 11]).all()
    assert (raw[:, 12] == raw[:, 13]).all()
    # some card saw a gap > 1 h and reset
    keys = tx["card_key"]
    last = {}
    resets = 0
    for i, k in enumerate(keys):
        if k in last and tx["ts_ms"][i] - last[k] > 3_600_000:
            assert raw[i, 10] == 0
            resets += 1
        last[k] = tx["ts_ms"][i]
    assert resets > 10


def test_sliding_windows_nested():
    tx, py, c = _setup(1, n_users=40, n_txn=3000, rate=0.05)
    raw, _ = c.run(tx)
    assert (raw[:, 9] <= raw[:, 10]).all() and (raw[:, 10] <= raw[:, 11]).all()
    assert (raw[:, 11] <= 8).all()  # ring of K = 8 events bounds the 24 h window
    assert (raw[:, 12] <= raw[:, 13] + 1e-9).all()


def test_vector_from_raw_matches_python():
    tx, py, c = _setup(0, n_txn=500)
    raw = py.run(tx)
    np.testing.assert_array_equal(vector_from_raw(raw), VR.vectors(raw).astype(np.float32))
