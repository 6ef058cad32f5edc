"""CPU: the feature-map oracle's known answers (hand-computed rows from FeatureExtractor.java /
TransactionProcessor.java / FeatureEnrichmentProcessor.java) and helpers."""
import math

import numpy as np

from oracle import fmap_ref as R


def _row(**over):
    raw = np.zeros((1, 16))
    raw[0, 0] = 100.0
    raw[0, 1] = math.log(101.0)
    raw[0, 2] = 23
    raw[0, 3] = 7
    raw[0, 4] = 1
    raw[0, 5] = 0.02
    raw[0, 6] = 1  # new device
    raw[0, 7] = 0.3
    raw[0, 8] = 10.0  # user avg -> ratio 10
    raw[0, 9], raw[0, 10], raw[0, 11] = 6, 21, 30
    raw[0, 12], raw[0, 13] = 500.0, 900.0
    raw[0, 14] = 0.9
    raw[0, 15] = 3  # account age days
    for k, v in over.items():
        raw[0, int(k[1:])] = v
    tx = {"card_key": np.array([7], np.uint64), "ts_ms": np.array([86400000 * 31], np.int64),
          "amount_cents": np.array([10000], np.int64), "merchant": np.array([0], np.int32),
          "device_fp": np.array([5], np.uint64), "ip_class": np.array([2], np.uint8),
          "hour": np.array([23], np.uint8), "weekend": np.array([255], np.uint8)}
    return tx, raw


def test_known_answer_high_risk_row():
    tx, raw = _row()
    users = {7: {"risk_score": 0.4, "kyc_status": 1, "verified": 0, "pref_start": 8, "pref_end": 20,
                 "weekend_activity": 0.2, "online_preference": 0.6, "intl_preference": 0.05, "txn_frequency": 3,
                 "has_patterns": 1}}
    merchants = {"fraud_rate": np.array([0.02]), "risk_multiplier": np.array([0.9])}
    mext = {"avg_amount": np.array([40.0]), "risk_level": np.array([2], np.uint8), "blacklisted": np.array([0], np.uint8),
            "category": np.array([5], np.uint8), "high_risk_category": np.array([1], np.uint8),
            "open_hour": np.array([9], np.uint8), "close_hour": np.array([21], np.uint8),
            "suspicious_name": np.array([1], np.uint8)}
    pay = np.zeros(256, np.uint8)
    pay[4] = 1
    ref = np.zeros(256, np.uint8)
    ctx = {"payment_method": np.array([4], np.uint8), "fraud_score": np.array([0.5])}
    fm, rules = R.feature_map(tx, ctx, raw, np.array([250.0]), users, merchants, mext, pay, ref)
    f = dict(zip(R.NAMES, fm[0]))
    assert f["is_round_amount"] == 1 and f["is_round_10"] == 1 and f["is_round_100"] == 1
    assert f["amount_to_user_avg_ratio"] == 10.0 and f["is_large_for_user"] == 1
    assert f["amount_to_merchant_avg_ratio"] == 2.5 and f["is_large_for_merchant"] == 1
    assert f["amount_category"] == 2  # medium: 100 <= amount < 1000
    assert f["day_of_month"] == 1  # 1970-02-01
    assert f["time_period"] == 3 and f["is_night_time"] == 1 and f["in_user_preferred_time"] == 0
    assert f["is_very_new_account"] == 1 and f["kyc_status"] == 1 and f["is_kyc_verified"] == 0
    assert f["within_merchant_hours"] == 0 and f["suspicious_merchant_name"] == 1
    assert f["high_velocity_5min"] == 1 and f["high_velocity_1hour"] == 1 and f["velocity_5min_amount"] == 250.0
    assert f["is_high_risk_payment"] == 1 and f["transaction_type"] == R.UNKNOWN
    assert math.isnan(f["latitude"]) and f["has_geolocation"] == 0 and math.isnan(f["suspicious_user_agent"])
    # FeatureEnrichmentProcessor: amount .3+.1 ; temporal .2+.15+.1 ; user .4+.3+.4*.5 ;
    # merchant .3+.02*2+.2+.15 ; velocity .6+.4+.2+.15 ; device .3+.3 -> weighted .7505 ; combined with .5
    fb = 0.0
    fb += (0.3 + 0.1) * 0.2
    fb += (0.2 + 0.15 + 0.1) * 0.1
    fb += (0.4 + 0.3 + 0.4 * 0.5) * 0.25
    fb += (0.3 + 0.02 * 2.0 + 0.2 + 0.15) * 0.2
    fb += (0.6 + 0.4 + 0.2 + 0.15) * 0.15
    fb += (0.3 + 0.3) * 0.1
    assert abs(rules["fe_score"][0] - ((0.5 * 0.6) + (fb * 0.4))) < 1e-15
    assert rules["fe_risk"][0] == R.MEDIUM and rules["fe_decision"][0] == R.REVIEW
    # TransactionProcessor: .25 + (.08+.1+.15) + (.2+.15) + (.15+.1+.05+.1) = 1.33 -> 1.0 -> DECLINE
    assert rules["tp_score"][0] == 1.0 and rules["tp_decision"][0] == R.DECLINE and rules["tp_risk"][0] == R.CRITICAL


def test_unknown_user_and_merchant_defaults():
    tx, raw = _row(r8=float("nan"), r15=0)
    tx["merchant"][0] = -1
    merchants = {"fraud_rate": np.array([0.02]), "risk_multiplier": np.array([0.9])}
    fm, rules = R.feature_map(tx, None, raw, np.array([0.0]), {}, merchants, None, np.zeros(256, np.uint8),
                              np.zeros(256, np.uint8))
    f = dict(zip(R.NAMES, fm[0]))
    assert (f["user_risk_score"], f["is_new_account"], f["kyc_status"]) == (0.8, 1.0, R.UNKNOWN)
    assert (f["merchant_fraud_rate"], f["merchant_risk_multiplier"], f["merchant_category"]) == (0.1, 2.0, R.UNKNOWN)
    assert math.isnan(f["within_merchant_hours"]) and math.isnan(f["amount_to_user_avg_ratio"])
    # minimal profiles: user .5*.2 + .15 ; merchant medium .1 ; unusual hour .05 -> .4 -> APPROVE / LOW
    assert abs(rules["tp_score"][0] - 0.4) < 1e-12 and rules["tp_decision"][0] == R.APPROVE


def test_day_of_month():
    assert R.day_of_month(0) == 1 and R.day_of_month(59) == 1 and R.day_of_month(-1) == 31
    assert R.day_of_month(20332) == 1  # 2025-09-01
