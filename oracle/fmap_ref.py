"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's cpu_baseline may import it; the product
never does). Pure-Python restatement (row loop, small cases) of the full FeatureExtractor feature map and
the Flink rule scores computed by realtime-fraud-detection_amd/csrc/features.hip feat_ext_kernel.

Reference (fl/ = services/flink-jobs/src/main/java/com/frauddetection/):
  FeatureExtractor.extractAllFeatures + extractors      fl/features/FeatureExtractor.java:50-493
  feature names / order                                 fl/features/FeatureStore.java:325-365
  FeatureEnrichmentProcessor score + updateRiskLevel    fl/processors/FeatureEnrichmentProcessor.java:80-93,122-367
  TransactionProcessor basic features, rules, decision  fl/processors/TransactionProcessor.java:143-473
  minimal profiles for unknown user / merchant          fl/processors/TransactionProcessor.java:489-508
PARITY UNPINNED: no JDK here, the reference has no tests, and UserProfile / MerchantProfile are missing
from its source; the declared semantics for their methods (isVerified, isNewAccount,
isHighRiskCategory, isOperatingAtHour) are the ones in DESIGN.md "Feature map".
"""
from __future__ import annotations

import math

import numpy as np

NAMES = (
    "amount", "amount_log", "amount_sqrt", "is_round_amount", "is_round_10", "is_round_100",
    "amount_to_user_avg_ratio", "amount_deviation_zscore", "is_large_for_user",
    "amount_to_merchant_avg_ratio", "is_large_for_merchant", "amount_category",
    "hour_of_day", "day_of_week", "day_of_month", "is_weekend", "time_period",
    "is_business_hours", "is_night_time", "in_user_preferred_time",
    "has_geolocation", "has_merchant_location", "latitude", "longitude",
    "is_high_risk_country", "distance_to_merchant_km", "user_intl_preference",
    "unexpected_intl_transaction",
    "account_age_days", "is_new_account", "is_very_new_account", "user_risk_score",
    "is_kyc_verified", "kyc_status", "weekend_activity_factor", "online_preference",
    "user_avg_amount", "user_transaction_frequency",
    "merchant_risk_level", "merchant_fraud_rate", "is_blacklisted_merchant",
    "merchant_category", "is_high_risk_category", "within_merchant_hours",
    "merchant_risk_multiplier", "suspicious_merchant_name",
    "is_known_device", "is_new_device", "is_private_ip", "ip_risk_score",
    "suspicious_user_agent",
    "velocity_5min_count", "velocity_5min_amount", "velocity_1hour_count",
    "velocity_1hour_amount", "velocity_24hour_count", "velocity_24hour_amount",
    "high_velocity_5min", "high_velocity_1hour",
    "payment_method", "is_high_risk_payment", "transaction_type", "is_refund", "card_type")
assert len(NAMES) == 64
IDX = {n: i for i, n in enumerate(NAMES)}
UNKNOWN = 254.0
CRITICAL, HIGH, MEDIUM, LOW, VERY_LOW = 4, 3, 2, 1, 0
APPROVE, REVIEW, DECLINE = 0, 1, 2
NaN = float("nan")


def _nan(x):
    return x is None or (isinstance(x, float) and math.isnan(x))


def _code(c):
    return UNKNOWN if c == 255 else float(c)


def day_of_month(days: int) -> int:
    import datetime
    return (datetime.date(1970, 1, 1) + datetime.timedelta(days=int(days))).day


def _operating(mext, m, h):
    if mext is None or m >= len(mext["open_hour"]) or mext["open_hour"][m] == 255 or mext["close_hour"][m] == 255:
        return True
    return int(mext["open_hour"][m]) <= h < int(mext["close_hour"][m])


def feature_map(txns, ctx, raw, vel5, users_ext, merchants, mext, vocab_pay, vocab_refund, threshold=0.7):
    """txns: SoA dict (fd_txn_batch fields); ctx: dict of the fd_txn_context arrays (missing keys = null);
    raw, vel5: the oracle feature state's outputs for the same batch; users_ext: {key: dict of profile
    fields}; merchants: {"fraud_rate", "risk_multiplier"}; mext: dict of fd_merchants_ext arrays or None.
    -> (fmap [n, 64] f64, rules structured array)."""
    n = len(raw)
    fm = np.full((n, 64), np.nan)
    rules = np.zeros(n, dtype=[("tp_score", "<f8"), ("fe_score", "<f8"), ("tp_decision", "u1"), ("tp_risk", "u1"),
                               ("fe_decision", "u1"), ("fe_risk", "u1"), ("pad", "u1", 4)])
    nm = len(merchants["fraud_rate"])
    g = lambda k, i, d: (ctx[k][i] if (ctx is not None and ctx.get(k) is not None) else d)  # noqa: E731
    for i in range(n):
        r = raw[i]
        f = fm[i]
        key = int(txns["card_key"][i]) or 1
        has_user = not math.isnan(r[8])
        ue = users_ext.get(key) if has_user else None
        ue = ue or {}
        risk = ue.get("risk_score", NaN)
        kyc = ue.get("kyc_status", 255)
        verified = bool(ue.get("verified", 0))
        ps, pe = ue.get("pref_start", -1), ue.get("pref_end", -1)
        weekend, online = ue.get("weekend_activity", NaN), ue.get("online_preference", NaN)
        intl = ue.get("intl_preference", NaN)
        freq = ue.get("txn_frequency", -1)
        patterns = bool(ue.get("has_patterns", 0))
        m = int(txns["merchant"][i])
        has_m = 0 <= m < nm
        mloaded = has_m and mext is not None and m < len(mext["risk_level"])
        mavg = mext["avg_amount"][m] if mloaded else NaN
        mrl = int(mext["risk_level"][m]) if mloaded else 255
        mbl = int(mext["blacklisted"][m]) if mloaded else 255
        mcat = int(mext["category"][m]) if mloaded else 255
        mhr = bool(mext["high_risk_category"][m]) if mloaded else False
        msus = int(mext["suspicious_name"][m]) if mloaded else 255
        mfr_raw = merchants["fraud_rate"][m] if has_m else NaN
        cents = int(txns["amount_cents"][i])
        amount = r[0]
        hour = int(r[2])
        hour_field = int(txns["hour"][i])
        age = int(r[15]) if has_user else -1
        age_known = has_user and age >= 0
        uavg = r[8] if has_user else NaN  # FeatureExtractor sees the avg (null -> 0.0 via r[8])
        known_device = r[6] < 0.5
        # amount
        f[0] = amount
        f[1] = r[1]
        f[2] = math.sqrt(amount)
        f[3] = 1.0 if cents % 100 == 0 else 0.0
        f[4] = 1.0 if cents % 1000 == 0 else 0.0
        f[5] = 1.0 if cents % 10000 == 0 else 0.0
        if has_user and not math.isnan(uavg) and uavg > 0:
            ratio = amount / uavg
            f[6] = ratio
            f[7] = (amount - uavg) / uavg
            f[8] = 1.0 if ratio > 3.0 else 0.0
        if has_m and not math.isnan(mavg) and mavg > 0:
            f[9] = amount / mavg
            f[10] = 1.0 if amount > mavg * 2.0 else 0.0
        f[11] = 0.0 if amount < 10 else 1.0 if amount < 100 else 2.0 if amount < 1000 else 3.0 if amount < 10000 else 4.0
        # temporal
        f[12] = float(hour)
        f[13] = r[3]
        ts = int(txns["ts_ms"][i])
        f[14] = float(day_of_month(ts // 86400000))
        f[15] = r[4]
        f[16] = 0.0 if 6 <= hour < 12 else 1.0 if 12 <= hour < 18 else 2.0 if 18 <= hour < 22 else 3.0
        f[17] = 1.0 if 9 <= hour <= 17 else 0.0
        f[18] = 1.0 if (hour <= 6 or hour >= 22) else 0.0
        if has_user and ps >= 0 and pe >= 0:
            f[19] = 1.0 if ps <= hour <= pe else 0.0
        # geographic
        glat, glon = g("geo_lat", i, NaN), g("geo_lon", i, NaN)
        mlat, mlon = g("merchant_lat", i, NaN), g("merchant_lon", i, NaN)
        f[20] = 1.0 if not (math.isnan(glat) and math.isnan(glon)) else 0.0
        f[21] = 1.0 if not (math.isnan(mlat) and math.isnan(mlon)) else 0.0
        if not math.isnan(glat) and not math.isnan(glon):
            f[22], f[23] = glat, glon
            f[24] = 1.0 if (abs(glat) > 60 or (abs(glat) < 10 and abs(glon) < 10)) else 0.0
            if not math.isnan(mlat) and not math.isnan(mlon):
                rad = 0.017453292519943295
                dlat, dlon = (mlat - glat) * rad, (mlon - glon) * rad
                a = (math.sin(dlat / 2) * math.sin(dlat / 2)
                     + math.cos(glat * rad) * math.cos(mlat * rad) * math.sin(dlon / 2) * math.sin(dlon / 2))
                f[25] = 6371 * (2 * math.atan2(math.sqrt(a), math.sqrt(1 - a)))
        if has_user and not math.isnan(intl):
            f[26] = intl
            f[27] = 1.0 if intl < 0.1 else 0.0
        # user behaviour
        if has_user:
            f[28] = float(age) if age_known else 0.0
            f[29] = 1.0 if (age_known and age < 30) else 0.0
            f[30] = 1.0 if (age_known and age < 7) else 0.0
            f[31] = 0.5 if math.isnan(risk) else risk
            f[32] = 1.0 if verified else 0.0
            f[33] = _code(kyc)
            if patterns:
                f[34] = 0.5 if math.isnan(weekend) else weekend
                f[35] = 0.7 if math.isnan(online) else online
            f[36] = 0.0 if math.isnan(uavg) else uavg
            f[37] = float(freq) if freq >= 0 else 0.0
        else:
            f[28], f[29], f[30], f[31], f[32], f[33] = 0.0, 1.0, 1.0, 0.8, 0.0, UNKNOWN
        # merchant
        if has_m:
            f[38] = _code(mrl)
            f[39] = 0.05 if math.isnan(mfr_raw) else mfr_raw
            f[40] = 1.0 if mbl == 1 else 0.0
            f[41] = _code(mcat)
            f[42] = 1.0 if mhr else 0.0
            if hour_field != 255:
                f[43] = 1.0 if _operating(mext if mloaded else None, m, hour_field) else 0.0
            f[44] = r[14]
            if msus != 255:
                f[45] = 1.0 if msus else 0.0
        else:
            f[38], f[39], f[40], f[41], f[42], f[44] = UNKNOWN, 0.1, 0.0, UNKNOWN, 0.0, 2.0
        # device / network
        f[46] = 1.0 if known_device else 0.0
        f[47] = 0.0 if known_device else 1.0
        ipc = int(txns["ip_class"][i])
        if ipc != 0:
            f[48] = 1.0 if ipc == 1 else 0.0
            f[49] = r[7]
        ua = int(g("user_agent_flag", i, 255))
        if ua != 255:
            f[50] = 1.0 if ua else 0.0
        # velocity
        f[51], f[52], f[53], f[54], f[55], f[56] = r[9], vel5[i], r[10], r[12], r[11], r[13]
        f[57] = 1.0 if r[9] > 5 else 0.0
        f[58] = 1.0 if r[10] > 20 else 0.0
        # contextual
        pay, tt, ct = int(g("payment_method", i, 255)), int(g("transaction_type", i, 255)), int(g("card_type", i, 255))
        f[59] = _code(pay)
        f[60] = 1.0 if (pay != 255 and vocab_pay[pay]) else 0.0
        f[61] = _code(tt)
        f[62] = 1.0 if (tt != 255 and vocab_refund[tt]) else 0.0
        f[63] = _code(ct)

        # FeatureEnrichmentProcessor
        T = lambda k: (not math.isnan(f[k])) and f[k] != 0.0  # noqa: E731
        F = lambda k: (not math.isnan(f[k])) and f[k] == 0.0  # noqa: E731
        sa = 0.0
        if T(8): sa += 0.3
        if T(5): sa += 0.1
        if f[11] == 4.0: sa += 0.2
        elif f[11] == 0.0: sa += 0.1
        st = 0.0
        if T(18): st += 0.2
        if F(19): st += 0.15
        if T(15) and not math.isnan(f[34]) and f[34] < 0.3: st += 0.1
        su = 0.0
        if T(30): su += 0.4
        elif T(29): su += 0.2
        if F(32): su += 0.3
        if not math.isnan(f[31]): su += f[31] * 0.5
        sm = 0.0
        if T(40): sm += 0.8
        if T(42): sm += 0.3
        if not math.isnan(f[39]): sm += f[39] * 2.0
        if T(45): sm += 0.2
        if F(43): sm += 0.15
        sv = 0.0
        if T(57): sv += 0.6
        if T(58): sv += 0.4
        if f[51] > 3: sv += 0.2
        if f[53] > 10: sv += 0.15
        sd = 0.0
        if T(47): sd += 0.3
        if not math.isnan(f[49]): sd += f[49]
        if T(50): sd += 0.2
        fb = 0.0
        fb += sa * 0.2
        fb += st * 0.1
        fb += su * 0.25
        fb += sm * 0.2
        fb += sv * 0.15
        fb += sd * 0.1
        fb = max(0.0, min(1.0, fb))
        existing = g("fraud_score", i, NaN)
        fe = fb if math.isnan(existing) else max(0.0, min(1.0, (existing * 0.6) + (fb * 0.4)))
        rules["fe_score"][i] = fe
        rules["fe_risk"][i] = CRITICAL if fe >= 0.95 else HIGH if fe >= 0.8 else MEDIUM if fe >= 0.6 else \
            LOW if fe >= 0.3 else VERY_LOW
        rules["fe_decision"][i] = DECLINE if fe >= 0.95 else REVIEW if fe >= 0.6 else APPROVE

        # TransactionProcessor (minimal profiles for unknown user / merchant)
        urisk = risk if has_user else 0.5
        uver = verified if has_user else False
        pu = 0.0
        if not math.isnan(urisk): pu += urisk * 0.2
        if age_known and age < 30: pu += 0.1
        if not uver: pu += 0.15
        rl = mrl if has_m else 1
        bl = has_m and mbl == 1
        fr = mfr_raw if has_m else 0.05
        pm = 0.0
        if rl == 2: pm += 0.2
        elif rl == 1: pm += 0.1
        if bl: pm += 0.4
        if not math.isnan(fr) and fr > 0.05: pm += fr * 2.0
        if has_m and mhr: pm += 0.15
        pf = 0.0
        if has_user and not math.isnan(uavg) and uavg > 0 and amount / uavg > 5.0: pf += 0.15
        if has_user and int(txns["device_fp"][i]) != 0 and not known_device: pf += 0.1
        if hour_field != 255 and (hour_field <= 5 or hour_field >= 23): pf += 0.05
        if hour_field != 255 and not _operating(mext if mloaded else None, m, hour_field): pf += 0.1
        tp = 0.0
        if not math.isnan(existing): tp = existing * 0.5
        tp += pu
        tp += pm
        tp += pf
        tp = max(0.0, min(1.0, tp))
        rules["tp_score"][i] = tp
        if tp >= 0.9: dec, rk = DECLINE, CRITICAL
        elif tp >= threshold: dec, rk = REVIEW, HIGH
        elif tp >= 0.5: dec, rk = APPROVE, MEDIUM
        else: dec, rk = APPROVE, LOW
        if bl: dec, rk = DECLINE, CRITICAL
        rules["tp_decision"][i], rules["tp_risk"][i] = dec, rk
    return fm, rules
