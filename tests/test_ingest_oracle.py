"""CPU: the JSON ingest codec — its scalar conversions (the same ingest_parse.h code the
device kernel runs, evaluated on the host through fd_ingest_scalar_host) pinned against Python's own
correctly rounded float(), decimal.Decimal and datetime; the identity hash; and known answers of the oracle
(oracle/ingest_ref.py) on simulator-format messages (services/data-simulator/src/main/python/simulator.py:186).
Bars: bit-exact (doubles compared as bit patterns, cents and epoch ms as integers)."""
import ctypes as C
import datetime as dt
import json
import math
import struct

import numpy as np
import pytest

from oracle import ingest_ref as R


def _scalar(kind, text):
    from fdengine import _native as N
    b = text.encode() if isinstance(text, str) else text
    arr = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    f, i, fl = C.c_double(), C.c_int64(), C.c_int32()
    N.call("fd_ingest_scalar_host", kind, C.c_void_p(arr.ctypes.data), len(b), C.byref(f), C.byref(i), C.byref(fl))
    return f.value, i.value, fl.value


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _number_corpus(rng, n):
    out = []
    for _ in range(n):
        kind = rng.integers(0, 6)
        if kind == 0:  # shortest repr of a random double (Python json.dumps of floats)
            out.append(repr(float(np.frombuffer(rng.bytes(8), np.float64)[0])))
        elif kind == 1:  # lat / lon style
            out.append(f"{rng.uniform(-180, 180):.{int(rng.integers(1, 8))}f}")
        elif kind == 2:  # 17 digit mantissas with exponents
            out.append(f"{rng.integers(10**16, 10**17)}e{rng.integers(-330, 300)}")
        elif kind == 3:  # amounts
            out.append(f"{rng.integers(0, 10**7)}.{rng.integers(0, 100):02d}")
        elif kind == 4:  # halfway-ish: 2^k-boundary decimal expansions
            m = int(rng.integers(1, 2**53))
            e = int(rng.integers(-60, 60))
            from decimal import Decimal
            out.append(str(Decimal(m) * (Decimal(2) ** e) + (Decimal(2) ** (e - 1))))
        else:  # long (> 19 digit) mantissas
            out.append("0." + "".join(str(int(d)) for d in rng.integers(0, 10, int(rng.integers(20, 40)))))
    return [s.replace("inf", "1e400").replace("nan", "0") for s in out]


def test_decimal_to_double_matches_python_float():
    rng = np.random.default_rng(1)
    corpus = _number_corpus(rng, 40000) + ["0", "-0", "-0.0", "1e-400", "2.2250738585072011e-308",
                                           "4.9406564584124654e-324", "2.4703282292062327e-324",
                                           "2.4703282292062328e-324", "1.7976931348623157e308",
                                           "1.7976931348623158e308", "9007199254740993", "0.1", "123.45",
                                           "1e22", "1e23", "8.98846567431158e307"]
    bad = []
    for s in corpus:
        if not R.NUMBER_RE.match(s):
            continue
        v, _, fl = _scalar(0, s)
        assert not (fl & 1), s
        if _bits(v) != _bits(float(s)) and not (fl & 2):
            bad.append((s, v, float(s)))
    assert not bad, bad[:5]


def test_number_grammar_errors():
    for s in ["", "-", "01", "1.", ".5", "1e", "1e+", "+1", "0x10", "1.5e3.2", "NaN", "Infinity", " 1"]:
        assert _scalar(0, s)[2] & 1, s


def test_cents_exact():
    from decimal import Decimal
    rng = np.random.default_rng(2)
    cases = [f"{rng.integers(0, 10**9)}.{rng.integers(0, 100):02d}" for _ in range(5000)]
    cases += ["1", "1.5", "0.005", "0.015", "0.025", "-3.335", "12.3", "1e2", "1.23e1", "99999999999999.99",
              "0.0000001", "7.125", "2.675"]
    for s in cases:
        _, c, fl = _scalar(1, s)
        ec, inexact = R.cents_of(Decimal(s))
        assert c == ec and bool(fl & 2) == inexact, (s, c, ec)


def test_iso_instants():
    rng = np.random.default_rng(3)
    for _ in range(3000):
        us = int(rng.integers(0, 4_102_444_800_000_000))
        t = dt.datetime(1970, 1, 1) + dt.timedelta(microseconds=us)
        s = t.isoformat()
        _, ms, fl = _scalar(2, s)
        assert fl == 0 and ms == us // 1000, s
        z = s + ("Z" if us % 2 else "+05:30")
        _, ms2, fl2 = _scalar(2, z)
        assert fl2 == 0 and ms2 == R.iso_to_ms(z), z
    for bad in ["2025-02-29T00:00:00", "2025-13-01T00:00:00", "2025-01-01 00:00:00", "2025-01-01T24:00:00",
                "2025-01-01T00:00:00.", "2025-01-01T00:00:00.1234567890", "2025-01-01T00:00:00+5:30", "x"]:
        assert _scalar(2, bad)[2] == 1 and R.iso_to_ms(bad) is None, bad
    assert _scalar(2, "2024-02-29T12:00:00.999999999-01:00")[1] == R.iso_to_ms("2024-02-29T12:00:00.999999999-01:00")


def test_hash64_matches_oracle():
    from fdengine.ingest import hash64
    for s in ["", "user_89346311", "é中", "\U0001F600", "a" * 1000]:
        assert hash64(s) == R.h64(s.encode("utf-8"))


def test_oracle_known_answers_simulator_message():
    from fdengine import synth
    sp = synth.sim_population(50, 10, seed=1)
    msg = synth.json_messages(sp, 1, seed=2)[0]
    doc = json.loads(msg)
    merchants = {m: i for i, m in enumerate(sp["merchant_ids"])}
    vocabs = [{s: i for i, s in enumerate(v)} for v in (synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                                                         synth.SIM_CARD_TYPES)]
    row = R.parse_message(msg, merchants, vocabs)
    assert row["status"] == 0
    assert row["card_key"] == R.h64(doc["user_id"].encode())
    assert row["amount_cents"] == round(doc["amount"] * 100)
    t = dt.datetime.fromisoformat(doc["timestamp"]).replace(tzinfo=dt.timezone.utc)
    assert row["ts_ms"] == int(t.timestamp() * 1000) // 1 or abs(row["ts_ms"] - t.timestamp() * 1000) < 1
    assert row["merchant"] == merchants.get(doc["merchant_id"], -1)
    assert row["geo_lat"] == doc["geolocation"]["lat"]
    assert row["merchant_lat"] == float(doc["merchant_location"]["lat"])  # Decimal -> str on the wire
    assert row["payment_method"] == vocabs[0][doc["payment_method"]]
    assert row["hour"] == doc["hour_of_day"] and row["weekend"] == int(doc["is_weekend"])
    assert row["is_fraud"] == int(doc["is_fraud"]) and row["fraud_score"] == doc["fraud_score"]


@pytest.mark.parametrize("raw,status", [
    (b'{"user_id": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00"}', 0),
    (b'{"user_id": "u", "amount": 1}', R.MISSING),
    (b'{"user_id": null, "amount": 1, "timestamp": "2025-01-01T00:00:00"}', R.MISSING),
    (b'{"user_id": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00",}', R.MALFORMED),
    (b'[1, 2]', R.MALFORMED),
    (b'{"user_id": "u", "amount": NaN, "timestamp": "2025-01-01T00:00:00"}', R.MALFORMED),
    (b'{"user_id": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00"} x', R.MALFORMED),
    (b'{"user_id": "u", "amount": "1.005", "timestamp": "2025-01-01T00:00:00"}', R.INEXACT),
    (b'{"user_id": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00", "payment_method": "crypto"}',
     R.UNKNOWN_VOCAB),
    (b'{"user_id": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00", "hour_of_day": -1}', R.MALFORMED),
    (b'{"userId": "u", "amount": 1, "timestamp": "2025-01-01T00:00:00Z", "user_id": "v"}', 0),
])
def test_oracle_status(raw, status):
    row = R.parse_message(raw, {}, [{"credit_card": 0}, {}, {}])
    assert row["status"] == status
    if raw.endswith(b'"user_id": "v"}'):
        assert row["card_key"] == R.h64(b"v")  # the last alias wins


def test_oracle_amount_edge():
    row = R.parse_message(b'{"user_id": "u", "amount": "12.30", "timestamp": "2025-01-01T00:00:00"}', {}, [{}] * 3)
    assert row["amount_cents"] == 1230 and row["status"] == 0
    assert math.isnan(row["geo_lat"]) and row["merchant"] == -1 and row["hour"] == 255
