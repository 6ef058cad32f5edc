"""GPU parity of the Kafka JSON ingest codec (ingest.hip) vs oracle/ingest_ref.py (Python's
json + Decimal + correctly rounded float) on the same messages: simulator-format streams
(json.dumps(asdict(Transaction), default=str), simulator.py:186) and an edge-case corpus — whitespace,
reordered / camelCase / duplicate keys, escapes and surrogate pairs, numbers as strings, exponents, nulls,
missing required fields, malformed JSON, oversize messages, nested unknown values.
Bar: every column bit-exact (doubles as bit patterns, NaN == NaN) on every row; parity vs Jackson unpinned."""
import json

import numpy as np
import pytest

from fdengine import synth
from fdengine._native import INGEST_FIELDS
from fdengine.ingest import IngestCodec, device_columns, pack
from oracle import ingest_ref as R

pytestmark = pytest.mark.gpu

VOCABS = (synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES, synth.SIM_CARD_TYPES)


def _codec(engine, sp):
    return IngestCodec(engine, sp["merchant_ids"], *VOCABS)


def _oracle(sp, msgs):
    merchants = {}
    for i, m in enumerate(sp["merchant_ids"]):
        merchants.setdefault(m, i)
    return R.parse_batch(msgs, merchants, [{s: i for i, s in enumerate(v)} for v in VOCABS])


def _same(got, exp, msgs=None):
    for k, _ in INGEST_FIELDS:
        g, e = got[k], exp[k]
        if g.dtype.kind == "f":
            g, e = g.view(np.uint64), e.view(np.uint64)
            # NaN payloads: compare canonically
            gn, en = np.isnan(got[k]), np.isnan(exp[k])
            ok = (g == e) | (gn & en)
        else:
            ok = g == e
        if not ok.all():
            i = int(np.flatnonzero(~ok)[0])
            raise AssertionError(f"{k}[{i}]: device {got[k][i]!r} oracle {exp[k][i]!r} status "
                                 f"{got['status'][i]}/{exp['status'][i]} msg {msgs[i][:300] if msgs else ''}")


def test_simulator_stream_host_and_device(engine):
    import torch
    sp = synth.sim_population(3000, 400, seed=4)
    msgs = synth.json_messages(sp, 20000, seed=5)
    codec = _codec(engine, sp)
    exp = _oracle(sp, msgs)
    got = codec.parse(msgs)
    _same(got, exp, msgs)
    assert (got["status"] == 0).mean() > 0.99 and (got["merchant"] == -1).any() and (got["ip_class"] == 1).any()
    assert (got["user_agent_flag"] == 1).any() and (got["user_agent_flag"] == 0).any()
    # device-resident batch -> device columns
    buf, off = pack(msgs)
    dbuf = torch.from_numpy(buf.copy()).cuda()
    doff = torch.from_numpy(off).cuda()
    cols, ptrs = device_columns(len(msgs))
    engine.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        codec.parse_device(dbuf.data_ptr(), doff.data_ptr(), len(msgs), ptrs)
        torch.cuda.synchronize()
    finally:
        engine.set_stream(None)
    dev = {k: cols[k].cpu().numpy().view(dt) for k, dt in INGEST_FIELDS}
    _same(dev, exp, msgs)


def _edge_corpus():
    base = dict(transaction_id="t-1", user_id="user_1", merchant_id="m0", amount=12.5, currency="USD",
                transaction_type="refund", payment_method="debit_card", card_type="visa",
                timestamp="2025-09-05T10:11:12.345678", ip_address="10.1.2.3", device_fingerprint="fp-1",
                user_agent="Mozilla/5.0 (X11; Linux x86_64) Firefox/121", geolocation={"lat": 1.5, "lon": -2.25},
                merchant_location={"lat": "3.000001", "lon": "-4.5"}, is_weekend=False, hour_of_day=10,
                is_fraud=True, fraud_type=None, fraud_score=0.875)
    d = lambda **kw: json.dumps(dict(base, **kw)).encode()  # noqa: E731
    out = [
        d(), json.dumps(base, indent=2).encode(), json.dumps(base, separators=(",", ":")).encode(),
        b"\r\n\t " + d() + b" \n",
        json.dumps(dict(reversed(list(base.items())))).encode(),
        d(user_id="usér_中\U0001F600"), d(user_id="us\\er\"q/\b\f\n\r\t"),
        json.dumps(dict(base, user_id="é中😀"), ensure_ascii=False).encode(),
        d(user_id="\ud800lone"),  # lone surrogate (escaped)
        d(amount="99.99"), d(amount=1e2), d(amount=0.005), d(amount=-3.5), d(amount=12345678901234.56),
        d(amount=None), d(timestamp=None), d(user_id=None), d(timestamp="2025-09-05T10:11:12Z"),
        d(timestamp="2025-09-05T10:11:12.5+05:30"), d(timestamp="2025-09-05 10:11:12"),
        d(timestamp="2025-02-30T00:00:00"), d(timestamp=12345), d(fraud_score="0.25"), d(fraud_score=None),
        d(fraud_score=1e-7), d(fraud_score=0.1234567890123456789012), d(fraud_score=[1]),
        d(geolocation=None), d(geolocation={}), d(geolocation={"lat": None, "lon": "7"}),
        d(geolocation={"lon": 1, "x": {"a": [1, {"b": "}"}]}, "lat": 2}), d(geolocation=[1, 2]),
        d(geolocation={"lat": True}), d(is_weekend="true"), d(is_weekend=1), d(is_weekend=0), d(is_weekend=None),
        d(is_weekend=1.5), d(is_fraud="false"), d(hour_of_day=23.7), d(hour_of_day="7"), d(hour_of_day=254),
        d(hour_of_day=255), d(hour_of_day=-0.0), d(hour_of_day=-1), d(hour_of_day=None), d(hour_of_day=2e1),
        d(payment_method="crypto"), d(payment_method=None), d(payment_method=7), d(card_type=True),
        d(transaction_type={"x": 1}), d(merchant_id="unknown"), d(merchant_id=None), d(merchant_id=5),
        d(ip_address="192.168.0.1"), d(ip_address="172.16.5.4"), d(ip_address="172.17.0.1"),
        d(ip_address="10."), d(ip_address="1"), d(ip_address=None),
        d(user_agent="Googlebot/2.1"), d(user_agent="short"), d(user_agent="x" * 19), d(user_agent="x" * 20),
        d(user_agent="\U0001F600" * 10), d(user_agent="\U0001F600" * 9 + "a"), d(user_agent="MyCrawler 1.0 crawler"),
        d(user_agent=None), d(device_fingerprint=None), d(transaction_id=None),
        # the cooperative user-agent scan: matches across its 64-byte steps, long / multi-byte / empty strings,
        # escapes (serial fallback), control bytes, duplicates, non-string values
        d(user_agent="A" * 62 + "bot"), d(user_agent="A" * 60 + "crawler" + "B" * 100), d(user_agent="A" * 63 + "crawle"),
        d(user_agent="b" * 64 + "ot"), d(user_agent="é" * 70), d(user_agent=""), d(user_agent='say "bot" loudly ok'),
        d(user_agent="tab\there and a long tail of text"), d(user_agent=12345678901234567890123),
        json.dumps(dict(base, user_agent="😀é中" * 30), ensure_ascii=False).encode(),
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "\\u0062ot-agent long"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "x\x01yyyyyyyyyyyyyyyyyyyyy"}',
        b'{"user_agent": "Mozilla bot", "user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", '
        b'"userAgent": "Mozilla/5.0 long enough string here"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "abc',
        d(user_agent="A" * 60 + "é中" + "bot"), d(user_agent="bo" + "é" + "t and more text here"),
        d(user_agent="x" * 61 + "\U0001F600" * 3 + "crawler"), d(user_agent="ends with backslashes \\\\"),
        d(user_agent='quote\\"bot\\\\' + "z" * 70), d(user_agent="é" * 19), d(user_agent="é" * 20),
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "' + b"y" * 62 +
        b'\\u00e9\\u4e2dcrawler"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "ro\\bot yyyyyyyyyyyyyyyy"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "c\\rawler yyyyyyyyyyyyyy"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "bad \\x escape yyyyyyyy"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "bad \\u12G4 hex yyyyyyy"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_agent": "cut \\u12"}',
        d(extra={"deep": [[[{"x": "]}"}]]], "s": "\\\"}"}), d(userId="camel"),
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_id": "b"}',
        b'{"userId": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "user_id": "b", "userId": "c"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00",}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00"',
        b'{"user_id": "a, "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00"}}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00"} {}',
        b'{"user_id": "a", "amount": 01, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a", "amount": 1., "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a", "amount": NaN, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a\x01", "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a\\x", "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id" "a", "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a" "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{, "user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00"}',
        b'{"user_id": "a", "amount": 1, "timestamp": "2025-01-01T00:00:00", "x": tru}',
        b"[1, 2, 3]", b"", b"   ", b"null", b'"str"', b"{}", b'{"a": 1}',
        d(blob="y" * 5000), d(blob="y" * 3500),
        json.dumps(dict(base, **{f"k{i}": i for i in range(45)})).encode(),  # 64 members: the limit
        json.dumps(dict(base, **{f"k{i}": i for i in range(46)})).encode(),  # 65 members
    ]
    return out


def test_edge_corpus(engine):
    sp = {"merchant_ids": ["m0", "m1", "5"]}
    msgs = _edge_corpus()
    codec = IngestCodec(engine, sp["merchant_ids"], *VOCABS)
    got = codec.parse(msgs)
    exp = _oracle(sp, msgs)
    _same(got, exp, msgs)
    st = got["status"]
    # coverage: every status class occurs
    for bit in (R.MALFORMED, R.TOO_LONG, R.UNKNOWN_VOCAB, R.INEXACT, R.MISSING):
        assert (st & bit).any(), bit
    assert (st == 0).sum() > 30


def test_unaligned_and_tail_offsets(engine):
    """messages packed at odd offsets; the last one ends exactly at the buffer end (no padding)"""
    sp = synth.sim_population(200, 50, seed=8)
    msgs = synth.json_messages(sp, 257, seed=9)
    msgs = [b" " * (i % 7) + m for i, m in enumerate(msgs)]
    codec = _codec(engine, sp)
    _same(codec.parse(msgs), _oracle(sp, msgs), msgs)
    one = codec.parse(msgs[:1])
    _same(one, _oracle(sp, msgs[:1]), msgs)
    empty = codec.parse([])
    assert all(len(v) == 0 for v in empty.values())


def test_vocab_growth(engine):
    sp = synth.sim_population(50, 10, seed=3)
    msgs = synth.json_messages(sp, 300, seed=4)
    codec = IngestCodec(engine, sp["merchant_ids"], ["credit_card"], [], [])
    first = codec.parse(msgs)
    assert (first["status"] & R.UNKNOWN_VOCAB).any()
    got = codec.parse(msgs, grow_vocab=True)
    assert not (got["status"] & R.UNKNOWN_VOCAB).any()
    assert codec.vocab[0][0] == "credit_card" and set(codec.vocab[0]) == set(synth.SIM_PAYMENT_METHODS)
    docs = [json.loads(m) for m in msgs]
    for i in range(0, 300, 17):
        assert codec.vocab[0][got["payment_method"][i]] == docs[i]["payment_method"]
        assert codec.vocab[1][got["transaction_type"][i]] == docs[i]["transaction_type"]
    pay, ref = codec.vocab_flags()
    assert ref[codec.vocab[1].index("refund")] == 1 and pay.sum() == 0
