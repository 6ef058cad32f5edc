"""GPU: snapshot / restore of the HBM keyed state (SURVEY §8(f) rank 4 — the counterpart of Flink keyed-state
checkpoints, fl/FraudDetectionJob.java:112-136, and the Redis RDB, config/redis/redis-master.conf:6-13).

Property bar (size-independent, bit-exact): a stream cut by snapshot -> restore (into a fresh engine with a
different table capacity) produces exactly the outputs of the uninterrupted stream — scoring vectors, the
64-column feature map, rule scores, LSTM history sequences and the Flink window results; re-sharding 2 -> 3
GPUs by restoring every old image on every new shard reproduces the unsharded engine per transaction.
Images are byte-identical for the same table; corrupt / truncated / mismatched images fail loudly."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from fdengine.engine import shard_of
from fdengine._native import CTX_FIELDS, FD_ERR_IO, TXN_FIELDS, NativeError

pytestmark = pytest.mark.gpu

UF = ("user_key", "window_start", "window_end", "first_ts", "last_ts", "count", "total_amount", "velocity_score")


def _setup(eng, pop, cap, mode, seq_len=0, windows=True, owner=None):
    """owner = (rank, world): load only the users this shard owns (each card lives on one shard)."""
    U, M = pop["users"], pop["merchants"]
    keep = np.ones(len(U["key"]), bool) if owner is None else shard_of(U["key"], owner[1]) == owner[0]
    eng.state_init(cap, mode, 8, seq_len)
    eng.load_users(U["key"][keep], U["avg_amount"][keep], U["account_age_days"][keep],
                   np.asarray(U["device_fp"]).reshape(-1, 3)[keep])
    eng.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    ue = synth.users_ext(pop)
    eng.load_users_ext(ue["key"][keep], **{k: v[keep] for k, v in ue.items() if k != "key"})
    me = synth.merchants_ext(pop)
    eng.load_merchants_ext(len(me["avg_amount"]), **me)
    pay, ref = synth.vocab_flags()
    eng.load_vocab(pay, ref)
    if windows:
        eng.windows_init(1 << 16)


def _stream(n_users=1200, n=16000, seed=3):
    pop = synth.population(n_users, 120, seed=seed)
    tx = synth.txn_stream(pop, n, seed=seed + 1, rate_per_s=3.0, unknown_user_frac=0.05,
                          unknown_merchant_frac=0.03)
    ctx = synth.txn_context(tx)
    return pop, tx, ctx


def _full(eng, part, cpart):
    import torch
    n = len(part["card_key"])
    dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
    dctx = {f: torch.from_numpy(np.ascontiguousarray(cpart[f])).cuda() for f in CTX_FIELDS}
    vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
    fmap = torch.empty((n, 64), dtype=torch.float64, device="cuda")
    rules = torch.empty((n, 24), dtype=torch.uint8, device="cuda")
    eng.features_full_device({f: t.data_ptr() for f, t in dev.items()}, {f: t.data_ptr() for f, t in dctx.items()},
                             n, vec.data_ptr(), fmap.data_ptr(), rules.data_ptr())
    torch.cuda.synchronize()
    return vec.cpu().numpy(), fmap.cpu().numpy(), rules.cpu().numpy()


def _windows(eng, part, flush=False):
    gu, gm = eng.windows_step_host(part["card_key"], part["ts_ms"], part["amount_cents"], part["merchant"],
                                   flush=flush)
    u = sorted(tuple(r[f].item() for f in UF) for r in gu)
    m = sorted((int(r["merchant"]), int(r["window_start"]), int(r["count"]), float(r["total_amount"]),
                float(r["amount_stddev"])) for r in gm)
    return u, m


def _cuts(n, k):
    e = np.linspace(0, n, k + 1).astype(int)
    return list(zip(e[:-1], e[1:]))


def _run(eng, tx, ctx, cuts, windows=True, flush=True):
    out = []
    for a, b in cuts:
        part = {k: v[a:b] for k, v in tx.items()}
        cpart = {k: v[a:b] for k, v in ctx.items()}
        res = _full(eng, part, cpart)
        if windows:
            res = res + _windows(eng, part)
        out.append(res)
    if windows and flush:
        empty = {k: v[:0] for k, v in tx.items()}
        out.append(_windows(eng, empty, flush=True))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for p, q in zip(x, y):
            if isinstance(p, np.ndarray):
                np.testing.assert_array_equal(p.view(np.uint8), q.view(np.uint8))
            else:
                assert p == q


@pytest.mark.parametrize("mode", [0, 1])
def test_resume_equals_uninterrupted(engine, tmp_path, mode):
    pop, tx, ctx = _stream(seed=3 + mode)
    cuts = _cuts(len(tx["card_key"]), 8)
    _setup(engine, pop, 8192, mode)
    _run(engine, tx, ctx, cuts[:4], flush=False)
    path = tmp_path / "state.fdsnap"
    nbytes = engine.state_snapshot(path)
    assert nbytes == path.stat().st_size > 256
    cards = engine.state_info()["cards"]
    ref = _run(engine, tx, ctx, cuts[4:])
    fresh = FraudEngine(0)
    try:
        fresh.state_init(1 << 15, mode, 8)  # different capacity: records land in other slots
        fresh.windows_init(1 << 16)
        assert fresh.state_restore(path) == cards
        got = _run(fresh, tx, ctx, cuts[4:])
    finally:
        fresh.close()
    _same(got, ref)
    assert sum(len(r[3]) for r in ref[:-1]) > 100  # user windows did fire after the cut


def _fnv_words(b: bytes) -> int:
    """snapshot.hip Fnv over a section whose length is a multiple of 8"""
    h, mask = 0xCBF29CE484222325, (1 << 64) - 1
    for w in np.frombuffer(b, dtype="<u8").tolist():
        h = ((h ^ w) * 0x100000001B3) & mask
    return h


def _downgrade_to_v2(blob: bytes, mode: int) -> bytes:
    """A v3 image rewritten as the v2 format (the card header before the round-5 relayout: key first, absolute oldest
    in-window times, the redis_compat session amount in its own word), checksum recomputed — what a pre-relayout
    engine wrote for the same state."""
    import struct
    hd = bytearray(blob[:256])
    n_cards, rec_bytes = struct.unpack_from("<qq", hd, 48)
    cards = bytearray(blob[256:256 + n_cards * rec_bytes])
    for r in range(n_cards):
        o = r * rec_bytes
        v3 = bytes(cards[o:o + 128])
        last_ts, rn, rh, us, _, wc0, wc1, wc2, _, flags, rc_cnt = struct.unpack_from("<q8BIi", v3, 0)
        ws = list(struct.unpack_from("<3q", v3, 24))
        wod = struct.unpack_from("<3I", v3, 48)
        key, avg, age = struct.unpack_from("<Qdi", v3, 64)
        fp = struct.unpack_from("<3Q", v3, 88)
        wc = (wc0, wc1, wc2)
        wo = [last_ts - wod[k] if wc[k] > 0 else 0 for k in range(3)]
        rc_sum = 0
        if mode == 0:  # redis_compat: the session amount had its own field
            rc_sum, ws[0] = ws[0], 0
        v2 = struct.pack("<QqdiI8B3Q3q3qqii", key, last_ts, avg, age, flags, rn, rh, us, 0, wc0, wc1, wc2, 0,
                         *fp, *ws, *wo, rc_sum, rc_cnt, 0)
        assert len(v2) == 128
        cards[o:o + 128] = v2
    struct.pack_into("<I", hd, 8, 2)
    struct.pack_into("<Q", hd, 136, _fnv_words(bytes(cards)))
    return bytes(hd) + bytes(cards) + blob[256 + n_cards * rec_bytes:]


@pytest.mark.parametrize("mode", [0, 1])
def test_v2_image_restores_as_v3(engine, tmp_path, mode):
    """images written before the round-5 header relayout (format v2) restore through a host-side
    header conversion and continue the stream exactly as the v3 image of the same state does; other versions are
    refused with FD_ERR_UNSUPPORTED."""
    import struct
    from fdengine._native import FD_ERR_UNSUPPORTED
    pop, tx, ctx = _stream(n_users=600, n=6000, seed=41 + mode)
    cuts = _cuts(len(tx["card_key"]), 4)
    _setup(engine, pop, 4096, mode)
    _run(engine, tx, ctx, cuts[:2], flush=False)
    v3 = tmp_path / "v3.fdsnap"
    engine.state_snapshot(v3)
    v2 = tmp_path / "v2.fdsnap"
    v2.write_bytes(_downgrade_to_v2(v3.read_bytes(), mode))
    v1 = bytearray(v3.read_bytes())
    struct.pack_into("<I", v1, 8, 1)
    (tmp_path / "v1.fdsnap").write_bytes(bytes(v1))
    outs = []
    for path in (v3, v2):
        fresh = FraudEngine(0)
        try:
            fresh.state_init(4096, mode, 8)
            fresh.windows_init(1 << 16)
            assert fresh.state_restore(path) == engine.state_info()["cards"]
            outs.append(_run(fresh, tx, ctx, cuts[2:]))
            if path == v2:
                with pytest.raises(NativeError, match="unsupported snapshot version") as ei:
                    fresh.state_restore(tmp_path / "v1.fdsnap")
                assert ei.value.code == FD_ERR_UNSUPPORTED
        finally:
            fresh.close()
    _same(outs[1], outs[0])


def test_resume_lstm_history(engine, tmp_path):
    import torch
    pop, tx, _ = _stream(n_users=800, n=9000, seed=11)
    cuts = _cuts(len(tx["card_key"]), 6)

    def run(eng, cs):
        out = []
        for a, b in cs:
            part = {k: v[a:b] for k, v in tx.items()}
            n = b - a
            dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
            vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
            seq = torch.empty((n, 10, 16), dtype=torch.float32, device="cuda")
            eng.features_seq_device({f: t.data_ptr() for f, t in dev.items()}, n, vec.data_ptr(), seq.data_ptr())
            torch.cuda.synchronize()
            out.append((vec.cpu().numpy(), seq.cpu().numpy()))
        return out

    _setup(engine, pop, 4096, 1, seq_len=10, windows=False)
    run(engine, cuts[:3])
    path = tmp_path / "lstm.fdsnap"
    engine.state_snapshot(path)
    ref = run(engine, cuts[3:])
    fresh = FraudEngine(0)
    try:
        fresh.state_init(3000, 1, 8, 10)
        fresh.state_restore(path)
        got = run(fresh, cuts[3:])
    finally:
        fresh.close()
    _same(got, ref)


def test_reshard_two_to_three(engine, tmp_path):
    """Emulated shards: old shard r of 2 sees only its cards' transactions; after the cut every new shard of 3
    restores both old images (keeping its own cards) and must match the unsharded engine per transaction."""
    pop, tx, ctx = _stream(n_users=1500, n=12000, seed=21)
    n = len(tx["card_key"])
    cuts = _cuts(n, 6)
    _setup(engine, pop, 1 << 14, 1, windows=False)
    ref = _run(engine, tx, ctx, cuts, windows=False)
    ref_vec = np.concatenate([r[0] for r in ref])
    ref_fmap = np.concatenate([r[1] for r in ref])
    ref_rules = np.concatenate([r[2] for r in ref])

    def sub(d, m):
        return {k: v[m] for k, v in d.items()}

    old = [FraudEngine(0) for _ in range(2)]
    new = [FraudEngine(0) for _ in range(3)]
    try:
        o2 = shard_of(tx["card_key"], 2)
        paths = []
        for r, e in enumerate(old):
            _setup(e, pop, 1 << 13, 1, windows=False, owner=(r, 2))
            for a, b in cuts[:3]:
                m = np.zeros(n, bool)
                m[a:b] = o2[a:b] == r
                _full(e, sub(tx, m), sub(ctx, m))
            p = tmp_path / f"state-{r}-of-2.fdsnap"
            e.state_snapshot(p, r, 2)
            paths.append(p)
        o3 = shard_of(tx["card_key"], 3)
        restored = 0
        vec = np.zeros_like(ref_vec)
        fmap = np.zeros_like(ref_fmap)
        rules = np.zeros_like(ref_rules)
        for r, e in enumerate(new):
            e.state_init(1 << 13, 1, 8)
            for p in paths:
                restored += e.state_restore(p, r, 3)
            for a, b in cuts[3:]:
                m = np.zeros(n, bool)
                m[a:b] = o3[a:b] == r
                v, f, ru = _full(e, sub(tx, m), sub(ctx, m))
                vec[m], fmap[m], rules[m] = v, f, ru
        tail = slice(cuts[3][0], n)
        np.testing.assert_array_equal(vec[tail].view(np.uint32), ref_vec[tail].view(np.uint32))
        np.testing.assert_array_equal(fmap[tail].view(np.uint64), ref_fmap[tail].view(np.uint64))
        np.testing.assert_array_equal(rules[tail], ref_rules[tail])
        assert restored == sum(e.state_info()["cards"] for e in old)
    finally:
        for e in old + new:
            e.close()


def test_image_deterministic_and_corruption_detected(engine, tmp_path):
    pop, tx, ctx = _stream(n_users=500, n=4000, seed=31)
    _setup(engine, pop, 2048, 0)
    _run(engine, tx, ctx, _cuts(4000, 2), flush=False)
    a, b = tmp_path / "a.fdsnap", tmp_path / "b.fdsnap"
    engine.state_snapshot(a)
    engine.state_snapshot(b)
    blob = a.read_bytes()
    assert blob == b.read_bytes()
    fresh = FraudEngine(0)
    try:
        fresh.state_init(2048, 0, 8)
        fresh.windows_init(1 << 16)
        bad = bytearray(blob)
        bad[256 + 1000] ^= 0x40  # a byte inside the card records
        (tmp_path / "bad.fdsnap").write_bytes(bytes(bad))
        with pytest.raises(NativeError, match="checksum") as ei:
            fresh.state_restore(tmp_path / "bad.fdsnap")
        assert ei.value.code == FD_ERR_IO
        assert fresh.state_info()["cards"] == 0  # verified before anything is restored
        bad = bytearray(blob)
        bad[len(blob) - 24] ^= 0x01  # a byte in the last section (window logs)
        (tmp_path / "bad2.fdsnap").write_bytes(bytes(bad))
        with pytest.raises(NativeError, match="checksum"):
            fresh.state_restore(tmp_path / "bad2.fdsnap")
        assert fresh.state_info()["cards"] == 0
        (tmp_path / "short.fdsnap").write_bytes(blob[: len(blob) // 2])
        fresh.state_clear()
        with pytest.raises(NativeError, match="truncated"):
            fresh.state_restore(tmp_path / "short.fdsnap")
        with pytest.raises(NativeError, match="cannot open"):
            fresh.state_restore(tmp_path / "missing.fdsnap")
        fresh.state_init(2048, 0, 8, 4)  # seq_len differs
        with pytest.raises(NativeError, match="seq_len"):
            fresh.state_restore(a)
        fresh.state_init(64, 0, 8)  # too small for the image's cards
        fresh.windows_init(1 << 16)
        with pytest.raises(NativeError, match="card table full"):
            fresh.state_restore(a)
    finally:
        fresh.close()
    fresh = FraudEngine(0)
    try:
        fresh.state_init(2048, 0, 8)  # the image holds window state; windows not initialised here
        with pytest.raises(ValueError, match="fd_windows_init"):
            fresh.state_restore(a)
        assert fresh.state_restore(a, skip_windows=True) == engine.state_info()["cards"]
    finally:
        fresh.close()


def test_image_carries_sink_and_ingest_tables(engine, tmp_path):
    """The image also holds the RedisTransactionSink aggregates (resume on the same shard) and the ingest codec's
    merchant / vocabulary tables: a fresh engine restored from it continues both exactly."""
    from fdengine._native import FD_AGG_HOURLY, FD_AGG_MERCHANT
    from fdengine.ingest import IngestCodec
    from oracle.sink_ref import SinkOracle
    batches = synth.window_stream(6, 3000, 300, 40, seed=17, batch_span_ms=900_000)
    engine.state_init(1 << 14, 1, 8)
    engine.sink_init(1 << 13, 1 << 15)
    sp = synth.sim_population(100, 30, seed=2)
    codec = IngestCodec(engine, sp["merchant_ids"], synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                        synth.SIM_CARD_TYPES)
    msgs = synth.json_messages(sp, 300, seed=3)
    before = codec.parse(msgs)
    o = SinkOracle()

    def feed(eng, b):
        eng.sink_update_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"], b["is_fraud"], b["fraud_score"])
        o.run_batch(b)

    for b in batches[:3]:
        feed(engine, b)
    path = tmp_path / "full.fdsnap"
    engine.state_snapshot(path)
    fresh = FraudEngine(0)
    try:
        fresh.state_init(1 << 12, 1, 8)
        fresh.state_restore(path)
        for b in batches[3:]:
            fresh.sink_update_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"], b["is_fraud"],
                                   b["fraud_score"])
            o.run_batch(b)
        hours = sorted(int(k.split(":")[1]) for k in o.redis if k.startswith("hourly:"))
        got = fresh.sink_query(FD_AGG_HOURLY, hours)
        assert [int(x) for x in got["total_count"]] == [o.redis[f"hourly:{h}"]["total_count"] for h in hours]
        mk = sorted((int(k.split(":")[1]), int(k.split(":")[2])) for k in o.redis if k.startswith("merchant:"))
        got = fresh.sink_query(FD_AGG_MERCHANT, [h for _, h in mk], [m for m, _ in mk])
        assert [int(x) for x in got["unique_user_count"]] == \
               [o.redis[f"merchant:{m}:{h}"]["unique_user_count"] for m, h in mk]
        # the codec tables came with the image (no set_merchants / set_vocab on the fresh engine)
        c2 = IngestCodec.__new__(IngestCodec)
        c2.eng = fresh
        c2.vocab = [list(v) for v in codec.vocab]
        after = c2._parse_packed(*__import__("fdengine.ingest", fromlist=["pack"]).pack(msgs))
        for k in ("merchant", "payment_method", "transaction_type", "card_type", "card_key", "status"):
            np.testing.assert_array_equal(after[k], before[k])
        with pytest.raises(NativeError, match="same shard"):
            fresh.state_restore(path, 1, 2)
        fresh.state_init(1 << 12, 1, 8)
        fresh.state_restore(path, 1, 2, skip_sink=True)
    finally:
        fresh.close()
