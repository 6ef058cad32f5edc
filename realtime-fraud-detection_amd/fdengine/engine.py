"""Thin object wrapper over the C-ABI (one FraudEngine per GPU).

Host-array calls (`predict`, `blend`) copy through engine-owned staging buffers; `*_device` calls
take device pointers (ints) so HBM-resident inputs (e.g. torch tensors' data_ptr()) are scored in
place. The engine never falls back to the CPU: every call goes through libfdengine.so.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Sequence

import numpy as np

from . import _native as N
from .forest import ForestArrays


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


class FraudEngine:
    def __init__(self, device: int = 0):
        h = C.c_void_p()
        N.call("fd_engine_create", int(device), C.byref(h))
        self._h = h
        self.device = int(device)
        self.forests: Dict[int, dict] = {}

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            N.call("fd_engine_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        """stream_ptr: a hipStream_t handle (torch.cuda.Stream.cuda_stream; 0 = the null/default
        stream). None restores the engine's own stream."""
        if stream_ptr is None:
            N.call("fd_engine_reset_stream", self._h)
        else:
            N.call("fd_engine_set_stream", self._h, C.c_void_p(int(stream_ptr)) if stream_ptr else None)

    def sync(self) -> None:
        N.call("fd_engine_sync", self._h)

    def set_timing(self, enable: bool) -> None:
        N.call("fd_engine_set_timing", self._h, 1 if enable else 0)

    def set_option(self, key: str, value: int) -> None:
        N.call("fd_engine_set_option", self._h, key.encode(), int(value))

    def counter(self, key: str) -> int:
        """fd_engine_get_counter: "pipelined_batches", "sharded_steps", "sharded_host_ns_<phase>" (include/fdengine.h)."""
        v = N._i64()
        N.call("fd_engine_get_counter", self._h, key.encode(), C.byref(v))
        return int(v.value)

    def read_timing(self, kinds=(N.FD_TIMING_XGB, N.FD_TIMING_IFOREST, N.FD_TIMING_FEATURES, N.FD_TIMING_BLEND,
                                 N.FD_TIMING_ROUTE, N.FD_TIMING_LSTM, N.FD_TIMING_WINDOWS, N.FD_TIMING_INGEST,
                                 N.FD_TIMING_ENSEMBLE),
                    reset: bool = True):
        """-> {kind: (total kernel ms, timed launches)} since the last reset (then resets).
        With a single int `kinds`, returns just that (ms, launches) pair."""
        single = isinstance(kinds, int)
        out = {}
        for k in ([kinds] if single else kinds):
            ms = C.c_double()
            cnt = C.c_int64()
            N.call("fd_timing_read", self._h, int(k), C.byref(ms), C.byref(cnt))
            out[k] = (ms.value, cnt.value)
        if reset:
            N.call("fd_timing_reset", self._h)
        return out[kinds] if single else out

    # ------------------------------------------------------------------ forests
    def load_forest(self, slot: int, fa: ForestArrays) -> None:
        p, t, keep = fa.c_structs()
        N.call("fd_load_forest", self._h, int(slot), C.byref(p), C.byref(t))
        del keep
        nt, d, nf = C.c_int32(), C.c_int32(), C.c_int32()
        N.call("fd_forest_info", self._h, int(slot), C.byref(nt), C.byref(d), C.byref(nf))
        self.forests[slot] = {"kind": fa.kind, "n_trees": nt.value, "depth": d.value, "num_feature": nf.value}

    def load_xgboost_file(self, slot: int, path) -> None:
        """The reference's XGBoost JSON model file, parsed by the engine itself (fd_load_xgboost_json)."""
        N.call("fd_load_xgboost_json", self._h, int(slot), os.fsencode(str(path)))
        nt, d, nf = C.c_int32(), C.c_int32(), C.c_int32()
        N.call("fd_forest_info", self._h, int(slot), C.byref(nt), C.byref(d), C.byref(nf))
        self.forests[slot] = {"kind": N.FD_FOREST_XGB_BINARY_LOGISTIC, "n_trees": nt.value, "depth": d.value,
                              "num_feature": nf.value}

    def unload_forest(self, slot: int) -> None:
        N.call("fd_unload_forest", self._h, int(slot))
        self.forests.pop(slot, None)

    def forest_info(self, slot: int) -> dict:
        if slot not in self.forests:
            raise ValueError(f"Model in slot {slot} not loaded")
        return dict(self.forests[slot])

    def predict(self, slot: int, X: np.ndarray, want_raw: bool = False, want_leaf: bool = False):
        """X: [n, ld] (cast to f32 as XGBoost's DMatrix / sklearn's validate_data do).
        -> prob f64 [n] (+ raw f64 [n], leaf int32 [n, T])."""
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float32))
        if X.ndim == 1:
            X = X.reshape(1, -1)
        n, ld = X.shape
        prob = np.empty(n, np.float64)
        raw = np.empty(n, np.float64) if want_raw else None
        T = self.forests.get(slot, {}).get("n_trees", 0)
        leaf = np.empty((n, T), np.int32) if want_leaf else None
        N.call("fd_forest_predict_host", self._h, int(slot), _ptr(X), n, ld, _ptr(prob), _ptr(raw), _ptr(leaf))
        out = [prob]
        if want_raw:
            out.append(raw)
        if want_leaf:
            out.append(leaf)
        return out[0] if len(out) == 1 else tuple(out)

    def predict_device(self, slot: int, X_ptr: int, n: int, ld: int, prob_ptr: int, raw_ptr: int = 0,
                       leaf_ptr: int = 0) -> None:
        N.call("fd_forest_predict_device", self._h, int(slot), C.c_void_p(X_ptr), int(n), int(ld),
               C.c_void_p(prob_ptr), C.c_void_p(raw_ptr) if raw_ptr else None,
               C.c_void_p(leaf_ptr) if leaf_ptr else None)

    # ------------------------------------------------------------------ card state + features
    _TXN_DTYPES = {"card_key": np.uint64, "ts_ms": np.int64, "amount_cents": np.int64, "merchant": np.int32,
                   "device_fp": np.uint64, "ip_class": np.uint8, "hour": np.uint8, "weekend": np.uint8}

    def state_init(self, capacity: int, window_mode: int = N.FD_WINDOW_REDIS_COMPAT, ring_k: int = 16,
                   seq_len: int = 0) -> None:
        """seq_len > 0 keeps each card's last seq_len events for the LSTM head (lstm_sequential)."""
        p = N.fd_state_params(int(capacity), int(window_mode), int(ring_k), int(seq_len))
        self.seq_len = int(seq_len)
        N.call("fd_state_init", self._h, C.byref(p))

    def state_clear(self) -> None:
        N.call("fd_state_clear", self._h)

    def state_info(self):
        cap, cards = C.c_int64(), C.c_int64()
        N.call("fd_state_info", self._h, C.byref(cap), C.byref(cards))
        return {"capacity": cap.value, "cards": cards.value}

    def load_users(self, key, avg_amount, account_age_days, device_fp) -> None:
        arr = [np.ascontiguousarray(key, np.uint64), np.ascontiguousarray(avg_amount, np.float64),
               np.ascontiguousarray(account_age_days, np.int32),
               np.ascontiguousarray(np.asarray(device_fp).reshape(-1, 3), np.uint64)]
        u = N.fd_users(len(arr[0]), *[a.ctypes.data for a in arr])
        N.call("fd_state_load_users_host", self._h, C.byref(u))

    def load_merchants(self, fraud_rate, risk_multiplier) -> None:
        arr = [np.ascontiguousarray(fraud_rate, np.float64), np.ascontiguousarray(risk_multiplier, np.float64)]
        m = N.fd_merchants(len(arr[0]), *[a.ctypes.data for a in arr])
        N.call("fd_load_merchants_host", self._h, C.byref(m))

    def features(self, txns: dict, want_raw: bool = False):
        """Host SoA batch (dict of arrays, arrival order) -> vectors f32 [n, 64] (+ raw f64 [n, 16])."""
        cols = [np.ascontiguousarray(txns[f], self._TXN_DTYPES[f]) for f in N.TXN_FIELDS]
        n = len(cols[0])
        vec = np.empty((n, N.FD_VECTOR_WIDTH), np.float32)
        raw = np.empty((n, N.FD_RAW_FEATURES), np.float64) if want_raw else None
        b = N.fd_txn_batch(*[c.ctypes.data for c in cols])
        N.call("fd_features_host", self._h, C.byref(b), n, _ptr(vec), _ptr(raw))
        return (vec, raw) if want_raw else vec

    def features_device(self, ptrs: dict, n: int, vec_ptr: int, raw_ptr: int = 0) -> None:
        """ptrs: field -> device pointer (see fdengine._native.TXN_FIELDS)."""
        b = N.fd_txn_batch(*[int(ptrs[f]) for f in N.TXN_FIELDS])
        N.call("fd_features_device", self._h, C.byref(b), int(n), C.c_void_p(vec_ptr),
               C.c_void_p(raw_ptr) if raw_ptr else None)

    def score_batch_device(self, params: N.fd_blend_params, slots: Sequence[int], txn_ptrs: dict, n: int,
                           fp_ptr: int, conf_ptr: int = 0, dec_ptr: int = 0, risk_ptr: int = 0,
                           vec_ptr: int = 0, model_probs_ptr: int = 0,
                           ext_ptrs: Optional[Sequence[Optional[int]]] = None,
                           present: Optional[Sequence[int]] = None) -> None:
        """Whole hot path for one device-resident micro-batch: features (card state updated) ->
        every forest model -> blend. All pointers are device pointers."""
        M = params.n_models
        sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        pres = np.array([1] * M if present is None else list(present), np.uint8)
        ext = (C.c_void_p * N.FD_MAX_MODELS)()
        if ext_ptrs:
            for i, p in enumerate(ext_ptrs):
                ext[i] = p if p else None
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        opt = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        N.call("fd_score_batch_device", self._h, C.byref(params), _ptr(sl), ext, _ptr(pres), C.byref(b), int(n),
               opt(vec_ptr), opt(model_probs_ptr), C.c_void_p(fp_ptr), opt(conf_ptr), opt(dec_ptr), opt(risk_ptr))

    def score_batch_pipelined(self, params: N.fd_blend_params, slots: Sequence[int], txn_ptrs: dict, n: int,
                              fp_ptr: int, conf_ptr: int = 0, dec_ptr: int = 0, risk_ptr: int = 0,
                              model_probs_ptr: int = 0, ext_ptrs: Optional[Sequence[Optional[int]]] = None,
                              present: Optional[Sequence[int]] = None, input_ready: int = 0,
                              vec_ptr: int = 0) -> None:
        """Streaming form of score_batch_device (fd_score_batch_pipelined): the batch's features run on the
        engine's feature stream, overlapping the previous batch's forests; outputs are ordered on the engine
        stream as with score_batch_device (written there by a copy from engine staging, so the caller may free
        them in that stream's order). input_ready: a hipEvent_t handle (e.g. torch.cuda.Event's cuda_event)
        recorded when the input columns were complete; 0 = complete before this call. The input columns must
        stay unchanged until the engine stream has passed the call."""
        M = params.n_models
        sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        pres = np.array([1] * M if present is None else list(present), np.uint8)
        ext = (C.c_void_p * N.FD_MAX_MODELS)()
        if ext_ptrs:
            for i, p in enumerate(ext_ptrs):
                ext[i] = p if p else None
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        opt = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        N.call("fd_score_batch_pipelined", self._h, C.byref(params), _ptr(sl), ext, _ptr(pres), C.byref(b),
               int(n), opt(vec_ptr), opt(model_probs_ptr), C.c_void_p(fp_ptr), opt(conf_ptr), opt(dec_ptr),
               opt(risk_ptr), opt(input_ready))

    def pipelined_scorer(self, params: N.fd_blend_params, slots: Sequence[int],
                         present: Optional[Sequence[int]] = None) -> "PipelinedScorer":
        """A prepared score_batch_pipelined for a fixed model set: per call only the batch's pointers change
        (the per-step host cost stays well below the GPU step)."""
        return PipelinedScorer(self, params, slots, present)

    def batch_scorer(self, params: N.fd_blend_params, slots: Sequence[int],
                     present: Optional[Sequence[int]] = None) -> "PipelinedScorer":
        """The same prepared call over score_batch_device (one stream; small latency batches, where the
        per-call host cost is the step's bound)."""
        return PipelinedScorer(self, params, slots, present, pipelined=False)

    def features_seq_device(self, ptrs: dict, n: int, vec_ptr: int, seq_ptr: int, raw_ptr: int = 0) -> None:
        """features_device plus each transaction's LSTM input sequence (n x seq_len x 16 f32)."""
        b = N.fd_txn_batch(*[int(ptrs[f]) for f in N.TXN_FIELDS])
        N.call("fd_features_seq_device", self._h, C.byref(b), int(n), C.c_void_p(vec_ptr),
               C.c_void_p(raw_ptr) if raw_ptr else None, C.c_void_p(seq_ptr) if seq_ptr else None)

    # ------------------------------------------------------------------ full feature map + rule scores
    _USER_EXT_DT = {"risk_score": np.float64, "kyc_status": np.uint8, "verified": np.uint8, "pref_start": np.int8,
                    "pref_end": np.int8, "weekend_activity": np.float64, "online_preference": np.float64,
                    "intl_preference": np.float64, "txn_frequency": np.int32, "has_patterns": np.uint8}
    _MERCH_EXT_DT = {"avg_amount": np.float64, "risk_level": np.uint8, "blacklisted": np.uint8, "category": np.uint8,
                     "high_risk_category": np.uint8, "open_hour": np.uint8, "close_hour": np.uint8,
                     "suspicious_name": np.uint8}

    def load_users_ext(self, key, **fields) -> None:
        """Extended UserProfile fields (fd_users_ext); omitted fields are null."""
        keep = {"key": np.ascontiguousarray(key, np.uint64)}
        for f, dt in self._USER_EXT_DT.items():
            if fields.get(f) is not None:
                keep[f] = np.ascontiguousarray(fields[f], dt)
        u = N.fd_users_ext(len(keep["key"]), keep["key"].ctypes.data,
                           *[keep[f].ctypes.data if f in keep else None for f in N.USER_EXT_FIELDS])
        N.call("fd_state_load_users_ext_host", self._h, C.byref(u))

    def load_merchants_ext(self, n: int, **fields) -> None:
        keep = {f: np.ascontiguousarray(fields[f], dt) for f, dt in self._MERCH_EXT_DT.items()
                if fields.get(f) is not None}
        m = N.fd_merchants_ext(int(n), *[keep[f].ctypes.data if f in keep else None for f in N.MERCHANT_EXT_FIELDS])
        N.call("fd_load_merchants_ext_host", self._h, C.byref(m))

    def load_vocab(self, payment_high_risk, type_is_refund) -> None:
        a = np.ascontiguousarray(payment_high_risk, np.uint8)
        b = np.ascontiguousarray(type_is_refund, np.uint8)
        assert len(a) == 256 and len(b) == 256
        N.call("fd_load_vocab_host", self._h, _ptr(a), _ptr(b))

    def features_full_device(self, txn_ptrs: dict, ctx_ptrs: Optional[dict], n: int, vec_ptr: int, fmap_ptr: int = 0,
                             rules_ptr: int = 0, raw_ptr: int = 0) -> None:
        """features_device plus the 64-wide FeatureExtractor map (f64) and the rule scores
        (N.RULE_DTYPE records); ctx_ptrs: field -> device pointer (N.CTX_FIELDS), missing = null."""
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        cx = N.fd_txn_context(*[int(ctx_ptrs[f]) if ctx_ptrs and ctx_ptrs.get(f) else None for f in N.CTX_FIELDS])
        opt = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        N.call("fd_features_full_device", self._h, C.byref(b), C.byref(cx), int(n), C.c_void_p(vec_ptr), opt(raw_ptr),
               opt(fmap_ptr), opt(rules_ptr))

    # ------------------------------------------------------------------ Flink window aggregates (a5)
    def windows_init(self, log_capacity: int, max_out_of_orderness_ms: int = 10000) -> None:
        """WindowProcessor's user-velocity (sliding 5 min / 1 min) and merchant (tumbling 1 h) windows
        (fl/windows/WindowProcessor.java:36-66); needs state_init (cards are keyed by its table)."""
        p = N.fd_window_params(int(log_capacity), int(max_out_of_orderness_ms))
        N.call("fd_windows_init", self._h, C.byref(p))

    def _windows_out(self, user_cap: int, merchant_cap: int):
        uo = np.zeros(max(int(user_cap), 1), N.USER_WINDOW_DTYPE)
        mo = np.zeros(max(int(merchant_cap), 1), N.MERCHANT_WINDOW_DTYPE)
        return uo, mo

    def windows_step_host(self, key, ts_ms, amount_cents, merchant, payment_method=None, is_fraud=None,
                          fraud_score=None, flush: bool = False, user_cap: int = 0, merchant_cap: int = 0):
        """Add one micro-batch (host arrays) and return (user windows, merchant windows) fired by it
        as numpy record arrays (N.USER_WINDOW_DTYPE / N.MERCHANT_WINDOW_DTYPE)."""
        n = len(key)
        keep = [np.ascontiguousarray(key, np.uint64), np.ascontiguousarray(ts_ms, np.int64),
                np.ascontiguousarray(amount_cents, np.int64), np.ascontiguousarray(merchant, np.int32)]
        b = N.fd_txn_batch(*[a.ctypes.data for a in keep], None, None, None, None)
        ins = [None if a is None else np.ascontiguousarray(a, dt)
               for a, dt in ((payment_method, np.uint8), (is_fraud, np.uint8), (fraud_score, np.float64))]
        wi = N.fd_window_inputs(*[None if a is None else a.ctypes.data for a in ins])
        held = self.windows_stats()
        ucap = user_cap or 5 * (n + held["user_events"]) + 16   # each event is in at most 5 user windows
        mcap = merchant_cap or n + held["merchant_events"] + 16
        uo, mo = self._windows_out(ucap, mcap)
        nu, nm = C.c_int64(), C.c_int64()
        N.call("fd_windows_step_host", self._h, C.byref(b), C.byref(wi), int(n), int(bool(flush)),
               uo.ctypes.data, int(ucap), C.byref(nu), mo.ctypes.data, int(mcap), C.byref(nm))
        return uo[:nu.value].copy(), mo[:nm.value].copy()

    def windows_step_device(self, txn_ptrs: dict, n: int, in_ptrs: Optional[dict] = None, flush: bool = False,
                            user_cap: int = 0, merchant_cap: int = 0):
        """Device-resident variant: txn_ptrs as features_device; in_ptrs: payment_method / is_fraud /
        fraud_score device pointers (missing = null)."""
        b = N.fd_txn_batch(*[int(txn_ptrs.get(f) or 0) or None for f in N.TXN_FIELDS])
        wi = N.fd_window_inputs(*[int(in_ptrs[f]) if in_ptrs and in_ptrs.get(f) else None
                                  for f in ("payment_method", "is_fraud", "fraud_score")])
        held = self.windows_stats()
        ucap = user_cap or 5 * (n + held["user_events"]) + 16   # each event is in at most 5 user windows
        mcap = merchant_cap or n + held["merchant_events"] + 16
        uo, mo = self._windows_out(ucap, mcap)
        nu, nm = C.c_int64(), C.c_int64()
        N.call("fd_windows_step_device", self._h, C.byref(b), C.byref(wi), int(n), int(bool(flush)),
               uo.ctypes.data, int(ucap), C.byref(nu), mo.ctypes.data, int(mcap), C.byref(nm))
        return uo[:nu.value].copy(), mo[:nm.value].copy()

    def windows_stats(self) -> dict:
        wm, ue, me = C.c_int64(), C.c_int64(), C.c_int64()
        N.call("fd_windows_stats", self._h, C.byref(wm), C.byref(ue), C.byref(me))
        return {"watermark": wm.value, "user_events": ue.value, "merchant_events": me.value}

    def windows_observe(self, max_event_ts: int) -> None:
        """Sharded windows: the node-wide micro-batch's largest event time (all-reduce MAX), so every shard
        advances one watermark (fd_windows_observe)."""
        N.call("fd_windows_observe", self._h, int(max_event_ts))

    # ------------------------------------------------------------------ RedisTransactionSink aggregates
    def sink_init(self, capacity: int, user_capacity: int) -> None:
        """Hourly / daily / merchant-hour summaries of RedisTransactionSink.updateAggregations
        (fl/sinks/RedisTransactionSink.java:140-262), HBM-resident."""
        p = N.fd_sink_params(int(capacity), int(user_capacity))
        N.call("fd_sink_init", self._h, C.byref(p))

    def sink_update_host(self, key, ts_ms, amount_cents, merchant, is_fraud=None, fraud_score=None) -> None:
        keep = [np.ascontiguousarray(key, np.uint64), np.ascontiguousarray(ts_ms, np.int64),
                np.ascontiguousarray(amount_cents, np.int64), np.ascontiguousarray(merchant, np.int32)]
        b = N.fd_txn_batch(*[a.ctypes.data for a in keep], None, None, None, None)
        fr = None if is_fraud is None else np.ascontiguousarray(is_fraud, np.uint8)
        fs = None if fraud_score is None else np.ascontiguousarray(fraud_score, np.float64)
        wi = N.fd_window_inputs(None, None if fr is None else fr.ctypes.data, None if fs is None else fs.ctypes.data)
        N.call("fd_sink_update_host", self._h, C.byref(b), C.byref(wi), len(keep[0]))

    def sink_update_device(self, txn_ptrs: dict, n: int, in_ptrs: Optional[dict] = None) -> None:
        b = N.fd_txn_batch(*[int(txn_ptrs.get(f) or 0) or None for f in N.TXN_FIELDS])
        wi = N.fd_window_inputs(None, *[int(in_ptrs[f]) if in_ptrs and in_ptrs.get(f) else None
                                        for f in ("is_fraud", "fraud_score")])
        N.call("fd_sink_update_device", self._h, C.byref(b), C.byref(wi), int(n))

    def sink_query(self, kind: int, buckets, merchants=None) -> np.ndarray:
        """RedisService.getAggregation for hourly / daily (bucket) or merchant (merchant, hour) keys."""
        bk = np.ascontiguousarray(buckets, np.int64)
        mk = None if merchants is None else np.ascontiguousarray(merchants, np.int32)
        out = np.zeros(len(bk), N.AGGREGATE_DTYPE)
        N.call("fd_sink_query_host", self._h, int(kind), _ptr(bk) if len(bk) else None,
               _ptr(mk) if mk is not None and len(mk) else None, len(bk), out.ctypes.data if len(bk) else None)
        return out

    def sink_evict_before(self, hour_key: int):
        a, b = C.c_int64(), C.c_int64()
        N.call("fd_sink_evict_before", self._h, int(hour_key), C.byref(a), C.byref(b))
        return a.value, b.value

    # ------------------------------------------------------------------ state snapshot / restore
    def state_snapshot(self, path, shard: int = 0, n_shards: int = 1) -> int:
        """Durable key-addressed image of the HBM keyed state (+ replicated tables, window logs);
        Flink keyed-state checkpoint / Redis RDB counterpart. Returns the bytes written."""
        nb = C.c_int64()
        N.call("fd_state_snapshot", self._h, os.fsencode(str(path)), int(shard), int(n_shards), C.byref(nb))
        return nb.value

    def state_restore(self, path, shard: int = 0, n_shards: int = 1, skip_windows: bool = False,
                      skip_sink: bool = False) -> int:
        """Re-insert an image's cards owned by `shard` of `n_shards` (any table capacity); returns the
        number of cards restored. Restore every old shard's image on each new shard to re-shard."""
        nc = C.c_int64()
        N.call("fd_state_restore", self._h, os.fsencode(str(path)), int(shard), int(n_shards),
               (N.FD_RESTORE_SKIP_WINDOWS if skip_windows else 0) | (N.FD_RESTORE_SKIP_SINK if skip_sink else 0),
               C.byref(nc))
        return nc.value

    # ------------------------------------------------------------------ LSTM head
    def load_lstm(self, model) -> None:
        """model: fdengine.lstm.LstmWeights (PyTorch layout, f32)."""
        keep = [np.ascontiguousarray(a, np.float32) if a is not None else None
                for a in (model.w_ih, model.w_hh, model.b_ih, model.b_hh, model.w_out, model.b_out)]
        ptr = [a.ctypes.data if a is not None else None for a in keep]
        p = N.fd_lstm_params(int(model.input_size), int(model.hidden), int(model.n_out), *ptr)
        N.call("fd_load_lstm", self._h, C.byref(p))
        self.lstm_info = {"input_size": model.input_size, "hidden": model.hidden, "n_out": model.n_out}

    def unload_lstm(self) -> None:
        N.call("fd_unload_lstm", self._h)
        self.lstm_info = None

    def lstm_predict(self, seq: np.ndarray) -> np.ndarray:
        """seq: [n, T, 16] (or [n, T, input_size], zero-padded here) -> P(fraud) f64 [n]."""
        seq = np.asarray(seq, np.float32)
        if seq.ndim != 3:
            raise ValueError(f"LSTM input must be [n, T, features], got shape {seq.shape}")
        n, T, I = seq.shape
        if I < N.FD_SEQ_INPUT:
            seq = np.concatenate([seq, np.zeros((n, T, N.FD_SEQ_INPUT - I), np.float32)], axis=2)
        seq = np.ascontiguousarray(seq)
        prob = np.empty(n, np.float64)
        N.call("fd_lstm_predict_host", self._h, _ptr(seq), n, T, _ptr(prob))
        return prob

    def lstm_predict_device(self, seq_ptr: int, n: int, T: int, prob_ptr: int) -> None:
        N.call("fd_lstm_predict_device", self._h, C.c_void_p(seq_ptr), int(n), int(T), C.c_void_p(prob_ptr))

    # ------------------------------------------------------------------ card-hash sharding (fdengine/sharding.py)
    def route_partition_device(self, txn_ptrs: dict, n: int, n_shards: int, records_ptr: int, counts_ptr: int) -> None:
        """Group one device-resident micro-batch by owner GPU: n records of FD_ROUTE_RECORD_BYTES at
        records_ptr (owner-major, arrival order kept), n_shards int64 counts at counts_ptr."""
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        N.call("fd_route_partition_device", self._h, C.byref(b), int(n), int(n_shards),
               C.c_void_p(records_ptr) if records_ptr else None, C.c_void_p(counts_ptr))

    def route_partition_ex_device(self, txn_ptrs: dict, extra_ptrs: Optional[dict], n: int, n_shards: int,
                                  records_ptr: int, counts_ptr: int) -> None:
        """route_partition_device with the owner's window / sink inputs riding in the records:
        extra_ptrs = {"payment_method": u8*, "is_fraud": u8*} device pointers (missing: null / false)."""
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        wi = N.fd_window_inputs(*[int(extra_ptrs[f]) if extra_ptrs and extra_ptrs.get(f) else None
                                  for f in ("payment_method", "is_fraud")], None)
        N.call("fd_route_partition_ex_device", self._h, C.byref(b), C.byref(wi), int(n), int(n_shards),
               C.c_void_p(records_ptr) if records_ptr else None, C.c_void_p(counts_ptr))

    def route_partition_stream(self, txn_ptrs: dict, extra_ptrs: Optional[dict], n: int, n_shards: int,
                               records_ptr: int, counts_ptr: int, stream_ptr: int) -> None:
        """route_partition_ex_device launched on `stream_ptr` (a hipStream_t), beside the pipelined stream."""
        b = N.fd_txn_batch(*[int(txn_ptrs[f]) for f in N.TXN_FIELDS])
        wi = N.fd_window_inputs(*[int(extra_ptrs[f]) if extra_ptrs and extra_ptrs.get(f) else None
                                  for f in ("payment_method", "is_fraud")], None)
        N.call("fd_route_partition_stream", self._h, C.byref(b), C.byref(wi), int(n), int(n_shards),
               C.c_void_p(records_ptr) if records_ptr else None, C.c_void_p(counts_ptr),
               C.c_void_p(int(stream_ptr)) if stream_ptr else None)

    def route_unpack_device(self, records_ptr: int, results_ptr: int, n: int, out_ptrs: dict, pm_ptr: int = 0,
                            fraud_ptr: int = 0, score_ptr: int = 0) -> None:
        """Owner side: received records (+ their result records) back to device columns (out_ptrs: any of
        TXN_FIELDS), payment method, isFraud and the fraud score (the result's fraud probability)."""
        opt = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        b = N.fd_txn_batch(*[int(out_ptrs.get(f) or 0) or None for f in N.TXN_FIELDS])
        N.call("fd_route_unpack_device", self._h, opt(records_ptr), opt(results_ptr), int(n), C.byref(b),
               opt(pm_ptr), opt(fraud_ptr), opt(score_ptr))

    def score_records_device(self, params: N.fd_blend_params, slots: Sequence[int], records_ptr: int, n: int,
                             results_ptr: int, present: Optional[Sequence[int]] = None) -> None:
        """Owner side: features (this GPU's card state) -> forests -> blend over n received records;
        n result records of FD_RESULT_RECORD_BYTES at results_ptr."""
        M = params.n_models
        sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        pres = np.array([1] * M if present is None else list(present), np.uint8)
        N.call("fd_score_records_device", self._h, C.byref(params), _ptr(sl), _ptr(pres),
               C.c_void_p(records_ptr) if records_ptr else None, int(n),
               C.c_void_p(results_ptr) if results_ptr else None)

    def score_records_pipelined(self, params: N.fd_blend_params, slots: Sequence[int], records_ptr: int, n: int,
                                results_ptr: int, input_ready: int = 0, present: Optional[Sequence[int]] = None) -> None:
        """Streaming form of score_records_device (fd_score_records_pipelined): the owner's features of this batch
        overlap the previous batch's forests; input_ready: a hipEvent_t recorded once the records had landed."""
        M = params.n_models
        sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        pres = np.array([1] * M if present is None else list(present), np.uint8)
        N.call("fd_score_records_pipelined", self._h, C.byref(params), _ptr(sl), _ptr(pres),
               C.c_void_p(records_ptr) if records_ptr else None, int(n),
               C.c_void_p(results_ptr) if results_ptr else None, C.c_void_p(input_ready) if input_ready else None)

    # ---- card-hash sharding over the engine's own RCCL communicators (fd_comm_* / fd_sharded_step)
    @staticmethod
    def comm_unique_id(rccl_path: str) -> bytes:
        buf = (C.c_uint8 * 128)()
        N.call("fd_comm_unique_id", os.fsencode(rccl_path), C.cast(buf, C.c_void_p))
        return bytes(buf)

    def comm_init(self, rccl_path: str, rank: int, world: int, id_fwd: bytes, id_back: bytes) -> None:
        a = (C.c_uint8 * 128).from_buffer_copy(id_fwd)
        b = (C.c_uint8 * 128).from_buffer_copy(id_back)
        N.call("fd_comm_init", self._h, os.fsencode(rccl_path), int(rank), int(world), C.cast(a, C.c_void_p),
               C.cast(b, C.c_void_p))

    def comm_destroy(self) -> None:
        N.call("fd_comm_destroy", self._h)

    def sharded_scorer(self, params: N.fd_blend_params, slots: Sequence[int],
                       present: Optional[Sequence[int]] = None) -> "ShardedStep":
        """fd_sharded_step with its model arguments marshalled once"""
        return ShardedStep(self, params, slots, present)

    def route_scatter_results_device(self, results_ptr: int, n: int, fp_ptr: int, conf_ptr: int = 0,
                                     dec_ptr: int = 0, risk_ptr: int = 0) -> None:
        """Ingest side: put the n returned result records back in micro-batch order."""
        opt = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        N.call("fd_route_scatter_results_device", self._h, opt(results_ptr), int(n), opt(fp_ptr), opt(conf_ptr),
               opt(dec_ptr), opt(risk_ptr))

    # ------------------------------------------------------------------ blend
    @staticmethod
    def blend_params(weights: Sequence[float], conf_mult: Sequence[float], strategy: int = 0,
                     fraud_threshold: float = 0.5, confidence_threshold: float = 0.7) -> N.fd_blend_params:
        p = N.fd_blend_params()
        p.n_models = len(weights)
        p.strategy = int(strategy)
        for i, (w, m) in enumerate(zip(weights, conf_mult)):
            p.weight[i] = float(w)
            p.conf_mult[i] = float(m)
        p.fraud_threshold = float(fraud_threshold)
        p.confidence_threshold = float(confidence_threshold)
        return p

    def blend(self, params: N.fd_blend_params, probs: Sequence[Optional[np.ndarray]]):
        """probs[m]: f64 [n] or None (model failed -> dropped). -> (fraud_prob, confidence, decision u8, risk u8)."""
        M = params.n_models
        assert len(probs) == M
        n = next((len(p) for p in probs if p is not None), 0)
        cols = [None if p is None else np.ascontiguousarray(p, dtype=np.float64) for p in probs]
        present = np.array([0 if c is None else 1 for c in cols], np.uint8)
        arr = (C.c_void_p * N.FD_MAX_MODELS)()
        for i, c in enumerate(cols):
            arr[i] = None if c is None else c.ctypes.data
        fp = np.empty(n, np.float64)
        conf = np.empty(n, np.float64)
        dec = np.empty(n, np.uint8)
        risk = np.empty(n, np.uint8)
        N.call("fd_blend_host", self._h, C.byref(params), n, arr, _ptr(present), _ptr(fp), _ptr(conf),
               _ptr(dec), _ptr(risk))
        return fp, conf, dec, risk

    def score_matrix(self, params: N.fd_blend_params, slots: Sequence[int], X: np.ndarray,
                     ext_probs: Optional[Sequence[Optional[np.ndarray]]] = None,
                     present: Optional[Sequence[int]] = None):
        """Every forest model (slots[m] >= 0) scores X, external columns fill the rest, then blend.
        -> (model_probs [M, n] f64, fraud_prob, confidence, decision u8, risk u8)."""
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float32))
        n, ld = X.shape
        M = params.n_models
        sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        pres = np.array([1] * M if present is None else list(present), np.uint8)
        ext = (C.c_void_p * N.FD_MAX_MODELS)()
        keep = []
        for m in range(M):
            if sl[m] < 0 and pres[m]:
                col = np.ascontiguousarray(ext_probs[m], dtype=np.float64)
                keep.append(col)
                ext[m] = col.ctypes.data
        mp = np.empty((M, n), np.float64)
        fp = np.empty(n, np.float64)
        conf = np.empty(n, np.float64)
        dec = np.empty(n, np.uint8)
        risk = np.empty(n, np.uint8)
        N.call("fd_score_matrix_host", self._h, C.byref(params), _ptr(sl), ext, _ptr(pres), _ptr(X), n, ld,
               _ptr(mp), _ptr(fp), _ptr(conf), _ptr(dec), _ptr(risk))
        return mp, fp, conf, dec, risk

    def blend_device(self, params: N.fd_blend_params, n: int, prob_ptrs: Sequence[Optional[int]],
                     fp_ptr: int, conf_ptr: int = 0, dec_ptr: int = 0, risk_ptr: int = 0) -> None:
        present = np.array([0 if p is None else 1 for p in prob_ptrs], np.uint8)
        arr = (C.c_void_p * N.FD_MAX_MODELS)()
        for i, p in enumerate(prob_ptrs):
            arr[i] = p if p else None
        N.call("fd_blend_device", self._h, C.byref(params), int(n), arr, _ptr(present), C.c_void_p(fp_ptr),
               C.c_void_p(conf_ptr) if conf_ptr else None, C.c_void_p(dec_ptr) if dec_ptr else None,
               C.c_void_p(risk_ptr) if risk_ptr else None)


def pack_forest_host(fa: ForestArrays):
    """Host-only repack (no GPU): -> (blob bytes, leaf_ids int32, fd_pack_info)."""
    p, t, keep = fa.c_structs()
    info = N.fd_pack_info()
    N.call("fd_pack_forest_host", C.byref(p), C.byref(t), None, 0, None, 0, C.byref(info))
    blob = np.empty(info.blob_bytes, np.uint8)
    ids = np.empty(info.n_leaf_ids, np.int32)
    N.call("fd_pack_forest_host", C.byref(p), C.byref(t), C.c_void_p(blob.ctypes.data), info.blob_bytes,
           C.c_void_p(ids.ctypes.data), info.n_leaf_ids, C.byref(info))
    del keep
    return blob.tobytes(), ids, info


def pack_forest_binned_host(fa: ForestArrays):
    """Host-only binned repack (no GPU): -> (blob bytes, thresholds f32, offsets int32, fd_pack_info).
    Raises NativeError(FD_ERR_UNSUPPORTED) when a feature has more than 65534 distinct thresholds."""
    p, t, keep = fa.c_structs()
    info = N.fd_pack_info()
    N.call("fd_pack_forest_binned_host", C.byref(p), C.byref(t), None, 0, None, 0, None, C.byref(info))
    blob = np.empty(info.blob_bytes, np.uint8)
    thr = np.empty(info.n_thresholds, np.float32)
    off = np.empty(fa.num_feature + 1, np.int32)
    N.call("fd_pack_forest_binned_host", C.byref(p), C.byref(t), C.c_void_p(blob.ctypes.data), info.blob_bytes,
           C.c_void_p(thr.ctypes.data), info.n_thresholds, C.c_void_p(off.ctypes.data), C.byref(info))
    del keep
    return blob.tobytes(), thr, off, info


def read_xgboost_json_native(path) -> ForestArrays:
    """Host-only: the engine's C++ reader of the XGBoost JSON file (fd_xgboost_json_read), as ForestArrays."""
    p = N.fd_forest_params()
    nt, nn = C.c_int32(), C.c_int64()
    N.call("fd_xgboost_json_read", os.fsencode(str(path)), C.byref(p), C.byref(nt), C.byref(nn), None)
    T, M = nt.value, nn.value
    fa = ForestArrays(kind=p.kind, num_feature=p.num_feature, offsets=np.zeros(T + 1, np.int64),
                      left=np.zeros(M, np.int32), right=np.zeros(M, np.int32), feature=np.zeros(M, np.int32),
                      threshold=np.zeros(M, np.float64), default_left=np.zeros(M, np.uint8),
                      leaf_value=np.zeros(M, np.float64), base_score=p.base_score)
    _, t, keep = fa.c_structs()
    N.call("fd_xgboost_json_read", os.fsencode(str(path)), C.byref(p), C.byref(nt), C.byref(nn), C.byref(t))
    out = ForestArrays(kind=fa.kind, num_feature=fa.num_feature, offsets=keep["offsets"], left=keep["left"],
                       right=keep["right"], feature=keep["feature"], threshold=keep["threshold"],
                       default_left=keep["default_left"], leaf_value=keep["leaf_value"], base_score=p.base_score)
    return out


def shard_of(keys, n_shards: int) -> np.ndarray:
    """Owner shard of each card key (host-only, no GPU): the partition fd_route_partition_device uses."""
    k = np.ascontiguousarray(keys, np.uint64)
    out = np.empty(len(k), np.int32)
    N.call("fd_shard_of_host", _ptr(k), len(k), int(n_shards), _ptr(out))
    return out


def device_count() -> int:
    c = C.c_int()
    rc = N.lib.fd_device_count(C.byref(c))
    return c.value if rc == N.FD_OK else 0


def merge_merchant_windows(parts) -> np.ndarray:
    """Combine merchant-window partials of several shards (N.MERCHANT_WINDOW_DTYPE arrays) into whole windows,
    sorted by (window_start, merchant): exact moments summed, derived fields recomputed by the library's own
    finalisation (fd_merchant_windows_merge, host only), so the result is bit-identical to an unsharded run."""
    a = np.concatenate([np.asarray(p, N.MERCHANT_WINDOW_DTYPE) for p in parts]) if len(parts) else \
        np.zeros(0, N.MERCHANT_WINDOW_DTYPE)
    a = np.ascontiguousarray(a)
    out = np.zeros(max(len(a), 1), N.MERCHANT_WINDOW_DTYPE)
    m = C.c_int64()
    N.call("fd_merchant_windows_merge", a.ctypes.data if len(a) else None, len(a), out.ctypes.data, C.byref(m))
    return out[:m.value].copy()


class PipelinedScorer:
    """fd_score_batch_pipelined (or, pipelined=False, fd_score_batch_device) with its model arguments marshalled
    once (FraudEngine.pipelined_scorer / batch_scorer)."""

    def __init__(self, eng: FraudEngine, params: N.fd_blend_params, slots: Sequence[int],
                 present: Optional[Sequence[int]] = None, pipelined: bool = True):
        M = params.n_models
        self.eng = eng
        self.params = params
        self._sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        self._pres = np.array([1] * M if present is None else list(present), np.uint8)
        self._ext = (C.c_void_p * N.FD_MAX_MODELS)()
        self._batch = N.fd_txn_batch()
        self.pipelined = pipelined
        self._fn = N.lib.fd_score_batch_pipelined if pipelined else N.lib.fd_score_batch_device
        self._args = [C.byref(params), _ptr(self._sl), self._ext, _ptr(self._pres), C.byref(self._batch)]

    def __call__(self, txn_ptrs: dict, n: int, fp_ptr: int, conf_ptr: int = 0, dec_ptr: int = 0, risk_ptr: int = 0,
                 input_ready: int = 0, vec_ptr: int = 0, model_probs_ptr: int = 0) -> None:
        b = self._batch
        for f in N.TXN_FIELDS:
            setattr(b, f, txn_ptrs[f])
        if self.pipelined:
            rc = self._fn(self.eng._h, *self._args, int(n), vec_ptr or None, model_probs_ptr or None, fp_ptr,
                          conf_ptr or None, dec_ptr or None, risk_ptr or None, input_ready or None)
            N.check(rc, "fd_score_batch_pipelined")
        else:
            rc = self._fn(self.eng._h, *self._args, int(n), vec_ptr or None, model_probs_ptr or None, fp_ptr,
                          conf_ptr or None, dec_ptr or None, risk_ptr or None)
            N.check(rc, "fd_score_batch_device")


class ShardedStep:
    """fd_sharded_step for a fixed model set (FraudEngine.sharded_scorer): per call only the batch pointers change.
    batch_id / next_id: the C-ABI's prefetch ids (include/fdengine.h): next_id (nonzero) names the prefetched batch,
    the call that scores it passes it as batch_id; 0 = not the prefetched batch."""

    def __init__(self, eng: FraudEngine, params: N.fd_blend_params, slots: Sequence[int],
                 present: Optional[Sequence[int]] = None):
        M = params.n_models
        self.eng, self.params = eng, params
        self._sl = np.array(list(slots) + [-1] * (N.FD_MAX_MODELS - len(slots)), np.int32)
        self._pres = np.array([1] * M if present is None else list(present), np.uint8)
        self._cur, self._next = N.fd_txn_batch(), N.fd_txn_batch()
        self.split_sizes = np.zeros(2 * 64, np.int64)
        self._fn = N.lib.fd_sharded_step

    def __call__(self, txn_ptrs: dict, n: int, fp_ptr: int, conf_ptr: int, dec_ptr: int, risk_ptr: int,
                 input_ready: int = 0, next_ptrs: Optional[dict] = None, next_n: int = 0, next_ready: int = 0,
                 batch_id: int = 0, next_id: int = 0) -> None:
        for f in N.TXN_FIELDS:
            setattr(self._cur, f, txn_ptrs[f])
        nxt = None
        if next_ptrs is not None:
            for f in N.TXN_FIELDS:
                setattr(self._next, f, next_ptrs[f])
            nxt = C.byref(self._next)
        rc = self._fn(self.eng._h, C.byref(self.params), self._sl.ctypes.data, self._pres.ctypes.data,
                      C.byref(self._cur), int(n), int(batch_id), input_ready or None, nxt, int(next_n), int(next_id),
                      next_ready or None, fp_ptr or None, conf_ptr or None, dec_ptr or None, risk_ptr or None,
                      self.split_sizes.ctypes.data)
        N.check(rc, "fd_sharded_step")
