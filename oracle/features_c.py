"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes wrapper of oracle_features.c."""
from __future__ import annotations

import ctypes as C

import numpy as np

RAW = 16
VEC = 64


def register(L) -> None:
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.orc_state_new.restype = vp
    L.orc_state_new.argtypes = [i64, i32, i32]
    L.orc_state_free.restype = None
    L.orc_state_free.argtypes = [vp]
    L.orc_state_load_users.restype = C.c_int
    L.orc_state_load_users.argtypes = [vp, i64, vp, vp, vp, vp]
    L.orc_state_load_merchants.restype = C.c_int
    L.orc_state_load_merchants.argtypes = [vp, i64, vp, vp]
    L.orc_features_run.restype = C.c_int
    L.orc_features_run.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.orc_features_run_ex.restype = C.c_int
    L.orc_features_run_ex.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.orc_vector_from_raw.restype = None
    L.orc_vector_from_raw.argtypes = [vp, vp]


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class OracleFeatureState:
    """Sequential CPU restatement of the card state + feature vector (see oracle_features.c)."""

    def __init__(self, capacity: int, window_mode: int = 0, ring_k: int = 16):
        from . import lib
        self.L = lib()
        cap = 1
        while cap < capacity:
            cap *= 2
        self.h = self.L.orc_state_new(cap, window_mode, ring_k)
        self.mode, self.K = int(window_mode), int(ring_k)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_state_free(self.h)
            self.h = None

    def load_users(self, keys, avg_amount, account_age, device_fp):
        keys, avg, age, fp = _c(keys, np.uint64), _c(avg_amount, np.float64), _c(account_age, np.int32), \
            _c(device_fp, np.uint64)
        assert self.L.orc_state_load_users(self.h, len(keys), keys.ctypes.data, avg.ctypes.data, age.ctypes.data,
                                           fp.ctypes.data) == 0

    def load_merchants(self, fraud_rate, risk_mult):
        fr, m = _c(fraud_rate, np.float64), _c(risk_mult, np.float64)
        assert self.L.orc_state_load_merchants(self.h, len(fr), fr.ctypes.data, m.ctypes.data) == 0

    def run_ex(self, txns: dict):
        """-> (raw [n,16], vectors [n,64], velocity_5min_amount [n])."""
        cols = [_c(txns["card_key"], np.uint64), _c(txns["ts_ms"], np.int64), _c(txns["amount_cents"], np.int64),
                _c(txns["merchant"], np.int32), _c(txns["device_fp"], np.uint64), _c(txns["ip_class"], np.uint8),
                _c(txns["hour"], np.uint8), _c(txns["weekend"], np.uint8)]
        n = len(cols[0])
        raw = np.empty((n, RAW), np.float64)
        vec = np.empty((n, VEC), np.float32)
        vel5 = np.empty(n, np.float64)
        rc = self.L.orc_features_run_ex(self.h, n, *[c.ctypes.data for c in cols], raw.ctypes.data, vec.ctypes.data,
                                        vel5.ctypes.data)
        assert rc == 0
        return raw, vec, vel5

    def run(self, txns: dict, want_raw: bool = True):
        cols = [_c(txns["card_key"], np.uint64), _c(txns["ts_ms"], np.int64), _c(txns["amount_cents"], np.int64),
                _c(txns["merchant"], np.int32), _c(txns["device_fp"], np.uint64), _c(txns["ip_class"], np.uint8),
                _c(txns["hour"], np.uint8), _c(txns["weekend"], np.uint8)]
        n = len(cols[0])
        raw = np.empty((n, RAW), np.float64) if want_raw else None
        vec = np.empty((n, VEC), np.float32)
        rc = self.L.orc_features_run(self.h, n, *[c.ctypes.data for c in cols],
                                     raw.ctypes.data if want_raw else None, vec.ctypes.data)
        assert rc == 0
        return raw, vec


def vector_from_raw(raw: np.ndarray) -> np.ndarray:
    from . import lib
    L = lib()
    raw = _c(raw, np.float64).reshape(-1, RAW)
    out = np.empty((len(raw), VEC), np.float32)
    for i in range(len(raw)):
        L.orc_vector_from_raw(raw[i].ctypes.data, out[i].ctypes.data)
    return out
