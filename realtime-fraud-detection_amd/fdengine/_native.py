"""ctypes binding of libfdengine.so (the C-ABI declared in include/fdengine.h).

The product path has exactly one implementation: the HIP library. If it is missing this module
raises at import time — there is no CPU fallback (the CPU restatement under oracle/ is test
infrastructure only and is never imported from here).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # realtime-fraud-detection_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ.get("FDENGINE_LIB", PKG_ROOT / "lib" / "libfdengine.so"))

FD_OK = 0
FD_ERR_INVALID_ARG = 1
FD_ERR_HIP = 2
FD_ERR_NOT_LOADED = 3
FD_ERR_UNSUPPORTED = 4
FD_ERR_OOM = 5
FD_ERR_IO = 6
FD_RESTORE_SKIP_WINDOWS = 1
FD_RESTORE_SKIP_SINK = 2

FD_FOREST_XGB_BINARY_LOGISTIC = 1
FD_FOREST_SKLEARN_IFOREST = 2

FD_MAX_MODELS = 8
FD_BLEND_WEIGHTED_AVERAGE = 0
FD_BLEND_VOTING = 1
FD_BLEND_STACKING = 2

DECISIONS = ("APPROVE", "REVIEW", "DECLINE", "APPROVE_WITH_MONITORING")
RISK_LEVELS = ("VERY_LOW", "LOW", "MEDIUM", "HIGH", "CRITICAL")


class fd_tree_arrays(C.Structure):
    _fields_ = [
        ("n_trees", C.c_int32),
        ("tree_offsets", C.POINTER(C.c_int64)),
        ("left", C.POINTER(C.c_int32)),
        ("right", C.POINTER(C.c_int32)),
        ("feature", C.POINTER(C.c_int32)),
        ("threshold", C.POINTER(C.c_double)),
        ("default_left", C.POINTER(C.c_uint8)),
        ("leaf_value", C.POINTER(C.c_double)),
    ]


class fd_forest_params(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("num_feature", C.c_int32),
        ("base_score", C.c_double),
        ("if_offset", C.c_double),
        ("if_denominator", C.c_double),
    ]


class fd_blend_params(C.Structure):
    _fields_ = [
        ("n_models", C.c_int32),
        ("strategy", C.c_int32),
        ("weight", C.c_double * FD_MAX_MODELS),
        ("conf_mult", C.c_double * FD_MAX_MODELS),
        ("fraud_threshold", C.c_double),
        ("confidence_threshold", C.c_double),
    ]


class fd_pack_info(C.Structure):
    _fields_ = [
        ("n_trees", C.c_int32),
        ("n_chunks", C.c_int32),
        ("chunk", C.c_int32),
        ("depth", C.c_int32),
        ("tree_bytes", C.c_int64),
        ("chunk_stride", C.c_int64),
        ("blob_bytes", C.c_int64),
        ("n_leaf_ids", C.c_int64),
        ("base_margin", C.c_float),
        ("layout", C.c_int32),
        ("n_thresholds", C.c_int64),
        ("bin_steps", C.c_int32),
    ]


class fd_state_params(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("window_mode", C.c_int32), ("ring_k", C.c_int32), ("seq_len", C.c_int32)]


class fd_txn_context(C.Structure):
    _fields_ = [("geo_lat", C.c_void_p), ("geo_lon", C.c_void_p), ("merchant_lat", C.c_void_p),
                ("merchant_lon", C.c_void_p), ("payment_method", C.c_void_p), ("transaction_type", C.c_void_p),
                ("card_type", C.c_void_p), ("user_agent_flag", C.c_void_p), ("fraud_score", C.c_void_p)]


class fd_users_ext(C.Structure):
    _fields_ = [("n", C.c_int64), ("key", C.c_void_p), ("risk_score", C.c_void_p), ("kyc_status", C.c_void_p),
                ("verified", C.c_void_p), ("pref_start", C.c_void_p), ("pref_end", C.c_void_p),
                ("weekend_activity", C.c_void_p), ("online_preference", C.c_void_p), ("intl_preference", C.c_void_p),
                ("txn_frequency", C.c_void_p), ("has_patterns", C.c_void_p)]


class fd_merchants_ext(C.Structure):
    _fields_ = [("n", C.c_int64), ("avg_amount", C.c_void_p), ("risk_level", C.c_void_p), ("blacklisted", C.c_void_p),
                ("category", C.c_void_p), ("high_risk_category", C.c_void_p), ("open_hour", C.c_void_p),
                ("close_hour", C.c_void_p), ("suspicious_name", C.c_void_p)]


CTX_FIELDS = ("geo_lat", "geo_lon", "merchant_lat", "merchant_lon", "payment_method", "transaction_type",
              "card_type", "user_agent_flag", "fraud_score")
USER_EXT_FIELDS = ("risk_score", "kyc_status", "verified", "pref_start", "pref_end", "weekend_activity",
                   "online_preference", "intl_preference", "txn_frequency", "has_patterns")
MERCHANT_EXT_FIELDS = ("avg_amount", "risk_level", "blacklisted", "category", "high_risk_category", "open_hour",
                       "close_hour", "suspicious_name")
FD_FEATURE_MAP_WIDTH = 64
FD_CODE_UNKNOWN = 254
RULE_DTYPE = [("tp_score", "<f8"), ("fe_score", "<f8"), ("tp_decision", "u1"), ("tp_risk", "u1"),
              ("fe_decision", "u1"), ("fe_risk", "u1"), ("pad", "u1", 4)]


class fd_lstm_params(C.Structure):
    _fields_ = [("input_size", C.c_int32), ("hidden", C.c_int32), ("n_out", C.c_int32), ("w_ih", C.c_void_p),
                ("w_hh", C.c_void_p), ("b_ih", C.c_void_p), ("b_hh", C.c_void_p), ("w_out", C.c_void_p),
                ("b_out", C.c_void_p)]


class fd_users(C.Structure):
    _fields_ = [("n", C.c_int64), ("key", C.c_void_p), ("avg_amount", C.c_void_p),
                ("account_age_days", C.c_void_p), ("device_fp", C.c_void_p)]


class fd_merchants(C.Structure):
    _fields_ = [("n", C.c_int64), ("fraud_rate", C.c_void_p), ("risk_multiplier", C.c_void_p)]


class fd_txn_batch(C.Structure):
    _fields_ = [("card_key", C.c_void_p), ("ts_ms", C.c_void_p), ("amount_cents", C.c_void_p),
                ("merchant", C.c_void_p), ("device_fp", C.c_void_p), ("ip_class", C.c_void_p),
                ("hour", C.c_void_p), ("weekend", C.c_void_p)]


FD_TIMING_ALL, FD_TIMING_XGB, FD_TIMING_IFOREST, FD_TIMING_FEATURES, FD_TIMING_BLEND = -1, 0, 1, 2, 3
FD_TIMING_ROUTE = 4
FD_TIMING_LSTM = 5
FD_TIMING_WINDOWS = 6
FD_TIMING_INGEST = 7
FD_TIMING_ENSEMBLE = 8

# JSON ingest codec (fd_ingest_out column order and dtypes)
INGEST_FIELDS = (("card_key", "<u8"), ("ts_ms", "<i8"), ("amount_cents", "<i8"), ("merchant", "<i4"),
                 ("device_fp", "<u8"), ("ip_class", "u1"), ("hour", "u1"), ("weekend", "u1"), ("geo_lat", "<f8"),
                 ("geo_lon", "<f8"), ("merchant_lat", "<f8"), ("merchant_lon", "<f8"), ("payment_method", "u1"),
                 ("transaction_type", "u1"), ("card_type", "u1"), ("user_agent_flag", "u1"),
                 ("fraud_score", "<f8"), ("is_fraud", "u1"), ("txn_hash", "<u8"), ("status", "u1"))
FD_VOCAB_OTHER = 254
FD_VOCAB_PAYMENT_METHOD, FD_VOCAB_TRANSACTION_TYPE, FD_VOCAB_CARD_TYPE = 0, 1, 2
FD_INGEST_MALFORMED, FD_INGEST_TOO_LONG, FD_INGEST_UNKNOWN_VOCAB, FD_INGEST_INEXACT, FD_INGEST_MISSING = 1, 2, 4, 8, 16
FD_INGEST_INVALID = FD_INGEST_MALFORMED | FD_INGEST_TOO_LONG | FD_INGEST_MISSING


class fd_sink_params(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("user_capacity", C.c_int64)]


FD_AGG_HOURLY, FD_AGG_DAILY, FD_AGG_MERCHANT = 1, 2, 3
AGGREGATE_DTYPE = [("total_count", "<i8"), ("fraud_count", "<i8"), ("high_risk_count", "<i8"),
                   ("unique_user_count", "<i8"), ("total_amount", "<f8"), ("fraud_rate", "<f8"),
                   ("avg_amount", "<f8"), ("found", "<i4"), ("pad", "<i4")]


class fd_ingest_out(C.Structure):
    _fields_ = [(name, C.c_void_p) for name, _ in INGEST_FIELDS]


class fd_window_params(C.Structure):
    _fields_ = [("log_capacity", C.c_int64), ("max_out_of_orderness_ms", C.c_int64)]


class fd_window_inputs(C.Structure):
    _fields_ = [("payment_method", C.c_void_p), ("is_fraud", C.c_void_p), ("fraud_score", C.c_void_p)]


# fd_user_window / fd_merchant_window as numpy record dtypes (the host result arrays)
USER_WINDOW_DTYPE = [("user_key", "<u8"), ("window_start", "<i8"), ("window_end", "<i8"), ("first_ts", "<i8"),
                     ("last_ts", "<i8"), ("count", "<i4"), ("fraud_count", "<i4"), ("high_risk_count", "<i4"),
                     ("unique_merchants", "<i4"), ("unique_payment_methods", "<i4"), ("pad", "<i4"),
                     ("total_amount", "<f8"), ("avg_amount", "<f8"), ("fraud_rate", "<f8"),
                     ("velocity_score", "<f8")]
MERCHANT_WINDOW_DTYPE = [("merchant", "<i4"), ("count", "<i4"), ("window_start", "<i8"), ("window_end", "<i8"),
                         ("first_ts", "<i8"), ("last_ts", "<i8"), ("fraud_count", "<i4"),
                         ("high_risk_count", "<i4"), ("unique_users", "<i4"), ("unique_payment_methods", "<i4"),
                         ("total_amount", "<f8"), ("fraud_amount", "<f8"), ("avg_amount", "<f8"),
                         ("fraud_rate", "<f8"), ("amount_stddev", "<f8"), ("risk_score", "<f8"),
                         ("cents", "<i8"), ("fraud_cents", "<i8"), ("sq_lo", "<u8"), ("sq_hi", "<u8"),
                         ("pm_mask", "<u8", (4,))]  # the exact moments fd_merchant_windows_merge combines
FD_MAX_SEQ_LEN = 16
FD_SLOT_LSTM = 64
FD_SEQ_INPUT = 16
FD_MAX_SHARDS = 64
FD_ROUTE_RECORD_BYTES = 48
FD_RESULT_RECORD_BYTES = 24
FD_WINDOW_REDIS_COMPAT = 0
FD_WINDOW_SLIDING = 1
FD_RAW_FEATURES = 16
FD_VECTOR_WIDTH = 64
TXN_FIELDS = ("card_key", "ts_ms", "amount_cents", "merchant", "device_fp", "ip_class", "hour", "weekend")

_vp = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_dp = C.POINTER(C.c_double)

# (name, restype, argtypes) for every function the header declares.
SIGNATURES = {
    "fd_last_error": (C.c_char_p, []),
    "fd_build_id": (C.c_char_p, []),
    "fd_abi_version": (C.c_int, []),
    "fd_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "fd_engine_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "fd_engine_destroy": (C.c_int, [_vp]),
    "fd_engine_set_stream": (C.c_int, [_vp, _vp]),
    "fd_engine_reset_stream": (C.c_int, [_vp]),
    "fd_engine_sync": (C.c_int, [_vp]),
    "fd_load_forest": (C.c_int, [_vp, C.c_int, C.POINTER(fd_forest_params), C.POINTER(fd_tree_arrays)]),
    "fd_unload_forest": (C.c_int, [_vp, C.c_int]),
    "fd_load_xgboost_json": (C.c_int, [_vp, C.c_int, C.c_char_p]),
    "fd_xgboost_json_read": (C.c_int, [C.c_char_p, C.POINTER(fd_forest_params), C.POINTER(_i32), C.POINTER(_i64),
                                       C.POINTER(fd_tree_arrays)]),
    "fd_forest_info": (C.c_int, [_vp, C.c_int, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "fd_forest_predict_device": (C.c_int, [_vp, C.c_int, _vp, _i64, _i32, _vp, _vp, _vp]),
    "fd_forest_predict_host": (C.c_int, [_vp, C.c_int, _vp, _i64, _i32, _vp, _vp, _vp]),
    "fd_blend_device": (C.c_int, [_vp, C.POINTER(fd_blend_params), _i64, C.POINTER(_vp), _vp, _vp, _vp, _vp, _vp]),
    "fd_blend_host": (C.c_int, [_vp, C.POINTER(fd_blend_params), _i64, C.POINTER(_vp), _vp, _vp, _vp, _vp, _vp]),
    "fd_score_matrix_device": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, C.POINTER(_vp), _vp, _vp, _i64, _i32,
                                         _vp, _vp, _vp, _vp, _vp]),
    "fd_score_matrix_host": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, C.POINTER(_vp), _vp, _vp, _i64, _i32,
                                       _vp, _vp, _vp, _vp, _vp]),
    "fd_state_init": (C.c_int, [_vp, C.POINTER(fd_state_params)]),
    "fd_state_clear": (C.c_int, [_vp]),
    "fd_state_info": (C.c_int, [_vp, C.POINTER(_i64), C.POINTER(_i64)]),
    "fd_state_load_users_host": (C.c_int, [_vp, C.POINTER(fd_users)]),
    "fd_load_merchants_host": (C.c_int, [_vp, C.POINTER(fd_merchants)]),
    "fd_features_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), _i64, _vp, _vp]),
    "fd_features_host": (C.c_int, [_vp, C.POINTER(fd_txn_batch), _i64, _vp, _vp]),
    "fd_score_batch_device": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, C.POINTER(_vp), _vp,
                                        C.POINTER(fd_txn_batch), _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fd_score_batch_pipelined": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, C.POINTER(_vp), _vp,
                                           C.POINTER(fd_txn_batch), _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fd_state_load_users_ext_host": (C.c_int, [_vp, C.POINTER(fd_users_ext)]),
    "fd_load_merchants_ext_host": (C.c_int, [_vp, C.POINTER(fd_merchants_ext)]),
    "fd_load_vocab_host": (C.c_int, [_vp, _vp, _vp]),
    "fd_features_full_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_txn_context), _i64, _vp, _vp,
                                          _vp, _vp]),
    "fd_load_lstm": (C.c_int, [_vp, C.POINTER(fd_lstm_params)]),
    "fd_unload_lstm": (C.c_int, [_vp]),
    "fd_lstm_predict_device": (C.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "fd_lstm_predict_host": (C.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "fd_features_seq_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), _i64, _vp, _vp, _vp]),
    "fd_shard_of_host": (C.c_int, [_vp, _i64, _i32, _vp]),
    "fd_route_partition_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), _i64, _i32, _vp, _vp]),
    "fd_route_partition_ex_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64, _i32,
                                               _vp, _vp]),
    "fd_route_unpack_device": (C.c_int, [_vp, _vp, _vp, _i64, C.POINTER(fd_txn_batch), _vp, _vp, _vp]),
    "fd_windows_observe": (C.c_int, [_vp, _i64]),
    "fd_merchant_windows_merge": (C.c_int, [_vp, _i64, _vp, C.POINTER(_i64)]),
    "fd_score_records_device": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, _vp, _vp, _i64, _vp]),
    "fd_score_records_pipelined": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, _vp, _vp, _i64, _vp, _vp]),
    "fd_comm_unique_id": (C.c_int, [C.c_char_p, _vp]),
    "fd_comm_init": (C.c_int, [_vp, C.c_char_p, _i32, _i32, _vp, _vp]),
    "fd_comm_destroy": (C.c_int, [_vp]),
    "fd_sharded_step": (C.c_int, [_vp, C.POINTER(fd_blend_params), _vp, _vp, C.POINTER(fd_txn_batch), _i64,
                                  C.c_uint64, _vp, C.POINTER(fd_txn_batch), _i64, C.c_uint64, _vp, _vp, _vp, _vp, _vp,
                                  _vp]),
    "fd_route_partition_stream": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64, _i32,
                                            _vp, _vp, _vp]),
    "fd_route_scatter_results_device": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp]),
    "fd_windows_init": (C.c_int, [_vp, C.POINTER(fd_window_params)]),
    "fd_windows_step_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64, C.c_int,
                                         _vp, _i64, C.POINTER(_i64), _vp, _i64, C.POINTER(_i64)]),
    "fd_windows_step_host": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64, C.c_int,
                                       _vp, _i64, C.POINTER(_i64), _vp, _i64, C.POINTER(_i64)]),
    "fd_windows_stats": (C.c_int, [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64)]),
    "fd_state_snapshot": (C.c_int, [_vp, C.c_char_p, _i32, _i32, C.POINTER(_i64)]),
    "fd_state_restore": (C.c_int, [_vp, C.c_char_p, _i32, _i32, _i32, C.POINTER(_i64)]),
    "fd_hash64": (C.c_int, [_vp, _i64, C.POINTER(C.c_uint64)]),
    "fd_sink_init": (C.c_int, [_vp, C.POINTER(fd_sink_params)]),
    "fd_sink_update_device": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64]),
    "fd_sink_update_host": (C.c_int, [_vp, C.POINTER(fd_txn_batch), C.POINTER(fd_window_inputs), _i64]),
    "fd_sink_query_host": (C.c_int, [_vp, _i32, _vp, _vp, _i64, _vp]),
    "fd_sink_evict_before": (C.c_int, [_vp, _i64, C.POINTER(_i64), C.POINTER(_i64)]),
    "fd_ingest_set_vocab": (C.c_int, [_vp, _i32, _vp, _vp, _i64]),
    "fd_ingest_set_merchants": (C.c_int, [_vp, _vp, _vp, _i64]),
    "fd_ingest_json_device": (C.c_int, [_vp, _vp, _vp, _i64, C.POINTER(fd_ingest_out)]),
    "fd_ingest_json_host": (C.c_int, [_vp, _vp, _vp, _i64, C.POINTER(fd_ingest_out)]),
    "fd_ingest_scalar_host": (C.c_int, [_i32, _vp, _i32, _dp, C.POINTER(_i64), C.POINTER(_i32)]),
    "fd_engine_set_timing": (C.c_int, [_vp, C.c_int]),
    "fd_engine_set_option": (C.c_int, [_vp, C.c_char_p, _i64]),
    "fd_engine_get_counter": (C.c_int, [_vp, C.c_char_p, C.POINTER(_i64)]),
    "fd_timing_read": (C.c_int, [_vp, C.c_int, _dp, C.POINTER(_i64)]),
    "fd_timing_reset": (C.c_int, [_vp]),
    "fd_pack_forest_host": (C.c_int, [C.POINTER(fd_forest_params), C.POINTER(fd_tree_arrays), _vp, _i64, _vp, _i64,
                                      C.POINTER(fd_pack_info)]),
    "fd_pack_forest_binned_host": (C.c_int, [C.POINTER(fd_forest_params), C.POINTER(fd_tree_arrays), _vp, _i64,
                                             _vp, _i64, _vp, C.POINTER(fd_pack_info)]),
}


class NativeError(RuntimeError):
    def __init__(self, code: int, fn: str, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


def _preload_hip_runtime() -> None:
    """One process, one HIP runtime. PyTorch-ROCm wheels bundle their own libamdhip64.so and NEED it
    by the unversioned name, so if libfdengine.so (NEEDED libamdhip64.so.7) pulled /opt/rocm's copy in
    first, a later `import torch` would map a SECOND runtime that finds no GPU. Load the copy torch
    will use first (by path, so the loader identifies it as the same file when torch asks for it)."""
    if os.environ.get("FDENGINE_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    cand = Path(spec.origin).parent / "lib" / "libamdhip64.so"
    if cand.exists():
        C.CDLL(str(cand), mode=C.RTLD_GLOBAL)


def _load() -> C.CDLL:
    _preload_hip_runtime()
    if not LIB_PATH.exists():
        raise ImportError(
            f"libfdengine.so not found at {LIB_PATH}. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback for the scoring path.")
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # refuse a library built from other sources than the tree it runs beside (FDENGINE_SRC_ROOT: check against
    # another copy of the package sources, used by tests)
    from . import _buildid
    src_pkg = Path(os.environ.get("FDENGINE_SRC_ROOT", PKG_ROOT))
    src_repo = Path(os.environ.get("FDENGINE_SRC_REPO", src_pkg.parent))
    if (src_pkg / "csrc").is_dir():
        _buildid.check(lib.fd_build_id().decode(), src_pkg, src_repo)
    return lib


lib = _load()


def check(code: int, fn: str) -> None:
    if code != FD_OK:
        msg = lib.fd_last_error().decode("utf-8", "replace")
        if code == FD_ERR_NOT_LOADED:
            raise ValueError(msg)
        raise NativeError(code, fn, msg)


def call(fn: str, *args) -> None:
    check(getattr(lib, fn)(*args), fn)
