"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's cpu_baseline may import it; the product
never does). NumPy restatement of the card-hash routing of realtime-fraud-detection_amd/csrc/route.hip.

Reference behaviour it stands for: the reference keys every per-card computation by user id (Flink
keyBy / Kafka partition key, services/flink-jobs/.../FraudDetectionJob.java, WindowProcessor.java:45-64)
so each card's transactions are processed in arrival order by one owner. Restated here:
  shard_of(key, G)  = ((fmix64(key or 1) >> 32) * G) >> 32
  partition         = stable grouping of a micro-batch by owner (arrival order kept inside a group)
  record layout     = 48 B {u64 key, i64 ts, i64 cents, u64 dfp, i32 merchant, u32 seq, u8 ipc, hour, wk, pad}
  result layout     = 24 B {f64 fraud_prob, f64 confidence, u32 seq, u8 decision, u8 risk, u16 pad}
"""
from __future__ import annotations

import numpy as np

RECORD = np.dtype([("key", "<u8"), ("ts", "<i8"), ("cents", "<i8"), ("dfp", "<u8"), ("merchant", "<i4"),
                   ("seq", "<u4"), ("ipc", "u1"), ("hour", "u1"), ("wk", "u1"), ("pm", "u1"), ("flags", "<u4")])
RESULT = np.dtype([("fraud_prob", "<f8"), ("confidence", "<f8"), ("seq", "<u4"), ("decision", "u1"),
                   ("risk", "u1"), ("pad", "<u2")])
assert RECORD.itemsize == 48 and RESULT.itemsize == 24

_M1 = np.uint64(0xff51afd7ed558ccd)
_M2 = np.uint64(0xc4ceb9fe1a85ec53)


def fmix64(k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, np.uint64).copy()
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33)
        k *= _M1
        k ^= k >> np.uint64(33)
        k *= _M2
        k ^= k >> np.uint64(33)
    return k


def shard_of(keys, G: int) -> np.ndarray:
    k = np.asarray(keys, np.uint64)
    k = np.where(k == 0, np.uint64(1), k)
    hi = fmix64(k) >> np.uint64(32)
    with np.errstate(over="ignore"):
        return ((hi * np.uint64(G)) >> np.uint64(32)).astype(np.int32)


def partition(txns: dict, G: int, payment_method=None, is_fraud=None):
    """-> (records [n] RECORD, owner-major and stable; counts [G] int64). payment_method / is_fraud (optional)
    ride in the records for the owner's windows and sink (fd_route_partition_ex_device)."""
    owner = shard_of(txns["card_key"], G)
    order = np.argsort(owner, kind="stable")
    n = len(owner)
    rec = np.zeros(n, RECORD)
    rec["key"] = np.asarray(txns["card_key"], np.uint64)[order]
    rec["ts"] = np.asarray(txns["ts_ms"], np.int64)[order]
    rec["cents"] = np.asarray(txns["amount_cents"], np.int64)[order]
    rec["dfp"] = np.asarray(txns["device_fp"], np.uint64)[order]
    rec["merchant"] = np.asarray(txns["merchant"], np.int32)[order]
    rec["seq"] = order.astype(np.uint32)
    rec["ipc"] = np.asarray(txns["ip_class"], np.uint8)[order]
    rec["hour"] = np.asarray(txns["hour"], np.uint8)[order]
    rec["wk"] = np.asarray(txns["weekend"], np.uint8)[order]
    rec["pm"] = 255 if payment_method is None else np.asarray(payment_method, np.uint8)[order]
    rec["flags"] = 0 if is_fraud is None else (np.asarray(is_fraud) != 0).astype(np.uint32)[order]
    return rec, np.bincount(owner, minlength=G).astype(np.int64)


def records_to_txns(rec: np.ndarray) -> dict:
    return {"card_key": rec["key"].copy(), "ts_ms": rec["ts"].copy(), "amount_cents": rec["cents"].copy(),
            "merchant": rec["merchant"].copy(), "device_fp": rec["dfp"].copy(), "ip_class": rec["ipc"].copy(),
            "hour": rec["hour"].copy(), "weekend": rec["wk"].copy()}


def scatter_results(res: np.ndarray):
    n = len(res)
    fp, conf = np.empty(n, np.float64), np.empty(n, np.float64)
    dec, risk = np.empty(n, np.uint8), np.empty(n, np.uint8)
    s = res["seq"].astype(np.int64)
    fp[s], conf[s], dec[s], risk[s] = res["fraud_prob"], res["confidence"], res["decision"], res["risk"]
    return fp, conf, dec, risk
