"""ORACLE — TEST INFRASTRUCTURE ONLY. Pure-Python tree walkers for small cases.

An independent second restatement of oracle_forest.c (which it cross-checks), plus a walker of the
ENGINE's repacked layout (fd_pack_forest_host output) so the CPU test suite can prove the repack is
equivalent to the original trees without a GPU.

XGBoost: xgboost 2.0.3 RegTree::GetNext (`fvalue < split_cond`, missing -> default child),
predictor sums f32 leaf weights in tree order from the f32 base margin
(reference call site ml/models/model_manager.py:309-311).
sklearn: tree.apply `(double)x <= threshold` (sklearn/tree/_tree.pyx), IsolationForest depth sum in
estimator order (sklearn/ensemble/_iforest.py _compute_score_samples; reference :338-346).
"""
from __future__ import annotations

import math
import struct

import numpy as np

TILE = 256


def _f32(v) -> float:
    return float(np.float32(v))


def xgb_walk(fa, x_row):
    """-> (margin f32 as float, [leaf ids])"""
    # ProbToMargin in f32 with the C library's logf (numpy's float32 log may differ by an ulp)
    from . import lib
    m = np.float32(lib().orc_xgb_base_margin(float(fa.base_score)))
    leaves = []
    for t in range(fa.n_trees):
        o = int(fa.offsets[t])
        nid = 0
        while fa.left[o + nid] != -1:
            f = int(fa.feature[o + nid])
            fv = np.float32(x_row[f]) if f < len(x_row) else np.float32("nan")
            if np.isnan(fv):
                nid = int(fa.left[o + nid] if fa.default_left[o + nid] else fa.right[o + nid])
            elif fv < np.float32(fa.threshold[o + nid]):
                nid = int(fa.left[o + nid])
            else:
                nid = int(fa.right[o + nid])
        m = np.float32(m + np.float32(fa.leaf_value[o + nid]))
        leaves.append(nid)
    return float(m), leaves


def iforest_walk(fa, x_row):
    d = 0.0
    leaves = []
    for t in range(fa.n_trees):
        o = int(fa.offsets[t])
        nid = 0
        while fa.left[o + nid] != -1:
            f = int(fa.feature[o + nid])
            fv = float(np.float32(x_row[f])) if f < len(x_row) else float("nan")
            if math.isnan(fv):
                nid = int(fa.left[o + nid] if fa.default_left[o + nid] else fa.right[o + nid])
            elif fv <= float(fa.threshold[o + nid]):
                nid = int(fa.left[o + nid])
            else:
                nid = int(fa.right[o + nid])
        d = d + float(fa.leaf_value[o + nid])
        leaves.append(nid)
    return d, leaves


def packed_walk(blob: bytes, leaf_ids: np.ndarray, info, kind_xgb: bool, x_row):
    """Walk the engine's packed layout exactly as forest_kernel does (x < thr, meta = f*TILE*4|dl<<31).
    -> (sum of leaf values in tree order (f32 for XGB / f64 for IF) from 0 or base margin, [leaf ids])"""
    D = info.depth
    NL = 1 << D  # 1-based heap: node records at slots 1..NL-1, children 2i / 2i+1, leaves after NL records
    acc = np.float32(info.base_margin) if kind_xgb else 0.0
    leaves = []
    for t in range(info.n_trees):
        base = (t // info.chunk) * info.chunk_stride + (t % info.chunk) * info.tree_bytes
        idx = 1
        for _ in range(D):
            thr_bits, meta = struct.unpack_from("<II", blob, base + idx * 8)
            thr = np.frombuffer(struct.pack("<I", thr_bits), np.float32)[0]
            f = (meta & 0x7FFFFFFF) // (TILE * 4)
            x = np.float32(x_row[f]) if f < len(x_row) else np.float32("nan")
            if np.isnan(x):
                right = 1 - (meta >> 31)
            else:
                right = 0 if x < thr else 1
            idx = 2 * idx + right
        s = idx - NL
        if kind_xgb:
            v = struct.unpack_from("<f", blob, base + NL * 8 + s * 4)[0]
            acc = np.float32(acc + np.float32(v))
        else:
            v = struct.unpack_from("<d", blob, base + NL * 8 + s * 8)[0]
            acc = acc + v
        leaves.append(int(leaf_ids[t * NL + s]))
    return float(acc), leaves


def bin_of(thr_f32: np.ndarray, v) -> int:
    """Binned layout: bin(x) = #{t in the feature's sorted distinct thresholds : t <= x}."""
    return int(np.searchsorted(thr_f32, np.float32(v), side="right"))


def packed_walk_binned(blob: bytes, leaf_ids: np.ndarray, thr: np.ndarray, off: np.ndarray, info, kind_xgb: bool,
                       x_row):
    """Walk the engine's BINNED layout as forest_kernel4 does: node word = j << 16 | f * 1024 | dl,
    go right iff bin(x_f) << 16 > node (i.e. bin > j); missing -> default direction."""
    D = info.depth
    NL = 1 << D  # 1-based heap: node words at slots 1..NL-1 (4 B), children 2i / 2i+1, then NL leaves
    acc = np.float32(info.base_margin) if kind_xgb else 0.0
    leaves = []
    for t in range(info.n_trees):
        base = (t // info.chunk) * info.chunk_stride + (t % info.chunk) * info.tree_bytes
        idx = 1
        for _ in range(D):
            (node,) = struct.unpack_from("<I", blob, base + idx * 4)
            f = (node & 0xFC00) // (TILE * 4)
            x = np.float32(x_row[f]) if f < len(x_row) else np.float32("nan")
            if np.isnan(x):
                right = 1 - (node & 1)
            else:
                b = bin_of(thr[off[f]:off[f + 1]], x)
                right = 1 if (b << 16) > node else 0
            idx = 2 * idx + right
        s = idx - NL
        if kind_xgb:
            v = struct.unpack_from("<f", blob, base + NL * 4 + s * 4)[0]
            acc = np.float32(acc + np.float32(v))
        else:
            v = struct.unpack_from("<d", blob, base + NL * 4 + s * 8)[0]
            acc = acc + v
        leaves.append(int(leaf_ids[t * NL + s]))
    return float(acc), leaves
