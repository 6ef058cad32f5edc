#!/usr/bin/env python3
"""bench.py — scored transactions/sec on the hot path (BASELINE.json metric: "scored transactions/sec
(whole node) at 1/2/4/8 GPUs; p99 micro-batch latency").

Default workload (BASELINE.json configs[3], "config 4" — the configuration the metric is quoted on):
card-hash-sharded keyed state + scoring. Each rank (one process per GPU) ingests its own 64k-transaction
micro-batch per step, drawn over ALL 100M cards of the node, and runs fdengine.sharding.ShardedScorer:
route partition -> RCCL all-to-all of 48-B records to the owner GPUs -> owner features (HBM card state,
sliding windows) + XGBoost 500x8 + IsolationForest 100 + blend -> all-to-all of results back -> arrival
order. At N=1 the same kernels run with no collective (all 100M cards resident on the one GPU).

`python bench.py --gpus N` (no torchrun env) starts N ranks itself (torch.distributed.run, spawned before
anything touches the GPU); under `torch.distributed.run --nproc-per-node N` it joins the given ranks.

Other workloads (`--workload`): config2 (XGBoost only on HBM-resident vectors), config3 (10M cards, one
GPU, no routing), config5 (+ LSTM head, 1k latency batches), ingest (JSON codec), config3j (config3 from
raw JSON).

Reported beside the throughput: p50/p99 micro-batch latency (host submit -> scores in host memory), the
dominant kernel's roofline against ITS bound (the forest walk: LDS issue, node-steps/s against the
LDS-array ceiling), the fused pipeline's algorithmic HBM bytes (SURVEY §8(d), 238 B/txn), per-kernel
times, and the CPU baseline: the oracle C restatement of the whole chain on a config-1-shaped stream
(100k simulator transactions), at 1 core and at the host threads available (rank 0, N=1 only).
"""
import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

# One hardware queue per stream: the sharded step keeps the engine stream, two pipeline streams, its forward stream
# and RCCL's streams busy at once; with HIP's default of 4 queues per process some would share a queue and a
# blocked RCCL kernel would stall a pipeline stream behind it (set before anything initialises HIP; <= 32).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "realtime-fraud-detection_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFLOPS = 157.3  # dense f32-input MFMA peak (MI355X_MICROARCH.md "Peak FP32 (matrix)")
# Forest walk: per node-step one ds_read_b32 (feature bin) + one ds_read_b64 (children pair) per lane; per
# 64-lane wave-instruction 2 + 2 LDS-array cycles (MI355X_MICROARCH.md §LDS) = 16 node-steps/clk/CU.
LDS_NODE_STEPS_PEAK = 256 * 2.4e9 * 16  # 9.83e12 node-steps/s
# The same read pair chased the way the walk chases it (each step's addresses from the previous step's data, random
# 1 KiB rows, conflict-free columns, 16 waves x 8 chains per CU): measured 4.19e9 node-steps in 0.867 ms on every CU
# (tools/micro/lds_width.hip, profiles/r05/lds_width/) — ~4 LDS cycles per wave-read, not the table's 2
LDS_NODE_STEPS_ATTAINABLE = 4.19e9 / 0.867e-3  # 4.83e12 node-steps/s
FUSED_BYTES_PER_TXN = 238  # txn 36 + card header R/W 96 + profiles 64 + outputs 10 + ring append 32
TIMING_EVERY = 8  # kernel-timing sample period (engine option "timing_every")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_threads():
    t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    return max(1, min(t, os.cpu_count() or 1, len(os.sched_getaffinity(0))))


def cpu_limits() -> dict:
    """The host cores this process may actually use: the scheduler affinity mask and the cgroup CPU quota (the
    GPU box shows the whole machine in os.cpu_count())."""
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def forest_blob_bytes(forest) -> int:
    """Model bytes one launch reads: the binned layout's 4-byte node words and leaf values of every
    tree padded to a perfect depth-D heap (2^D node slots + 2^D leaves per tree)."""
    from fdengine import pack_forest_host
    _, _, info = pack_forest_host(forest)
    leaf = 4 if forest.kind == 1 else 8
    return int(forest.n_trees * (1 << int(info.depth)) * (4 + leaf))


FOREST_KERNEL = "forest_kernel6<D={d},{t},{k}> (binned node-only chunks)"


def pmc_traffic(workload, B, kernel_symbol, root=None):
    """HBM bytes per launch of `kernel_symbol` (its demangled name as rocprofv3 reports it) from the committed
    rocprofv3 PMC summary profiles/pmc_<workload>.json; None unless that file measured this kernel at this batch
    size (a summary of another kernel, e.g. an older build's, is never reported as this one's traffic)."""
    p = Path(root or REPO / "profiles") / f"pmc_{workload}.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        if int(d.get("batch", -1)) != B:
            return None
        k = d.get("kernels", {}).get(kernel_symbol)
        return int(k["hbm_bytes_per_launch"]) if k else None
    except Exception:
        return None


def pmc_counters(workload, B, groups, live_us, root=None):
    """north_star's counter figures for this workload's hot kernels: from the committed rocprofv3 PMC summary
    profiles/pmc_<workload>.json (tools/gpu/pmc_r03.sh + tools/pmc_kernels.py, same batch size only), HBM bytes per
    launch (2*FETCH_SIZE + WRITE_SIZE), L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS)) and MFMA busy, joined with
    THIS run's event-timed average duration of the same launches: achieved HBM GB/s = bytes / duration.
    groups: {label: ([kernel names in the PMC file], key of live_us)}; a kernel reported per grid size in the file
    is taken at this batch's grid only — a group whose kernels were not measured at this grid is omitted (another
    launch's counters are never reported as this one's)."""
    p = Path(root or REPO / "profiles") / f"pmc_{workload}.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
    except Exception:
        return None
    if int(d.get("batch", -1)) != B:
        return None
    ks = d.get("kernels", {})
    grid = (B + 255) // 256 * 256
    out = {}
    for label, (names, key) in groups.items():
        found, used = [], []
        for nm in names:
            kn = nm if nm in ks else f"{nm} [grid {grid}]"
            k = ks.get(kn)
            if k is None or "hbm_bytes_per_launch" not in k:
                break
            found.append((nm, k))
            used.append(kn)
        else:
            by = sum(k["hbm_bytes_per_launch"] for _, k in found)
            us = (live_us or {}).get(key)
            e = {"kernels": names, "pmc_entries": used, "hbm_bytes_per_launch": by,
                 "achieved_GBs": round(by / (us * 1e-6) / 1e9, 2) if us else None, "live_avg_us": us,
                 "peak_GBs": HBM_PEAK_GBS, "l2_hit_rate": {nm: k.get("l2_hit_rate") for nm, k in found}}
            mf = {nm: k["mfma_busy"] for nm, k in found if k.get("mfma_busy")}
            if mf:
                e["mfma_busy"] = mf
            out[label] = e
    if not out:
        return None
    out["basis"] = (f"profiles/pmc_{workload}.json (rocprofv3 --pmc, one pass per counter group, kernels serialised "
                    "by the collection) x this run's HIP-event durations")
    return out


def ensemble_symbol(out, wide):
    return f"fd::anon::ensemble_kernel<8, {out}, {'true' if wide else 'false'}, true>"
FOREST6_SYMBOL = "fd::anon::forest_kernel6<8, 24, float, 1, 0>"
LSTM4_SYMBOL = "fd::anon::lstm_kernel4"
INGEST_SYMBOL = "fd::anon::ingest_json_kernel"


def forest_roofline(timing, kind, forest, depth, B, workload, label, forests=None, out=0, wide=True, vec_bytes=256,
                    fused_single=False):
    """Roofline of a forest launch against its real bound: LDS issue of the dependent walk. With the fused
    ensemble kernel (FD_TIMING_ENSEMBLE) timed, that launch is the one reported (both forests' node steps)."""
    from fdengine import _native as N
    ms, launches = timing.get(kind, (0.0, 0))
    symbol = FOREST6_SYMBOL
    if forests and timing.get(N.FD_TIMING_ENSEMBLE, (0.0, 0))[1]:
        ms, launches = timing[N.FD_TIMING_ENSEMBLE]
        steps = B * sum(f.n_trees for f in forests) * depth
        label = "ensemble_kernel<D=8> (XGBoost 500 + IsolationForest 100 over one merged-bin tile + blend)"
        forest_bytes = sum(forest_blob_bytes(f) for f in forests)
        # the instantiation that ran: output form (0 columns, 1 route result records) and chunk layout (wide
        # unless the engine has RCCL communicators: engine option ensemble_chunks)
        symbol = ensemble_symbol(out, wide)
    elif fused_single or timing.get(N.FD_TIMING_ENSEMBLE, (0.0, 0))[1]:  # one forest through the fused kernel
        # (config 2: fd_forest_predict on >= 128 tiles without raw / leaf outputs runs ensemble_kernel<D, 2>, timed
        # under the forest's own kind)
        if not fused_single:
            ms, launches = timing[N.FD_TIMING_ENSEMBLE]
        steps = B * forest.n_trees * depth
        forest_bytes = forest_blob_bytes(forest)
        label = "ensemble_kernel<D=8> over one forest (probabilities only)"
        symbol = ensemble_symbol(2, True)
    else:
        steps = B * forest.n_trees * depth
        forest_bytes = forest_blob_bytes(forest)
    avg = (ms / 1e3) / max(1, launches)
    achieved = steps / avg
    model_bytes = forest_bytes
    return {"bound": "lds", "achieved": round(achieved, 1), "peak": LDS_NODE_STEPS_PEAK, "unit": "node-steps/s",
            "frac": round(achieved / LDS_NODE_STEPS_PEAK, 6), "traffic": pmc_traffic(workload, B, symbol),
            "traffic_basis": f"profiles/pmc_{workload}.json, kernel {symbol}: 2*FETCH_SIZE + WRITE_SIZE per launch",
            "kernel": label, "kernel_symbol": symbol, "kernel_avg_us": round(avg * 1e6, 3),
            "kernel_samples": launches, "node_steps_per_launch": steps,
            "peak_basis": "per node-step 1 ds_read_b32 + 1 ds_read_b64 per lane = 4 LDS-array cycles per 64 "
                          "node-steps: 16/clk/CU x 256 CUs x 2.4 GHz",
            "attainable": {"peak": round(LDS_NODE_STEPS_ATTAINABLE, 1),
                           "frac": round(achieved / LDS_NODE_STEPS_ATTAINABLE, 6),
                           "basis": "the walk's dependent ds_read_u16 + ds_read_b64 pair chased on every CU (16 waves "
                                    "x 8 chains, random rows, conflict-free banks; tools/micro/lds_width.hip, "
                                    "profiles/r05/lds_width): 4.19e9 node-steps in 0.867 ms"},
            "hbm_view": {"algorithmic_bytes_per_launch": B * (vec_bytes + 8) + model_bytes,
                         "vector_bytes_per_txn": vec_bytes,
                         "achieved_GBs": round((B * (vec_bytes + 8) + model_bytes) / avg / 1e9, 3),
                         "peak_GBs": HBM_PEAK_GBS}}


def product_blend(names):
    """Blend constants the way the product computes them: EnsemblePredictor._get_model_weights over the
    enabled models of the registry (fdengine/ensemble.py, ensemble_predictor.py:62-73)."""
    from fdengine import ensemble as E
    from fdengine.registry import ScoringConfig
    cfg = ScoringConfig("/nonexistent-models")
    for n in list(cfg.models):
        if n not in names:
            cfg.disable_model(n)
    ep = E.EnsemblePredictor(None, cfg)
    return ep.blend_params(names), [ep.model_weights[n] for n in names], [E._CONF_MULT[n] for n in names]


_HIP = None


def _diag_blocks() -> int:
    return int(os.environ.get("FD_BENCH_BLOCKS", "0") or 0)


def _dump_fprof(tag) -> None:
    """FD_BENCH_DUMP_FPROF=prefix with the profiling library (FDENGINE_LIB=.../libfdengine_prof.so): the feature
    kernels' per-workgroup phase stamps of the last launch, saved as prefix.<tag>.npy (tools/lean_phases.py)"""
    pre = os.environ.get("FD_BENCH_DUMP_FPROF")
    if not pre:
        return
    import ctypes
    import numpy as np
    from fdengine import _native
    buf = np.zeros(4096 * 8, np.uint64)
    _native.lib.fd_debug_feat_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if _native.lib.fd_debug_feat_profile(buf.ctypes.data, buf.size) == 0:
        np.save(f"{pre}.{tag}.npy", buf)
    buf2 = np.zeros(4096 * 4, np.uint64)
    _native.lib.fd_debug_feat_profile2.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if _native.lib.fd_debug_feat_profile2(buf2.ctypes.data, buf2.size) == 0:
        np.save(f"{pre}.{tag}.c.npy", buf2)


def _diag_offset() -> int:
    """FD_BENCH_BATCH_OFFSET=N (diagnostics): skip N resident micro-batches after the parity check"""
    return int(os.environ.get("FD_BENCH_BATCH_OFFSET", "0") or 0)


def _parity_record(batches, path, rows_per_batch):
    """the parity_vs_oracle record: the timed path's batches (no vectors requested) and the vectors-requested twin"""
    def leg():
        return {"rows": 0, "max_abs_prob_diff": 0.0, "max_abs_conf_diff": 0.0, "prob_exact_rows": 0,
                "decision_mismatches": 0, "risk_mismatches": 0, "decision_mismatches_off_threshold": 0}
    twin = dict(leg(), vector_mismatched_elements=0, vector_max_ulp=0, max_abs_model_prob_diff=0.0)
    return {"batches_checked": batches, "rows_per_batch": rows_per_batch, "path": path, "timed_path": leg(),
            "twin": twin, "bar": "fraud_prob / confidence within 1e-5 (north star), decision / risk exact (off a "
                                 "decision threshold by more than 1e-6)"}


def _parity_compare(rec, got, ref):
    """fraud_prob, confidence, decision, risk of one batch against the oracle chain's"""
    import numpy as np
    gfp, gconf, gdec, grisk = got
    fp, conf, dec, risk = ref
    rec["rows"] += len(fp)
    rec["max_abs_prob_diff"] = max(rec["max_abs_prob_diff"], float(np.abs(gfp - fp).max()) if len(fp) else 0.0)
    rec["max_abs_conf_diff"] = max(rec["max_abs_conf_diff"], float(np.abs(gconf - conf).max()) if len(fp) else 0.0)
    rec["prob_exact_rows"] += int((gfp == fp).sum())
    bad = gdec != dec
    rec["decision_mismatches"] += int(bad.sum())
    rec["risk_mismatches"] += int((grisk != risk).sum())
    near = np.abs(conf - 0.7) < 1e-6  # an f32 sigmoid an ulp from the oracle's may cross a threshold
    for thr in (0.6, 0.8, 0.95):
        near |= np.abs(fp - thr) < 1e-6
    rec["decision_mismatches_off_threshold"] += int((bad & ~near).sum())


def _parity_vectors(rec, V, rvec):
    import numpy as np
    diff = V != rvec
    rec["vector_mismatched_elements"] += int(diff.sum())
    if diff.any():
        ulp = np.abs(V.view(np.int32)[diff].astype(np.int64) - rvec.view(np.int32)[diff].astype(np.int64))
        rec["vector_max_ulp"] = max(rec["vector_max_ulp"], int(ulp.max()))


def hip_memcpy_async(dst: int, src: int, nbytes: int, kind: int, stream: int) -> None:
    """hipMemcpyAsync on `stream` (the process's HIP runtime: torch's libamdhip64, loaded globally by fdengine);
    kind 1 host -> device, 2 device -> host. Straight to the runtime: torch's copy_ between pinned and device memory
    also does the caching host allocator's per-copy event bookkeeping, measured to stall the host ~6 ms about once
    per 100-200 copies at this rate"""
    global _HIP
    import ctypes
    if _HIP is None:
        _HIP = ctypes.CDLL(None).hipMemcpyAsync
        _HIP.restype = ctypes.c_int
        _HIP.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    rc = _HIP(dst, src, nbytes, kind, stream)
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed ({rc})")


def hip_d2h(dst: int, src: int, nbytes: int, stream: int) -> None:
    hip_memcpy_async(dst, src, nbytes, 2, stream)


class PackedColumns:
    """A micro-batch's input columns packed into one buffer (256-B aligned column offsets), so a host batch
    crosses PCIe in ONE hipMemcpyAsync: `host` pinned blocks (one per batch) and two device staging blocks with
    per-field views."""

    def __init__(self, like: dict, n_host: int, device):
        import torch
        from fdengine import _native as N
        self.layout, off = [], 0
        for f in N.TXN_FIELDS:
            t = like[f]
            nb = t.numel() * t.element_size()
            self.layout.append((f, off, t.dtype, t.numel()))
            off += (nb + 255) // 256 * 256
        self.nbytes = off
        self.host = []
        for _ in range(n_host):
            self.host.append(torch.empty(self.nbytes, dtype=torch.uint8).pin_memory())
        self.dev = [torch.empty(self.nbytes, dtype=torch.uint8, device=device) for _ in range(2)]
        self.dev_views = [self.views(d) for d in self.dev]

    def views(self, buf) -> dict:
        return {f: buf[off:off + n * _itemsize(dt)].view(dt) for f, off, dt, n in self.layout}

    def fill(self, q: int, cols: dict) -> None:
        """host block q <- the columns (host tensors)"""
        v = self.views(self.host[q])
        for f, _, _, _ in self.layout:
            v[f].copy_(cols[f])


def _itemsize(dt) -> int:
    import torch
    return torch.empty(0, dtype=dt).element_size()


class HostOutRing:
    """k sets of a micro-batch's outputs (fraud_prob f64, confidence f64, decision u8, risk u8) in host-mapped
    pinned memory (hipHostMalloc mapped): the engine's output kernel writes them over PCIe, so the results reach
    host memory with the step itself — no hipMemcpyAsync per step (measured: the runtime's D2H call stalls the
    host ~6 ms about once per 100-200 calls at this rate, FD_STALL_TRACE)"""

    def __init__(self, B: int, k: int):
        import ctypes
        import numpy as np
        self.hip = ctypes.CDLL(None)
        self.hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        self.hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
        self.hip.hipHostFree.argtypes = [ctypes.c_void_p]
        self.B, self.sets, self.host = B, [], []
        nbytes = 18 * B + 64
        for _ in range(k):
            h, d = ctypes.c_void_p(), ctypes.c_void_p()
            if self.hip.hipHostMalloc(ctypes.byref(h), nbytes, 2) != 0:  # hipHostMallocMapped
                raise RuntimeError("hipHostMalloc failed")
            if self.hip.hipHostGetDevicePointer(ctypes.byref(d), h, 0) != 0:
                raise RuntimeError("hipHostGetDevicePointer failed")
            self.host.append(h.value)
            base = d.value
            self.sets.append((base, base + 8 * B, base + 16 * B, base + 17 * B))
        self.np = np

    def fraud_prob(self, q: int):
        import ctypes
        return self.np.ctypeslib.as_array((ctypes.c_double * self.B).from_address(self.host[q]))

    def close(self):
        for h in self.host:
            self.hip.hipHostFree(h)
        self.host, self.sets = [], []


def fit_models(dev_index, T, D, mode, K):
    """Models in the reference's file formats on realistic scoring vectors: a 20k-card population's stream
    through the ENGINE's own feature kernel (a scratch engine with a small table), then a random XGBoost
    500 x depth 8 with hist-style cuts of those vectors and an IsolationForest trained with the reference
    trainer's recipe (synth.isolation_forest)."""
    import numpy as np
    import fdengine
    from fdengine import synth
    spop = synth.population(20000, 500, seed=11)
    stx = synth.txn_stream(spop, 40000, seed=12, rate_per_s=20.0)
    scratch = fdengine.FraudEngine(dev_index)
    try:
        scratch.state_init(1 << 16, mode, K)
        U, M = spop["users"], spop["merchants"]
        scratch.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        scratch.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        X = scratch.features(stx)
    finally:
        scratch.close()
    xgb = fdengine.xgboost_from_json_doc(synth.xgboost_doc(T, D, 64, X[-8192:], seed=13))
    ifm = fdengine.iforest_from_sklearn(synth.isolation_forest(X[-8192:].astype(np.float64)))
    return xgb, ifm


def cpu_chain_baseline(xgb, ifm, weights, mults, mode, K, lstm=None, seq_len=10, n=100_000):
    """BASELINE config 1 shape: 100k simulator transactions (10k users, 5k merchants: simulator.py:481-482)
    through the oracle chain — features (C, sequential by definition) -> XGBoost -> IsolationForest
    (-> LSTM) -> blend (OpenMP) — at 1 thread and at every host thread available. kind "port": the
    reference's own Python never reaches the GPU box (≈2.8k txn/s/core in the build container)."""
    import numpy as np
    import oracle
    from fdengine import synth
    from oracle.features_c import OracleFeatureState
    pop = synth.population(10000, 5000, seed=1)
    tx = synth.txn_stream(pop, n, seed=2)
    U, M = pop["users"], pop["merchants"]

    def run(th):
        import torch
        torch.set_num_threads(th)
        o = OracleFeatureState(1 << 15, mode, K)
        o.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        o.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        a = time.perf_counter()
        raw, V = o.run(tx, want_raw=lstm is not None)
        cols = [oracle.xgb_predict(xgb, V, nthreads=th)[0].astype(np.float64),
                oracle.iforest_predict(ifm, V, nthreads=th)[0]]
        if lstm is not None:
            from oracle import lstm_ref
            cols.append(lstm_ref.lstm_forward(lstm, lstm_ref.SequenceState(seq_len).run(tx["card_key"], raw)))
        oracle.blend_weighted(np.stack(cols), weights, mults, nthreads=th)
        return n / (time.perf_counter() - a)

    th = cpu_threads()
    one = run(1)
    many = run(th) if th > 1 else one
    chain = "features C 1 thread -> XGBoost 500x8 -> IsolationForest 100" + (" -> LSTM(128) torch fp32" if lstm else "") \
        + " -> blend"
    return {"value": round(many, 1), "unit": "txn/s", "cores": th, "kind": "port",
            "sample": f"config-1 shape: {n} simulator transactions (10k users, 5k merchants) through the oracle chain "
                      f"({chain}; forests/blend OpenMP), whole stream, {th} threads; CPU: {cpu_model()}",
            "host_cpus": cpu_limits(),
            "single_core": {"value": round(one, 1), "cores": 1}}


# --------------------------------------------------------------------------------------- config 2
class Config2:
    name = "config2"
    dtype = "f32"

    def __init__(self, args, rank, dev, eng):
        import numpy as np
        import torch
        import fdengine
        from fdengine import synth
        self.np, self.torch = np, torch
        self.args = args
        self.B, self.F, self.T, self.D = args.batch, args.features, args.trees, args.depth
        X_ref = synth.feature_matrix(2048, self.F, seed=7)
        doc = synth.xgboost_doc(self.T, self.D, self.F, X_ref, seed=8)
        with tempfile.TemporaryDirectory() as td:  # exercise the unchanged-file load path
            path = os.path.join(td, "fraud_classifier.json")
            synth.write_xgboost_json(path, doc)
            self.forest = fdengine.load_xgboost_json(path)
        self.eng = eng
        eng.load_forest(0, self.forest)
        self.info = eng.forest_info(0)
        self.pool = max(1, args.pool)
        self.Xpool = synth.feature_matrix(self.pool * self.B, self.F, seed=1000 + rank)
        self.X_dev = torch.from_numpy(self.Xpool).to(dev)
        self.prob = torch.empty(self.pool * self.B, dtype=torch.float64, device=dev)
        self.host_out = torch.empty(self.B, dtype=torch.float64, pin_memory=True)

    def step(self, i):
        s = i % self.pool
        self.eng.predict_device(0, self.X_dev.data_ptr() + s * self.B * self.F * 4, self.B, self.F,
                                self.prob.data_ptr() + s * self.B * 8)

    def fetch(self, i):
        s = i % self.pool
        src = self.prob[s * self.B:(s + 1) * self.B]
        hip_d2h(self.host_out.data_ptr(), src.data_ptr(), src.numel() * 8, self.torch.cuda.current_stream().cuda_stream)

    def parity(self):
        import oracle
        np = self.np
        worst = 0.0
        for s in range(min(self.pool, 2)):  # two whole micro-batches
            self.step(s)
            self.torch.cuda.synchronize()
            rp, _, _ = oracle.xgb_predict(self.forest, self.Xpool[s * self.B:(s + 1) * self.B], nthreads=cpu_threads())
            worst = max(worst, float(np.abs(self.prob[s * self.B:(s + 1) * self.B].cpu().numpy() - rp).max()))
        return {"batches_checked": min(self.pool, 2), "max_abs_prob_diff": worst}

    def roofline(self, timing):
        from fdengine import _native as N
        # the engine's default for a 64 k batch without raw / leaf outputs: the fused kernel over the one forest
        # (unless --engine-option ensemble=0 or forest_kernel=N forces a per-model kernel)
        forced = any(kv.replace(" ", "").startswith(("ensemble=0", "forest_kernel=")) and not
                     kv.replace(" ", "").endswith("forest_kernel=0") for kv in self.args.engine_option)
        fused = not forced and (self.B + 255) // 256 >= 128 and self.info["depth"] <= 8
        return forest_roofline(timing, N.FD_TIMING_XGB, self.forest, self.info["depth"], self.B, self.name,
                               FOREST_KERNEL.format(d=self.info['depth'], t="f32", k="XGB"), fused_single=fused)

    def kernels(self, timing):
        from fdengine import _native as N
        ms, c = timing.get(N.FD_TIMING_XGB, (0.0, 0))
        return {"xgboost_forest": round(ms / c * 1e3, 3)} if c else {}

    def config(self, world):
        return {"workload": "config2: XGBoost binary:logistic 500 trees depth 8, 50 features, "
                            "64k-txn micro-batches, features resident in HBM",
                "trees": self.T, "depth": self.D, "features": self.F, "batch": self.B,
                "parallelism": f"replicas x{world} (one process per GPU, no data-path collective)"}

    def cpu_baseline(self, seconds):
        import oracle

        def rate(th, rows):
            a = time.perf_counter()
            oracle.xgb_predict(self.forest, self.Xpool[:rows], nthreads=th)
            return rows / (time.perf_counter() - a)

        th = cpu_threads()
        one = rate(1, 16384)
        many = rate(th, min(len(self.Xpool), max(16384, int(one * th * seconds / 2))))
        return {"value": round(many, 1), "unit": "txn/s", "cores": th, "kind": "port",
                "sample": f"config-2 vectors (500 trees x depth 8, 50 features) through oracle/oracle_forest.c "
                          f"orc_xgb_predict, {th} OpenMP threads; CPU: {cpu_model()}",
                "host_cpus": cpu_limits(),
                "single_core": {"value": round(one, 1), "cores": 1}}


# --------------------------------------------------------------------------------------- config 3
class Config3:
    name = "config3"
    dtype = "f32 (features f64, forests f32/f64, blend f64)"
    with_lstm = False
    pipelined_default = True  # 64k batches: batch i+1's features overlap batch i's forests
    seq_len = 10  # lstm_sequential sequence_length (ml/utils/config.py:152)

    def __init__(self, args, rank, dev, eng):
        import numpy as np
        import torch
        from fdengine import _native as N
        from fdengine import synth
        self.np, self.torch, self.N = np, torch, N
        self.args = args
        self.B, self.T, self.D = args.batch, args.trees, args.depth
        self.cards, self.mode, self.K = args.cards, (1 if args.window == "sliding" else 0), args.ring_k
        self.eng = eng
        t = time.time()
        self.xgb, self.ifm = fit_models(dev.index, self.T, self.D, self.mode, self.K)
        eng.load_forest(0, self.xgb)
        eng.load_forest(1, self.ifm)
        self.names = ["xgboost_primary", "isolation_forest"]
        self.slots = [0, 1]
        if self.with_lstm:
            from fdengine import lstm as L
            self.lw = L.random_weights(16, 128, 1, seed=14)
            eng.load_lstm(self.lw)
            self.names.append("lstm_sequential")
            self.slots.append(N.FD_SLOT_LSTM)
        self.params, self.weights, self.mults = product_blend(self.names)
        # population: cards resident in HBM
        self.pop = synth.population(self.cards, 5000, seed=100 + rank)
        cap = 1
        while cap < int(self.cards * 1.6):
            cap *= 2
        self.cap = cap
        eng.state_init(cap, self.mode, self.K, seq_len=self.seq_len if self.with_lstm else 0)
        U, M = self.pop["users"], self.pop["merchants"]
        eng.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        eng.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        self.n_batches = args.warmup + args.steps + args.latency_iters + args.alone_iters + args.parity_batches + 1 \
            + args.loaded_iters + args.timing_steps + 1 + _diag_blocks() * args.steps + _diag_offset()
        self.tx = synth.txn_stream(self.pop, self.n_batches * self.B, seed=200 + rank)
        self.dev = {f: torch.from_numpy(np.ascontiguousarray(self.tx[f])).to(dev) for f in N.TXN_FIELDS}
        self.elem = {f: self.tx[f].dtype.itemsize for f in N.TXN_FIELDS}
        B = self.B
        self.fp = torch.empty(B, dtype=torch.float64, device=dev)
        self.conf = torch.empty(B, dtype=torch.float64, device=dev)
        self.dec = torch.empty(B, dtype=torch.uint8, device=dev)
        self.risk = torch.empty(B, dtype=torch.uint8, device=dev)
        self.mp = torch.empty((len(self.names), B), dtype=torch.float64, device=dev)
        self.vec = torch.empty((B, 64), dtype=torch.float32, device=dev)
        self.h_fp = torch.empty(B, dtype=torch.float64, pin_memory=True)
        self.h_dec = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        self.h_risk = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        # the pipelined stream (parity batches included: they run the timed path), outputs alternating two sets
        self.pipe, self.cur = (self.pipelined_default or args.pipeline) and not args.no_pipeline, 0
        self.outs = [[self.fp, self.conf, self.dec, self.risk],
                     [torch.empty_like(t) for t in (self.fp, self.conf, self.dec, self.risk)]]
        self.scorer = eng.pipelined_scorer(self.params, self.slots)
        self.serial = eng.batch_scorer(self.params, self.slots)
        self.next_batch = 0
        self.parity_batches = args.parity_batches
        log(f"[rank {rank}] {self.name} setup {time.time() - t:.1f}s: {self.cards} cards, capacity {cap}, "
            f"{self.n_batches} batches resident, window={'sliding' if self.mode else 'redis_compat'}")

    def _ptrs(self, b):
        if not hasattr(self, "_base"):
            self._base = {f: (t.data_ptr(), self.B * self.elem[f]) for f, t in self.dev.items()}
        return {f: p + b * w for f, (p, w) in self._base.items()}

    def step(self, i, vectors=False):
        """One micro-batch through the product path the timed region runs: the pipelined stream (config 3; the fused
        kernel reads the compact 64-B rows) or fd_score_batch_device per step (config 5). vectors: also ask
        for the scoring vectors and per-model probabilities (the parity twin batch; the non-compact variant)."""
        b = self.next_batch
        if b >= self.n_batches:
            raise RuntimeError("stream exhausted: raise n_batches")
        self.next_batch += 1
        vp = self.vec.data_ptr() if vectors else 0
        mp = self.mp.data_ptr() if vectors else 0
        if self.pipe:
            self.cur = b & 1
            fp, conf, dec, risk = self.outs[self.cur]
            self.scorer(self._ptrs(b), self.B, fp.data_ptr(), conf.data_ptr(), dec.data_ptr(), risk.data_ptr(),
                        vec_ptr=vp, model_probs_ptr=mp)
            return
        self.cur = 0
        self.serial(self._ptrs(b), self.B, self.fp.data_ptr(), self.conf.data_ptr(), self.dec.data_ptr(),
                    self.risk.data_ptr(), vec_ptr=vp, model_probs_ptr=mp)

    def fetch(self, i):
        fp, _, dec, risk = self.outs[self.cur]
        st = self.torch.cuda.current_stream().cuda_stream
        for h, d in ((self.h_fp, fp), (self.h_dec, dec), (self.h_risk, risk)):
            hip_d2h(h.data_ptr(), d.data_ptr(), d.numel() * d.element_size(), st)

    def parity(self):
        """The first parity_batches micro-batches (fresh state, carried across them) through the timed path — no
        vectors requested, so the pipelined stream's fused kernel reads the compact 64-B rows — against the
        oracle chain, which computes its own vectors; then one twin batch with the vectors and per-model
        probabilities requested (the non-compact variant), whose vectors are compared too."""
        return self._parity()

    def outputs(self):
        return self.outs[self.cur] if self.pipe else (self.fp, self.conf, self.dec, self.risk)

    def _parity(self):
        import oracle
        from oracle.features_c import OracleFeatureState
        np = self.np
        U, M = self.pop["users"], self.pop["merchants"]
        o = OracleFeatureState(self.cap, self.mode, self.K)
        o.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        o.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        hist = None
        if self.with_lstm:
            from oracle import lstm_ref
            hist = lstm_ref.SequenceState(self.seq_len)
        P = self.parity_batches
        c0 = self.eng.counter("pipelined_compact_batches") if self.pipe else None
        q0 = self.eng.counter("pipelined_split_batches") if self.pipe else None
        out = _parity_record(P, "pipelined stream, fused kernel from compact vectors" if self.pipe else
                             "fd_score_batch_device (latency path)", self.B)
        for b in range(P + 1):
            twin = b == P  # the vectors-requested twin batch
            part = {f: self.tx[f][b * self.B:(b + 1) * self.B] for f in self.N.TXN_FIELDS}
            self.step(b, vectors=twin)
            self.torch.cuda.synchronize()
            rraw, rvec = o.run(part, want_raw=self.with_lstm)
            cols = [oracle.xgb_predict(self.xgb, rvec, nthreads=cpu_threads())[0].astype(np.float64),
                    oracle.iforest_predict(self.ifm, rvec, nthreads=cpu_threads())[0]]
            if self.with_lstm:
                from oracle import lstm_ref
                cols.append(lstm_ref.lstm_forward(self.lw, hist.run(part["card_key"], rraw)))
            ref = oracle.blend_weighted(np.stack(cols), self.weights, self.mults)
            got = [t.cpu().numpy() for t in self.outputs()]
            _parity_compare(out["twin" if twin else "timed_path"], got, ref)
            if twin:
                V = self.vec.cpu().numpy()
                _parity_vectors(out["twin"], V, rvec)
                Mp = self.mp.cpu().numpy()
                for m, col in enumerate(cols):
                    out["twin"]["max_abs_model_prob_diff"] = max(out["twin"]["max_abs_model_prob_diff"],
                                                                 float(np.abs(Mp[m] - col).max()))
        if c0 is not None:
            out["timed_path"]["compact_batches"] = self.eng.counter("pipelined_compact_batches") - c0
            out["timed_path"]["split_row_batches"] = self.eng.counter("pipelined_split_batches") - q0
        del o
        return out

    def roofline(self, timing):
        sc = getattr(self, "scorer", None)
        native = bool(getattr(sc, "native", False))
        routed = bool(getattr(sc, "route", False))
        be = getattr(sc, "be", None)
        pipelined = bool(getattr(be, "pipelined", getattr(self, "pipe", False)))
        # the pipelined stream hands the fused kernel the compact 64-B row (14 f32 + 8 byte slots) unless vectors are requested
        return forest_roofline(timing, self.N.FD_TIMING_XGB, self.xgb, 8, self.B, self.name,
                               FOREST_KERNEL.format(d=8, t="f32", k="XGB") + " dominant", [self.xgb, self.ifm],
                               out=1 if routed else 0, wide=not native, vec_bytes=64 if pipelined else 256)

    def kernels(self, timing):
        N = self.N
        names = {N.FD_TIMING_XGB: "xgboost_forest", N.FD_TIMING_IFOREST: "iforest_forest",
                 N.FD_TIMING_FEATURES: "features", N.FD_TIMING_BLEND: "blend",
                 N.FD_TIMING_ROUTE: "route_partition (count+scan+scatter)", N.FD_TIMING_LSTM: "lstm_head",
                 N.FD_TIMING_WINDOWS: "windows", N.FD_TIMING_INGEST: "ingest_json",
                 N.FD_TIMING_ENSEMBLE: "ensemble (XGBoost + IsolationForest + blend, fused)"}
        return {names[k]: round(ms / max(1, c) * 1e3, 3) for k, (ms, c) in timing.items() if c}

    def counter_groups(self, roof):
        """the hot kernels whose PMC figures the line carries: the feature pair and the scoring kernel"""
        lean = getattr(self, "pipe", None)
        if lean is None:
            lean = bool(getattr(getattr(getattr(self, "scorer", None), "be", None), "pipelined", True))
        # the lean kernel's template form: split scoring rows (<1, true>, the default when nothing asks for the
        # vectors) or the compact / full rows (<1, false>), as this run's engine counted them
        split = False
        try:
            split = self.eng.counter("pipelined_split_batches") > 0
        except Exception:
            pass
        bucket = (f"fd::anon::feat_bucket_lean_kernel<1, {'true' if split else 'false'}>" if lean
                  else "fd::anon::feat_bucket_kernel<1>")
        g = {"features": (["fd::anon::feat_slot_kernel", bucket], "features")}
        sym = (roof or {}).get("kernel_symbol")
        if sym:
            g["ensemble"] = ([sym], "ensemble (XGBoost + IsolationForest + blend, fused)")
        return g

    def config(self, world):
        return {"workload": "config3: card-state features (sliding 5m/1h/24h windows, HBM-resident) -> "
                            "XGBoost 500x8 + IsolationForest 100 -> blend/decision, 64k-txn micro-batches",
                "cards": self.cards, "window_mode": "sliding" if self.mode else "redis_compat", "ring_k": self.K,
                "trees": self.T, "depth": self.D, "features": 64, "batch": self.B,
                "parallelism": f"replicas x{world}"}

    def cpu_baseline(self, seconds):
        return cpu_chain_baseline(self.xgb, self.ifm, self.weights, self.mults, self.mode, self.K,
                                  lstm=self.lw if self.with_lstm else None, seq_len=self.seq_len)


# --------------------------------------------------------------------------------------- config 5
class Config5(Config3):
    """BASELINE configs[4]: the ensemble with the LSTM sequence head on the matrix cores, latency-bound
    1k-transaction micro-batches: card-state features (+ each card's last 10 events) -> XGBoost 500x8
    + IsolationForest 100 (main stream) || LSTM(128) over the card histories (f32 MFMA, second stream)
    -> blend/decision. p99 micro-batch latency is the headline here."""
    name = "config5"
    with_lstm = True
    pipelined_default = False  # 1k latency batches: the per-call cost is the bound, one stream is faster
    # a captured hipGraph per step measured slower here (0.103 vs 0.097 ms/step, round 2) and was removed

    def roofline(self, timing):
        N = self.N
        ms, launches = timing[N.FD_TIMING_LSTM]
        avg = (ms / 1e3) / max(1, launches)
        H, I, T = 128, 16, self.seq_len
        flops = self.B * T * 2 * 4 * H * (I + H) + self.B * 2 * H  # gates GEMMs + dense head
        achieved = flops / avg / 1e12
        return {"bound": "mfma", "achieved": round(achieved, 4), "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / F32_MFMA_PEAK_TFLOPS, 6),
                "traffic": pmc_traffic(self.name, self.B, LSTM4_SYMBOL), "kernel_samples": launches,
                "kernel": "lstm_kernel4 (v_mfma_f32_4x4x1_16b_f32, 4 transactions per workgroup)",
                "kernel_avg_us": round(avg * 1e6, 3), "flops_per_launch": flops, "flops_per_txn": flops // self.B,
                "note": "latency-bound 1k batch; f32 MFMA = reference fp32 precision; the launch also carries the forest "
                        "pair's tree-split binning workgroups (engine option latency_prebin, DESIGN §3), timed with it"}

    def counter_groups(self, roof):
        # batches of <= 4096 transactions: the slot pass runs inside the bucket launch (engine option slot_gather)
        gather = self.B <= 4096 and "slot_gather=0" not in [kv.replace(" ", "") for kv in self.args.engine_option]
        feats = (["fd::anon::feat_bucket_gather_kernel<1>"] if gather
                 else ["fd::anon::feat_slot_kernel", "fd::anon::feat_bucket_kernel<1>"])
        return {"features": (feats, "features"), "lstm_head": ([LSTM4_SYMBOL], "lstm_head")}

    def config(self, world):
        c = super().config(world)
        c["workload"] = ("config5: card-state features (sliding windows + last-10-event history) -> XGBoost 500x8 "
                         "+ IsolationForest 100 || LSTM(128) head on f32 MFMA -> blend/decision, latency-bound "
                         "1k-txn micro-batches")
        c["lstm"] = {"hidden": 128, "seq_len": self.seq_len, "input": 16, "head": "dense(1)+sigmoid"}
        return c


# --------------------------------------------------------------------------------------- config 4
class Config4(Config3):
    """BASELINE configs[3] (the metric's configuration): card-hash-sharded keyed state + scoring, RCCL
    all-to-all routing. Each rank ingests its own 64k-txn micro-batch per step (drawn over ALL cards) and
    routes every transaction to the GPU owning its card (fdengine.sharding.ShardedScorer). Cards: 100M
    over the node (each GPU holds only the cards it owns). At N=1 the whole node's cards are on the one GPU and
    ShardedScorer scores the ingest batch itself (fd_score_batch_pipelined: no routing kernels, no collective).

    Stream (--stream warm, the default): every card transacts floor(Gamma(2,2)) + 1 times a day
    (simulator.py:229), arrivals are Poisson at the node's rate sum(freq) / 86 400 s (each rank ingests 1/N of
    it), and --history-hours (24) of that stream run through the engine's feature path before the first
    measured batch, so the 5 min / 1 h / 24 h windows hold the events the reference's per-user state would
    (fdengine.synth_gpu.warm_workload). --stream cold: round 2's stream — cards uniform over all 100M at
    2,000 txn/s from an empty state (most transactions meet a card with no history)."""
    name = "config4"

    def __init__(self, args, rank, dev, eng):
        import numpy as np
        import torch
        from fdengine import _native as N
        from fdengine import synth
        from fdengine.sharding import EngineShardBackend, ShardedScorer
        self.np, self.torch, self.N = np, torch, N
        self.B, self.T, self.D = args.batch, args.trees, args.depth
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = rank
        self.cards = args.cards
        self.mode, self.K = (1 if args.window == "sliding" else 0), args.ring_k
        self.eng = eng
        self.stream = args.stream
        self.hours = args.history_hours if args.stream == "warm" else 0.0
        t = time.time()
        self.merchants = synth.merchants_table(5000, seed=100)
        self.xgb, self.ifm = fit_models(dev.index, self.T, self.D, self.mode, self.K)
        eng.load_forest(0, self.xgb)
        eng.load_forest(1, self.ifm)
        self.names = ["xgboost_primary", "isolation_forest"]
        self.with_lstm = False
        self.params, self.weights, self.mults = product_blend(self.names)
        n_own_est = self.cards // self.world
        cap = 1
        # load factor ~0.75 (1.25 slots per owned card, as a power of two): the open-addressed key array stays a
        # linear probe of a line or two, and 100 M cards with K = 64 ring events (1152 B per slot) fit one GPU's HBM
        # (2^27 slots = 155 GB); the same factor at every N keeps the per-GPU work the same (weak scaling)
        while cap < int(n_own_est * args.slots_per_card) + 65536:
            cap *= 2
        self.cap = cap
        eng.state_init(cap, self.mode, self.K)
        eng.load_merchants(self.merchants["fraud_rate"], self.merchants["risk_multiplier"])
        self.parity_batches = args.parity_batches
        # + 1: the parity twin batch (vectors requested)
        self.n_batches = args.warmup + args.steps + args.latency_iters + args.alone_iters + args.parity_batches + 1 \
            + args.loaded_iters + args.timing_steps + 1 + _diag_blocks() * args.steps + _diag_offset()
        B = self.B
        h2d_batches = args.latency_iters if args.latency_iters > 0 else 0
        self.warm_info = None
        if self.stream == "warm":
            from fdengine import synth_gpu
            gather = None
            if self.world > 1 and self.parity_batches:  # the node's parity batches touch cards of every owner
                import torch.distributed as dist

                def gather(k):
                    parts = [torch.empty_like(k) for _ in range(self.world)]
                    dist.all_gather(parts, k)
                    return torch.cat(parts)
            w = synth_gpu.warm_workload(eng, dev, self.cards, rank, self.world, self.n_batches, B, hours=self.hours,
                                        keep_batches=self.parity_batches + 1, host_batches=h2d_batches, log=log,
                                        gather_keys=gather)
            self.dev = w["resident"]
            self.tx = w["head"]  # host copies of the parity batches
            self.hist_rows, self.profiles = w["history_rows"], w["profiles"]
            self.n_owned = w["n_owned"]
            self.h2d_pool = w["host_batches"]
            self.warm_info = {"history_hours": self.hours, "history_transactions": w["history_transactions"],
                              "history_setup_s": w["history_seconds"], "node_rate_txn_per_s": round(
                                  w["rate_per_s_node"], 1), "card_frequency": "floor(Gamma(2,2))+1 per day"}
            del w
        else:
            own = synth.owned_cards(self.cards, rank, self.world, seed=42)  # this GPU's cards
            self.n_owned = len(own["key"])
            eng.load_users(own["key"], own["avg_amount"], own["account_age_days"], own["device_fp"])
            del own
            self.tx = synth.txn_stream_cards(self.cards, self.merchants, (self.n_batches + h2d_batches) * B,
                                             seed=200 + rank, card_seed=42, rate_per_s=2000.0)
            self.dev = {f: torch.from_numpy(np.ascontiguousarray(self.tx[f][:self.n_batches * B])).to(dev)
                        for f in N.TXN_FIELDS}
            self.h2d_pool = [{f: torch.from_numpy(np.ascontiguousarray(
                self.tx[f][(self.n_batches + q) * B:(self.n_batches + q + 1) * B]))
                for f in N.TXN_FIELDS} for q in range(h2d_batches)]
            self.hist_rows = None
        # world 1: the stream of resident micro-batches goes through fd_score_batch_pipelined (batch i+1's
        # features overlap batch i's forests); the inputs were complete before the first step (setup sync)
        self.scorer = ShardedScorer(EngineShardBackend(eng, self.params, [0, 1],
                                                       pipelined=not args.no_pipeline), rank, self.world)
        self.out = None
        # the latency loops' host-mapped output ring, allocated here: allocated at the first step_to_host it cost that
        # step 1.77 ms of host time (hipHostMalloc x 8: the loaded loop's sample 0 at 1.92 ms)
        self.host_out = HostOutRing(B, 8) if (self.world == 1 or self.scorer.native) else None
        # the resident micro-batches as column views, made once (a serving loop hands the scorer batches it already
        # holds; slicing nine columns per step is harness cost, ~10-20 us of Python)
        self.parts = [{f: t[b * B:(b + 1) * B] for f, t in self.dev.items()} for b in range(self.n_batches)]
        # caller-owned outputs, two sets alternating by batch (ShardedScorer.step out=: the engine's output copy
        # writes them in stream order, so batch i+2 reuses batch i's set after it); the Python exchange (gloo
        # rehearsal) allocates its own
        self.out_sets = None
        if self.world == 1 or self.scorer.native:
            self.out_sets = [tuple(torch.empty(B, dtype=d, device=dev) for d in (torch.float64, torch.float64,
                                                                                  torch.uint8, torch.uint8))
                             for _ in range(2)]
        self.h_fp = torch.empty(B, dtype=torch.float64, pin_memory=True)
        self.h_dec = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        self.h_risk = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        # host-resident micro-batches for the PCIe-inclusive latency line, packed into one pinned block each (fresh
        # batches continuing the stream after the resident ones): ONE H2D of the 35 B/txn columns on the engine
        # stream, the step on the staged copy (input_ready event), results into host-mapped memory
        self.h2d = None
        if self.h2d_pool:
            self.h2d = PackedColumns(self.h2d_pool[0], len(self.h2d_pool), dev)
            for q, cols in enumerate(self.h2d_pool):
                self.h2d.fill(q, cols)
            self.h2d_pool = self.h2d.host
            self.h2d_ev = [torch.cuda.Event() for _ in range(2)]
            for ev in self.h2d_ev:  # created at their first record, before any timed loop
                ev.record()
        self.h2d_bytes = self.h2d.nbytes if self.h2d else 0
        self.next_batch = 0
        self.next_h2d = 0
        torch.cuda.synchronize()
        log(f"[rank {rank}] config4 setup {time.time() - t:.1f}s ({self.stream} stream): {self.cards} cards over "
            f"{self.world} GPU(s), {self.n_owned} owned here, capacity {cap}, {self.n_batches} batches resident")

    def step(self, i, **kw):
        b = self.next_batch
        if b >= self.n_batches:
            raise RuntimeError("stream exhausted: raise n_batches")
        self.next_batch += 1
        B = self.B
        # the batch the previous step prefetched is passed as the very same mapping (ShardedScorer names a prefetch
        # to the engine by identity, not by address)
        part = self.parts[b]  # views made once at setup (the same mapping object when it was the prefetch)
        if self.world > 1 and b + 1 < self.n_batches:  # the next batch's partition + count exchange, one step ahead
            kw["prefetch"] = (self.parts[b + 1], B)
        if "out" not in kw and self.out_sets is not None:
            kw["out"] = self.out_sets[b & 1]
        self.out = self.scorer.step(part, B, **kw)

    def step_to_host(self, i, q):
        """one step whose outputs land in host-mapped pinned memory (HostOutRing set q): no separate D2H"""
        if self.world > 1 and not self.scorer.native:  # out= needs one shard or the native sharded step
            self.step(i)
            self.fetch(i)
            return
        if self.host_out is None:
            self.host_out = HostOutRing(self.B, 8)
        self.step(i, out=self.host_out.sets[q % 8])

    def step_h2d(self, i):
        """One micro-batch from pinned host memory: one H2D copy of the packed columns, the step on the staged copy,
        its results into host-mapped pinned memory (the engine's output kernel; no D2H call) — or, where the step
        cannot take host outputs (N > 1 over the Python exchange), a D2H of the results."""
        if self.next_h2d >= len(self.h2d_pool):
            raise RuntimeError("host stream exhausted")
        src = self.h2d_pool[self.next_h2d]
        self.next_h2d += 1
        q = i & 1
        st = self.torch.cuda.current_stream()
        hip_memcpy_async(self.h2d.dev[q].data_ptr(), src.data_ptr(), self.h2d.nbytes, 1, st.cuda_stream)
        ev = self.h2d_ev[q]
        ev.record(st)
        if self.world > 1 and not self.scorer.native:
            self.out = self.scorer.step(self.h2d.dev_views[q], self.B, input_ready=ev)
            self.fetch(i)
            return
        if self.host_out is None:
            self.host_out = HostOutRing(self.B, 8)
        self.out = self.scorer.step(self.h2d.dev_views[q], self.B, input_ready=ev, out=self.host_out.sets[i % 8])

    def fetch(self, i):
        """the step's fraud_prob / decision / risk to pinned host memory, queued on the stream (hipMemcpyAsync
        directly: torch's copy_ into pinned memory also does the caching host allocator's per-copy event
        bookkeeping, measured to stall the host for ~6 ms about once per 100-200 copies; FD_FETCH=torch for it)"""
        fp, conf, dec, risk = self.out
        if os.environ.get("FD_FETCH") == "torch":
            self.h_fp.copy_(fp, non_blocking=True)
            self.h_dec.copy_(dec, non_blocking=True)
            self.h_risk.copy_(risk, non_blocking=True)
            return
        st = self.torch.cuda.current_stream().cuda_stream
        for h, d in ((self.h_fp, fp), (self.h_dec, dec), (self.h_risk, risk)):
            hip_d2h(h.data_ptr(), d.data_ptr(), d.numel() * d.element_size(), st)

    def parity(self):
        """N=1: the first parity_batches micro-batches through the product path (the pipelined ShardedScorer step,
        vectors and model probabilities requested) against the oracle chain. The oracle state holds just the cards
        those batches touch: their profiles and, on the warm stream, their history rows (per-card state is
        independent), replayed before the batches. N>1: every rank steps the same number of batches (the exchange
        is checked by tests/test_sharding.py, gloo, and tests/test_gpu_sharding*.py)."""
        if self.world > 1:
            return self._parity_sharded()
        import oracle
        from fdengine import synth
        from oracle.features_c import OracleFeatureState
        np, torch = self.np, self.torch
        P, B = self.parity_batches, self.B
        o = OracleFeatureState(1 << 22, self.mode, self.K)
        if self.stream == "warm":
            at = self.profiles
        else:
            at = synth.card_attrs(self.tx["card_id"][:(P + 1) * B], 42)  # the profiles of the cards these batches touch
            _, first = np.unique(at["key"], return_index=True)
            at = {k: v[first] for k, v in at.items()}
        o.load_users(at["key"], at["avg_amount"], at["account_age_days"], at["device_fp"])
        o.load_merchants(self.merchants["fraud_rate"], self.merchants["risk_multiplier"])
        if self.hist_rows is not None and len(self.hist_rows["card_key"]):
            o.run(self.hist_rows, want_raw=False)
        out = _parity_record(P, "ShardedScorer world 1 -> fd_score_batch_pipelined, no vectors requested: the fused "
                             "ensemble kernel from the compact 64-B rows (the timed variant); twin: one more "
                             "batch with vectors + model probabilities requested (64-wide vectors)", B)
        out["stream"] = self.stream
        vec = torch.empty((B, 64), dtype=torch.float32, device=self.dev["ts_ms"].device)
        mp = torch.empty((2, B), dtype=torch.float64, device=vec.device)
        raws = []
        sat0 = _saturated(self.eng, self)
        c0 = self.eng.counter("pipelined_compact_batches")
        q0 = self.eng.counter("pipelined_split_batches")
        s0 = self.eng.counter("pipelined_slot_stream_batches")
        for b in range(P + 1):
            twin = b == P
            part = {f: self.tx[f][b * B:(b + 1) * B] for f in self.N.TXN_FIELDS}
            if twin:
                self.step(b, vectors=vec, model_probs=mp)
            else:
                self.step(b)
            torch.cuda.synchronize()
            raw, rvec = o.run(part, want_raw=True)
            raws.append(raw)
            px, _, _ = oracle.xgb_predict(self.xgb, rvec, nthreads=cpu_threads())
            pi, _, _ = oracle.iforest_predict(self.ifm, rvec, nthreads=cpu_threads())
            ref = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), self.weights, self.mults)
            leg = out["twin" if twin else "timed_path"]
            _parity_compare(leg, [t.cpu().numpy() for t in self.out], ref)
            if twin:
                _parity_vectors(leg, vec.cpu().numpy(), rvec)
                M = mp.cpu().numpy()
                leg["max_abs_model_prob_diff"] = max(float(np.abs(M[0] - px).max()), float(np.abs(M[1] - pi).max()))
        out["timed_path"]["compact_batches"] = self.eng.counter("pipelined_compact_batches") - c0
        out["timed_path"]["split_row_batches"] = self.eng.counter("pipelined_split_batches") - q0
        out["timed_path"]["slot_stream_batches"] = self.eng.counter("pipelined_slot_stream_batches") - s0
        from fdengine.synth_gpu import occupancy
        allraw = np.concatenate(raws)
        self.occupancy = dict(occupancy(allraw), basis=f"the {P} parity micro-batches (raw velocity "
                              "counts of the oracle, whose vectors equal the engine's)")
        if sat0 is not None:  # transactions whose 24 h window held all K ring events: engine counter vs oracle
            out["window_saturated"] = {"engine": _saturated(self.eng, self) - sat0,
                                       "oracle": int((allraw[:, 11] >= self.K).sum())}
        del o
        return out

    def _parity_sharded(self):
        """N > 1: every rank scores its first parity_batches micro-batches through the product path (ShardedScorer ->
        fd_sharded_step over RCCL, the next batch prefetched as in the timed steps); rank 0 gathers every rank's
        batches, results, kept history rows (the owned cards any rank's parity batches touch, warm_workload
        gather_keys) and profiles, and replays the node's stream through the oracle chain in the order the sharded
        step defines — step-major, then ingest rank, then index (keyBy, WindowProcessor.java:44,63)."""
        import torch.distributed as dist
        np, torch = self.np, self.torch
        P, B, G = self.parity_batches, self.B, self.world
        outs = []
        for b in range(P):
            self.step(b)
            outs.append([t.cpu().numpy() for t in self.out])
        mine = {"head": self.tx, "hist": self.hist_rows, "profiles": self.profiles, "outs": outs,
                "stream": self.stream}
        got = [None] * G if self.rank == 0 else None
        dist.gather_object(mine, got, dst=0)
        if self.rank != 0:
            return None
        import oracle
        from oracle.features_c import OracleFeatureState
        o = OracleFeatureState(1 << 23, self.mode, self.K)
        if self.stream == "warm":
            prof = {k: np.concatenate([g["profiles"][k] for g in got]) for k in got[0]["profiles"]}
            _, first = np.unique(prof["key"], return_index=True)
            prof = {k: v[first] for k, v in prof.items()}
            o.load_users(prof["key"], prof["avg_amount"], prof["account_age_days"], prof["device_fp"])
        else:
            from fdengine import synth
            at = synth.card_attrs(np.concatenate([g["head"]["card_id"][:P * B] for g in got]), 42)
            _, first = np.unique(at["key"], return_index=True)
            at = {k: v[first] for k, v in at.items()}
            o.load_users(at["key"], at["avg_amount"], at["account_age_days"], at["device_fp"])
        o.load_merchants(self.merchants["fraud_rate"], self.merchants["risk_multiplier"])
        hist = [g["hist"] for g in got if g["hist"] is not None and len(g["hist"]["card_key"])]
        if hist:  # disjoint card sets (each card's history lives on its owner), each in arrival order
            o.run({f: np.concatenate([h[f] for h in hist]) for f in self.N.TXN_FIELDS}, want_raw=False)
        out = {"batches_checked": P * G, "ranks": G, "path": "ShardedScorer -> fd_sharded_step (RCCL all-to-all)",
               "order": "step-major, then ingest rank, then index", "stream": self.stream,
               "max_abs_prob_diff": 0.0, "max_abs_conf_diff": 0.0, "decision_mismatches": 0, "risk_mismatches": 0,
               "decision_mismatches_off_threshold": 0, "history_rows_replayed": int(sum(len(h["card_key"])
                                                                                       for h in hist))}
        for b in range(P):
            for r in range(G):
                part = {f: got[r]["head"][f][b * B:(b + 1) * B] for f in self.N.TXN_FIELDS}
                _, V = o.run(part, want_raw=False)
                px, _, _ = oracle.xgb_predict(self.xgb, V, nthreads=cpu_threads())
                pi, _, _ = oracle.iforest_predict(self.ifm, V, nthreads=cpu_threads())
                fp, conf, dec, risk = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), self.weights,
                                                            self.mults)
                gfp, gconf, gdec, grisk = got[r]["outs"][b]
                out["max_abs_prob_diff"] = max(out["max_abs_prob_diff"], float(np.abs(gfp - fp).max()))
                out["max_abs_conf_diff"] = max(out["max_abs_conf_diff"], float(np.abs(gconf - conf).max()))
                bad = gdec != dec
                out["decision_mismatches"] += int(bad.sum())
                out["risk_mismatches"] += int((grisk != risk).sum())
                near = np.zeros(len(fp), bool)  # the f32 XGBoost sigmoid may sit an ulp from the oracle's
                for thr in (0.6, 0.8, 0.95):
                    near |= np.abs(fp - thr) < 1e-6
                near |= np.abs(conf - 0.7) < 1e-6
                out["decision_mismatches_off_threshold"] += int((bad & ~near).sum())
        del o
        return out

    def config(self, world):
        return {"workload": "config4: card-hash-sharded keyed state (fmix64 owner) + RCCL all-to-all routing "
                            "(48-B txn records out, 24-B results back) -> features + XGBoost 500x8 + "
                            "IsolationForest 100 + blend on the owner, 64k-txn micro-batch per GPU per step",
                "cards": self.cards, "cards_per_gpu": self.n_owned, "card_slots": self.cap, "window_mode": "sliding" if self.mode else
                "redis_compat", "ring_k": self.K, "trees": self.T, "depth": self.D, "features": 64,
                "batch_per_gpu": self.B, "global_batch": self.B * world,
                "stream": self.stream, "warm_state": self.warm_info,
                "window_occupancy": getattr(self, "occupancy", None),
                "parallelism": f"card-hash shards x{world}, RCCL all-to-all" if world > 1 else
                "1 shard (all cards on one GPU): the ingest batch scored in place through fd_score_batch_pipelined "
                "- no routing kernels, no collective"}


# --------------------------------------------------------------------------------------- ingest
class Ingest:
    """The Kafka JSON codec alone: 64k simulator-format messages (~790 B) resident in
    HBM -> SoA columns in HBM, one fd_ingest_json_device per step. A pool of distinct batches is cycled so the
    256 MB MALL cannot hold the input."""
    name = "ingest"
    dtype = "u8 (bytes; f64 for parsed decimals)"
    OUT_BYTES = 8 * 10 + 4 + 1 * 10  # the 20 output columns per message

    def __init__(self, args, rank, dev, eng):
        import numpy as np
        import torch
        from fdengine import _native as N
        from fdengine import synth
        from fdengine.ingest import IngestCodec, device_columns, pack
        self.np, self.torch, self.N = np, torch, N
        self.B = args.batch
        self.eng = eng
        t = time.time()
        self.merchant_ids = [f"merchant_{i:08x}" for i in range(5000)]
        self.codec = IngestCodec(eng, self.merchant_ids, synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                                 synth.SIM_CARD_TYPES)
        self.msgs = synth.json_messages_fast(self.B, 10_000_000, self.merchant_ids, seed=300 + rank)
        buf, off = pack(self.msgs)
        self.nbytes = int(off[-1])
        self.pool = max(1, args.pool)
        stride = (self.nbytes + 4095) & ~4095  # pool copies at distinct addresses (16-B aligned strides)
        host = np.zeros(self.pool * stride, np.uint8)
        for p in range(self.pool):
            host[p * stride:p * stride + self.nbytes] = buf
        self.stride = stride
        self.buf = torch.from_numpy(host).to(dev)
        self.off = torch.from_numpy(off).to(dev)
        self.offsets = off
        self.cols, self.ptrs = device_columns(self.B, dev.index)
        self.h_status = torch.empty(self.B, dtype=torch.uint8, pin_memory=True)
        log(f"[rank {rank}] ingest setup {time.time() - t:.1f}s: {self.B} messages, {self.nbytes / self.B:.0f} B avg, "
            f"pool {self.pool}")

    def step(self, i):
        s = i % self.pool
        self.codec.parse_device(self.buf.data_ptr() + s * self.stride, self.off.data_ptr(), self.B, self.ptrs)

    def fetch(self, i):
        d = self.cols["status"]
        hip_d2h(self.h_status.data_ptr(), d.data_ptr(), d.numel() * d.element_size(),
                self.torch.cuda.current_stream().cuda_stream)

    def parity(self):
        from oracle import ingest_ref as R
        from fdengine import synth
        np = self.np
        self.step(0)
        self.torch.cuda.synchronize()
        k = 4096
        exp = R.parse_batch(self.msgs[:k], {m: i for i, m in enumerate(self.merchant_ids)},
                            [{s: i for i, s in enumerate(v)} for v in (synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                                                                      synth.SIM_CARD_TYPES)])
        bad = 0
        for name, dt in self.N.INGEST_FIELDS:
            g = self.cols[name][:k].cpu().numpy().view(dt)
            e = exp[name]
            if g.dtype.kind == "f":
                bad += int((~((g.view(np.uint64) == e.view(np.uint64)) | (np.isnan(g) & np.isnan(e)))).sum())
            else:
                bad += int((g != e).sum())
        return {"messages_checked": k, "mismatched_values": bad,
                "invalid_rows": int((exp["status"] & R.INVALID != 0).sum())}

    def _avg(self, timing):
        ms, launches = timing[self.N.FD_TIMING_INGEST]
        return (ms / 1e3) / max(1, launches)

    def roofline(self, timing):
        avg = self._avg(timing)
        per_launch = self.nbytes + 8 * (self.B + 1) + self.OUT_BYTES * self.B
        achieved = per_launch / avg / 1e9
        return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(self.name, self.B, INGEST_SYMBOL),
                "kernel": "ingest_json_kernel (wave per message, LDS-staged)", "kernel_avg_us": round(avg * 1e6, 3),
                "algorithmic_bytes_per_launch": per_launch,
                "bytes_per_txn": round(per_launch / self.B, 1)}

    def kernels(self, timing):
        return {"ingest_json": round(self._avg(timing) * 1e6, 3)}

    def config(self, world):
        return {"workload": "ingest: Kafka JSON codec — 64k simulator-format transaction messages "
                            "(json.dumps(asdict(Transaction), default=str)) resident in HBM -> SoA columns",
                "batch": self.B, "avg_message_bytes": round(self.nbytes / self.B, 1),
                "parallelism": f"replicas x{world}"}

    def cpu_baseline(self, seconds):
        """The reference's CPU path for this step restated: Python json.loads + the field mapping
        (oracle/ingest_ref.py) on one core, over the batch's messages."""
        from oracle import ingest_ref as R
        from fdengine import synth
        merch = {m: i for i, m in enumerate(self.merchant_ids)}
        voc = [{s: i for i, s in enumerate(v)} for v in (synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                                                          synth.SIM_CARD_TYPES)]
        done, a = 0, time.perf_counter()
        while time.perf_counter() - a < seconds:
            R.parse_message(self.msgs[done % self.B], merch, voc)
            done += 1
        dt = time.perf_counter() - a
        return {"value": round(done / dt, 1), "unit": "txn/s", "cores": 1, "kind": "port",
                "sample": f"{done} messages of the batch through oracle/ingest_ref.py (json.loads + field mapping, "
                          f"1 core), {dt:.2f} s, CPU: {cpu_model()}"}


# --------------------------------------------------------------------------------------- config 3 from JSON
class Config3J(Config3):
    """config 3 fed from the wire format: per step one micro-batch of 64k raw Kafka JSON messages (resident in
    HBM) -> ingest codec -> card-state features (10M cards) -> XGBoost 500x8 + IsolationForest -> blend.
    Cards are keyed by fd_hash64(user_id) as the codec keys them."""
    name = "config3j"

    def __init__(self, args, rank, dev, eng):
        import numpy as np
        import torch
        from fdengine import _native as N
        from fdengine import synth
        from fdengine.ingest import IngestCodec, device_columns, pack
        self.np, self.torch, self.N = np, torch, N
        self.B, self.T, self.D = args.batch, args.trees, args.depth
        self.cards, self.mode, self.K = args.cards, (1 if args.window == "sliding" else 0), args.ring_k
        self.eng = eng
        self.with_lstm = False
        t = time.time()
        self.xgb, self.ifm = fit_models(dev.index, self.T, self.D, self.mode, self.K)
        eng.load_forest(0, self.xgb)
        eng.load_forest(1, self.ifm)
        self.names = ["xgboost_primary", "isolation_forest"]
        self.slots = [0, 1]
        self.params, self.weights, self.mults = product_blend(self.names)
        # users keyed as the codec keys them: fd_hash64("user_xxxxxxxx"), fingerprints fd_hash64("fp-xxxxxxxx")
        idx = np.arange(self.cards, dtype=np.uint64)
        self.ukeys = synth.hash64_fixed(synth.fixed_ids("user_", idx))
        self.uavg = np.exp(4.0 + np.sqrt(2) * synth._erfinv(2 * synth._u01(idx, 42, 0) - 1))
        self.uage = (synth._u01(idx, 42, 1) * 730).astype(np.int32)
        self.ufp = np.stack([synth.hash64_fixed(synth.fixed_ids("fp-", idx * np.uint64(3) + np.uint64(k)))
                             for k in range(3)], axis=1)
        self.merchant_ids = [f"merchant_{i:08x}" for i in range(5000)]
        self.merchants = synth.merchants_table(5000, seed=100 + rank)
        cap = 1
        while cap < int(self.cards * 1.6):
            cap *= 2
        self.cap = cap
        eng.state_init(cap, self.mode, self.K)
        eng.load_users(self.ukeys, self.uavg, self.uage, self.ufp)
        eng.load_merchants(self.merchants["fraud_rate"], self.merchants["risk_multiplier"])
        # pipelined (default): the codec runs on an engine of its own with its own stream, so batch i+1's parse
        # overlaps batch i's scoring on the pipelined stream; two column sets, handed over by events (the scoring
        # waits for its parse; a set's next parse waits for the scoring that read it)
        self.pipe, self.cur = not args.no_pipeline, 0
        self.extra_engines = []
        codec_eng = eng
        if self.pipe:
            import fdengine
            self.ceng = fdengine.FraudEngine(dev.index)
            self.cstream = torch.cuda.Stream(device=dev)
            self.ceng.set_stream(self.cstream.cuda_stream)
            for kv in args.engine_option:  # --engine-option applies to the codec engine too
                k, v = kv.split("=")
                self.ceng.set_option(k.strip(), int(v))
            self.extra_engines = [self.ceng]
            codec_eng = self.ceng
        self.codec = IngestCodec(codec_eng, self.merchant_ids, synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES,
                                 synth.SIM_CARD_TYPES)
        self.pool = max(1, min(args.pool, 4))
        self.msgs, bufs, offs = [], [], []
        for p in range(self.pool):
            ms = synth.json_messages_fast(self.B, self.cards, self.merchant_ids, seed=400 + 17 * rank + p,
                                          t0_ms=1_757_030_400_000 + p * 60_000)
            b, o = pack(ms)
            self.msgs.append(ms)
            bufs.append(torch.from_numpy(b.copy()).to(dev))
            offs.append(torch.from_numpy(o).to(dev))
        self.bufs, self.offs = bufs, offs
        # three column sets: batch i+3's parse reuses batch i's set after its scoring — the parse of i+1 (whose
        # VALU-bound workgroups fill the CUs' registers, so batch i's feature kernels mostly run after it) and batch
        # i's scoring then never stall the codec stream (with two sets it idled ~90 us per batch)
        self.nsets = 3 if self.pipe else 1
        self.csets = [device_columns(self.B, dev.index) for _ in range(self.nsets)]
        self.cols, self.cptrs = self.csets[0]
        self.ready = [torch.cuda.Event() for _ in range(self.nsets)]
        self.freed, self.freed_live = [torch.cuda.Event() for _ in range(self.nsets)], [False] * self.nsets
        self.dev_stream = torch.cuda.current_stream(dev)
        B = self.B
        self.fp = torch.empty(B, dtype=torch.float64, device=dev)
        self.conf = torch.empty(B, dtype=torch.float64, device=dev)
        self.dec = torch.empty(B, dtype=torch.uint8, device=dev)
        self.risk = torch.empty(B, dtype=torch.uint8, device=dev)
        self.mp = torch.empty((len(self.names), B), dtype=torch.float64, device=dev)
        self.vec = torch.empty((B, 64), dtype=torch.float32, device=dev)
        self.h_fp = torch.empty(B, dtype=torch.float64, pin_memory=True)
        self.h_dec = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        self.h_risk = torch.empty(B, dtype=torch.uint8, pin_memory=True)
        self.outs = [[self.fp, self.conf, self.dec, self.risk]] + [
            [torch.empty_like(t) for t in (self.fp, self.conf, self.dec, self.risk)]
            for _ in range(max(2, self.nsets) - 1)]  # Config3.fetch
        self.scorer = eng.pipelined_scorer(self.params, self.slots)
        self.nbytes = [int(o[-1].item()) for o in offs]
        log(f"[rank {rank}] config3j setup {time.time() - t:.1f}s: {self.cards} cards, capacity {cap}, "
            f"{self.pool} JSON batches resident ({self.nbytes[0] / B:.0f} B/message)")

    def step(self, i):
        s = i % self.pool
        if not self.pipe:  # one stream (the codec on the engine's), vectors kept
            self.codec.parse_device(self.bufs[s].data_ptr(), self.offs[s].data_ptr(), self.B, self.cptrs)
            txn = {f: self.cptrs[f] for f in self.N.TXN_FIELDS}
            self.cur = 0
            self.eng.score_batch_device(self.params, self.slots, txn, self.B, self.fp.data_ptr(),
                                        self.conf.data_ptr(), self.dec.data_ptr(), self.risk.data_ptr(),
                                        vec_ptr=self.vec.data_ptr(), model_probs_ptr=self.mp.data_ptr())
            return
        k = i % self.nsets
        _, cptrs = self.csets[k]
        if self.freed_live[k]:
            self.cstream.wait_event(self.freed[k])
        self.codec.parse_device(self.bufs[s].data_ptr(), self.offs[s].data_ptr(), self.B, cptrs)
        self.ready[k].record(self.cstream)
        self.cur = k
        fp, conf, dec, risk = self.outs[k]
        self.scorer({f: cptrs[f] for f in self.N.TXN_FIELDS}, self.B, fp.data_ptr(), conf.data_ptr(), dec.data_ptr(),
                    risk.data_ptr(), input_ready=self.ready[k].cuda_event)
        self.freed[k].record(self.dev_stream)  # the engine stream: past this batch's scoring (its output copy)
        self.freed_live[k] = True

    def parity(self):
        """Batch 0 (fresh state) through the timed path (codec stream -> pipelined scoring from compact vectors; with
        --no-pipeline one stream, vectors kept and compared too) against oracle ingest -> oracle features -> forests
        -> blend on the oracle's own vectors, first 8192 rows."""
        import oracle
        from fdengine import synth
        from oracle import ingest_ref as R
        from oracle.features_c import OracleFeatureState
        np = self.np
        k = 8192
        o = OracleFeatureState(self.cap, self.mode, self.K)
        o.load_users(self.ukeys, self.uavg, self.uage, self.ufp)
        o.load_merchants(self.merchants["fraud_rate"], self.merchants["risk_multiplier"])
        c0 = self.eng.counter("pipelined_compact_batches")
        q0 = self.eng.counter("pipelined_split_batches")
        self.step(0)
        self.torch.cuda.synchronize()
        cols = R.parse_batch(self.msgs[0][:k], {m: i for i, m in enumerate(self.merchant_ids)},
                             [{s: i for i, s in enumerate(v)} for v in (synth.SIM_PAYMENT_METHODS,
                                                                         synth.SIM_TXN_TYPES, synth.SIM_CARD_TYPES)])
        _, rvec = o.run({f: cols[f] for f in self.N.TXN_FIELDS}, want_raw=False)
        del o
        px, _, _ = oracle.xgb_predict(self.xgb, rvec, nthreads=cpu_threads())
        pi, _, _ = oracle.iforest_predict(self.ifm, rvec, nthreads=cpu_threads())
        ref = [np.ascontiguousarray(a) for a in oracle.blend_weighted(np.stack([px.astype(np.float64), pi]),
                                                                       self.weights, self.mults)]
        got = [t[:k].cpu().numpy() for t in self.outs[self.cur]]
        out = _parity_record(1, "codec stream -> pipelined stream, fused kernel from compact vectors" if self.pipe
                             else "codec -> fd_score_batch_device", k)
        _parity_compare(out["timed_path"], got, ref)
        out["timed_path"]["compact_batches"] = self.eng.counter("pipelined_compact_batches") - c0
        out["timed_path"]["split_row_batches"] = self.eng.counter("pipelined_split_batches") - q0
        if not self.pipe:
            _parity_vectors(out["timed_path"], self.vec[:k].cpu().numpy(), rvec)
        del out["twin"]
        return out

    def kernels(self, timing):
        out = super().kernels(timing)
        ms, c = timing.get(self.N.FD_TIMING_INGEST, (0.0, 0))
        if c:
            out["ingest_json"] = round(ms / c * 1e3, 3)
        return out

    def roofline(self, timing):
        """The dominant kernel of this line is the JSON codec, not the forest."""
        ms, launches = timing[self.N.FD_TIMING_INGEST]
        avg = (ms / 1e3) / max(1, launches)
        per_launch = self.nbytes[0] + 8 * (self.B + 1) + Ingest.OUT_BYTES * self.B
        achieved = per_launch / avg / 1e9
        return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(self.name, self.B, INGEST_SYMBOL),
                "kernel": "ingest_json_kernel (wave per message, LDS-staged; dominant)",
                "kernel_avg_us": round(avg * 1e6, 3), "algorithmic_bytes_per_launch": per_launch,
                "bytes_per_txn": round(per_launch / self.B, 1)}

    def config(self, world):
        d = super().config(world)
        d["workload"] = ("config3j: config3 fed from the wire format — 64k raw Kafka JSON messages per micro-batch "
                         "resident in HBM -> ingest codec -> features (HBM card state) -> XGBoost 500x8 + "
                         "IsolationForest 100 -> blend/decision")
        d["avg_message_bytes"] = round(self.nbytes[0] / self.B, 1)
        return d


WORKLOADS = {"config2": Config2, "config3": Config3, "config4": Config4, "config5": Config5, "ingest": Ingest,
             "config3j": Config3J}


def _engines(eng, wl):
    """the scoring engine and any engine the workload runs beside it (config 3j's codec engine)"""
    return [eng] + list(getattr(wl, "extra_engines", []))


def _read_timing(eng, wl):
    out = {}
    for e in _engines(eng, wl):
        for k, (ms, c) in e.read_timing().items():
            a, b = out.get(k, (0.0, 0))
            out[k] = (a + ms, b + c)
    return out


def _host_counters(eng):
    """the engine's cumulative host-side counters for the pipelined / sharded step (None where unsupported)"""
    out = {}
    for k in ("pipelined_batches", "pipelined_host_ns", "sharded_steps", "rccl_ops"):
        try:
            out[k] = eng.counter(k)
        except Exception:
            out[k] = None
    return out


def _host_breakdown(h0, h1, submit_s, steps):
    """host submit time per step split into the native step call (HIP launches, event records / waits inside
    fd_score_batch_pipelined) and everything above it (bench loop, ShardedScorer, ctypes)"""
    if h0.get("pipelined_host_ns") is None or h1.get("pipelined_host_ns") is None:
        return None
    calls = h1["pipelined_batches"] - h0["pipelined_batches"]
    if calls <= 0:
        return None
    native = (h1["pipelined_host_ns"] - h0["pipelined_host_ns"]) / 1e3 / steps
    total = submit_s * 1e6 / steps
    out = {"native_us_per_step": round(native, 2), "above_native_us_per_step": round(total - native, 2),
           "pipelined_calls": calls, "basis": "engine counter pipelined_host_ns (steady_clock around "
                                              "fd_score_batch_pipelined's body) over the timed region"}
    if h0.get("rccl_ops") is not None and h1.get("rccl_ops") is not None and h1["rccl_ops"] > h0["rccl_ops"]:
        out["rccl_ops_per_step"] = round((h1["rccl_ops"] - h0["rccl_ops"]) / steps, 2)  # N > 1: sends / recvs / gathers
    return out


def _saturated(eng, wl):
    """the engine's cumulative window_saturated counter (sliding-window workloads; None otherwise)"""
    if getattr(wl, "mode", 0) != 1 or not hasattr(wl, "K"):
        return None
    try:
        return eng.counter("window_saturated")
    except Exception:
        return None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# RCCL ("nccl") is the product path: one rank per GPU. FD_BENCH_DIST_BACKEND=gloo is a rehearsal of the N-rank
# control flow on fewer GPUs (ranks share devices, exchanges staged through host memory): its numbers are not
# the metric, the line says so in config.dist_backend.
DIST_BACKEND = os.environ.get("FD_BENCH_DIST_BACKEND", "nccl")


LAT_SPLIT = ("total", "submit", "native", "wait", "gpu", "query_max", "gap_max")  # latency_split's columns (ms)


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: start N ranks (one process per GPU) with torch.distributed.run
    as children — before this process touches the GPU — and return their exit code."""
    import torch  # device_count() does not initialise the GPU on this image
    visible = torch.cuda.device_count()
    if n > visible and DIST_BACKEND == "nccl":
        log(f"--gpus {n} but only {visible} GPU(s) visible: refusing to oversubscribe")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    log("[bench] launching ranks:", " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config4")
    ap.add_argument("--batch", type=int, default=None, help="micro-batch per GPU (default 64k; config5: 1k)")
    ap.add_argument("--trees", type=int, default=500)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--features", type=int, default=50)
    ap.add_argument("--pool", type=int, default=8, help="config2/ingest: distinct HBM-resident micro-batches cycled")
    ap.add_argument("--cards", type=int, default=None,
                    help="cards resident in HBM (config4 default 100M over the node; config3 default 10M)")
    ap.add_argument("--window", choices=["sliding", "redis"], default="sliding")
    ap.add_argument("--slots-per-card", type=float, default=1.25,
                    help="config 4: card-table slots per owned card before rounding up to a power of two (1.25: "
                         "2^27 slots at 100 M cards, load ~0.75)")
    ap.add_argument("--ring-k", type=int, default=64,
                    help="sliding windows: ring events per card (the bench line reports window_saturation: "
                         "transactions whose 24 h window held all K)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", default=None,
                    help="config 4 at N = 1: other BASELINE configurations run after the line's own measurements, each "
                         "as a child process (its own engine, 200 steps), their results embedded as "
                         "secondary_workloads (comma list; default config5,config2,config3,config3j; 'none' or "
                         "FD_BENCH_SECONDARY=0 to skip)")
    ap.add_argument("--pipeline", action="store_true",
                    help="config5: the pipelined stream (batch i+1's features beside batch i's scoring) instead of "
                         "fd_score_batch_device per step")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="config3/4 at N=1: fd_score_batch_device per step instead of the pipelined stream")
    ap.add_argument("--small-streams", type=int, choices=[0, 1, 2], default=None,
                    help="engine option small_streams (latency batches: side streams for the LSTM / other forests)")
    ap.add_argument("--lstm-rows", type=int, choices=[0, 4, 16], default=None,
                    help="engine option lstm_rows (LSTM tile: 0 auto, 4 or 16 transactions per workgroup)")
    ap.add_argument("--engine-option", action="append", default=[], metavar="KEY=VALUE",
                    help="fd_engine_set_option before the workload's setup (A/B runs; the product defaults otherwise)")
    ap.add_argument("--latency-iters", type=int, default=200)
    ap.add_argument("--alone-iters", type=int, default=20,
                    help="steps run one at a time after the latency loop, every launch timed: each kernel's "
                         "duration with nothing beside it (roofline.alone)")
    ap.add_argument("--parity-batches", type=int, default=2)
    ap.add_argument("--timing-steps", type=int, default=160,
                    help="back-to-back steps after the timed region, kernel timing still sampled (kernel averages over "
                         ">= 20 launches even for short --steps)")
    ap.add_argument("--stream", choices=["warm", "cold"], default="warm",
                    help="config4: warm = SURVEY §8(d) stream (Gamma(2,2)+1 txn/card/day, Poisson arrivals) after "
                         "--history-hours of history through the feature path; cold = round 2's uniform stream "
                         "from an empty state")
    ap.add_argument("--history-hours", type=float, default=24.0)
    ap.add_argument("--loaded-inflight", type=int, default=3,
                    help="loaded-latency loop: micro-batches submitted and not yet returned at most")
    ap.add_argument("--loaded-iters", type=int, default=200,
                    help="steps of the loaded-latency loop: back to back like the timed region, each step's results "
                         "copied to pinned host memory, per-batch submit -> results-on-host times")
    return ap


def parse_args(argv=None):
    args = make_parser().parse_args(argv)
    if args.batch is None:
        args.batch = 1024 if args.workload == "config5" else 65536
    if args.cards is None:
        args.cards = 100_000_000 if args.workload == "config4" else 10_000_000
    return args


def main():
    args = parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[rank {rank}] note: --gpus {args.gpus} but WORLD_SIZE={world}; n_gpus reports the ranks running")

    import numpy as np
    import torch

    import fdengine

    dist = None
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count()) if DIST_BACKEND == "gloo" else local
        torch.cuda.set_device(local)
        if DIST_BACKEND == "gloo":
            dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
        else:
            dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank,
                                    device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng = fdengine.FraudEngine(dev.index)
    for kv in args.engine_option:
        k, v = kv.split("=")
        eng.set_option(k.strip(), int(v))
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    wl = WORKLOADS[args.workload](args, rank, dev, eng)
    if args.lstm_rows is not None:
        eng.set_option("lstm_rows", args.lstm_rows)
    if args.small_streams is not None:
        eng.set_option("small_streams", args.small_streams)

    parity = None
    try:
        parity = wl.parity()
    except Exception as e:  # the oracle is only a checker; report, never fall back
        log(f"[rank {rank}] parity spot-check unavailable: {e!r}")

    if _diag_offset() and hasattr(wl, "next_batch"):
        wl.next_batch += _diag_offset()
    # a serving process's setup is done: move every object allocated so far out of the cyclic collector's view
    # (a full collection over the setup's objects stalls the host for milliseconds mid-stream)
    gc.collect()
    gc.freeze()
    # p50 / p99: one micro-batch at a time, then the same from pinned host memory (run after the throughput region:
    # run before it they left the pipelined steps ~7 % slower for hundreds of steps, profiles/r05/warm_blocks)
    # the latency loops' wait for a batch's results: a spin on an event query (what a latency-bound consumer does);
    # hipStreamSynchronize blocks on an interrupt after a short active wait, and its wake-up is at the mercy of the
    # host scheduler (FD_LAT_WAIT=sync for it)
    spin = os.environ.get("FD_LAT_WAIT", "spin") != "sync"
    lat_ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for ev in lat_ev:  # created at their first record, before the loops
        ev.record(stream)
    torch.cuda.synchronize()

    spin_stat = [0.0, 0.0]  # the last wait's longest hipEventQuery call, and its longest gap between two calls (s)

    def wait_done():
        if spin:
            lat_ev[2].record(stream)
            q_max = g_max = 0.0
            t_prev = time.perf_counter()
            while True:
                t_a = time.perf_counter()
                done = lat_ev[2].query()
                t_b = time.perf_counter()
                q_max, g_max = max(q_max, t_b - t_a), max(g_max, t_a - t_prev)
                t_prev = t_b
                if done:
                    break
            spin_stat[0], spin_stat[1] = q_max, g_max
        else:
            stream.synchronize()

    def latency_loops():
        lat, split = [], []
        native = hasattr(eng, "counter")
        for i in range(args.latency_iters):
            n0 = eng.counter("pipelined_host_ns") if native else 0
            lat_ev[0].record(stream)
            a = time.perf_counter()
            if hasattr(wl, "step_to_host"):
                wl.step_to_host(i, i)
            else:
                wl.step(i)
                wl.fetch(i)
            b = time.perf_counter()
            lat_ev[1].record(stream)
            wait_done()
            c = time.perf_counter()
            lat.append(c - a)
            n1 = eng.counter("pipelined_host_ns") if native else 0
            # per sample: total, host submit, of which inside the engine's native call, the wait, the GPU span
            # (stream events around the submission: from the stream reaching the step to its results copied)
            split.append((c - a, b - a, (n1 - n0) * 1e-9, c - b, lat_ev[0].elapsed_time(lat_ev[1]) * 1e-3,
                          spin_stat[0], spin_stat[1]))
        lat_ms = np.array(lat) * 1e3 if lat else np.zeros(1)
        latency_split.clear()
        if split:
            S = np.array(split) * 1e3
            worst = np.argsort(S[:, 0])[::-1][:5]
            latency_split.update({
                "wait": "spin on hipEventQuery" if spin else "hipStreamSynchronize",
                "p50_ms": {k: round(float(np.percentile(S[:, j], 50)), 4) for j, k in enumerate(LAT_SPLIT)},
                "p99_ms": {k: round(float(np.percentile(S[:, j], 99)), 4) for j, k in enumerate(LAT_SPLIT)},
                "max_ms": {k: round(float(S[:, j].max()), 4) for j, k in enumerate(LAT_SPLIT)},
                "worst": [[int(q)] + [round(float(x), 4) for x in S[q]] for q in worst],
                "columns": ["sample"] + list(LAT_SPLIT),
                "basis": "isolated loop, per sample: total = host submit + wait; native = host ns inside the engine's "
                         "pipelined call (counter pipelined_host_ns); gpu = stream events around the submission; "
                         "query_max / gap_max = the wait's longest single hipEventQuery call and its longest time "
                         "between two calls (the polling thread not running: host scheduling)"})
        p99 = float(np.percentile(lat_ms, 99))
        # the same with the input columns crossing PCIe from pinned host memory first (workloads that support it)
        lat_h2d = []
        if hasattr(wl, "step_h2d") and args.latency_iters > 0:
            for i in range(min(args.latency_iters, len(getattr(wl, "h2d_pool", [])) or args.latency_iters)):
                a = time.perf_counter()
                wl.step_h2d(i)  # H2D, the step, results in host memory
                wait_done()
                lat_h2d.append(time.perf_counter() - a)
        p99_h2d = float(np.percentile(np.array(lat_h2d) * 1e3, 99)) if lat_h2d else -1.0
        if dist:  # the node's p99: the worst rank's
            t = torch.tensor([p99, p99_h2d], dtype=torch.float64, device=dev if DIST_BACKEND == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            p99, p99_h2d = (float(v) for v in t.tolist())
        return lat, lat_ms, p99, lat_h2d, p99_h2d


    for i in range(args.warmup):
        wl.step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    _read_timing(eng, wl)
    sat0 = _saturated(eng, wl)
    host0 = _host_counters(eng)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    # the timed region: exactly --steps back-to-back steps, no instrumentation inside (kernel timing is off)
    t0 = time.perf_counter()
    for i in range(args.steps):
        wl.step(i)
    t_sub = time.perf_counter()  # host submission done (the GPU may still be working through the queue)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    host1 = _host_counters(eng)
    _dump_fprof(0)
    # diagnostics (FD_BENCH_BLOCKS=N): N more blocks of --steps steps after the timed region, each bracketed by a
    # synchronize, their ms per step in the line (is a short region's rate a first-block effect or its fill / drain?)
    blocks = []
    for _ in range(_diag_blocks()):
        torch.cuda.synchronize()
        a = time.perf_counter()
        for i in range(args.steps):
            wl.step(i)
        torch.cuda.synchronize()
        blocks.append(round((time.perf_counter() - a) / args.steps * 1e3, 5))
        _dump_fprof(len(blocks))
    # kernel durations: HIP events on the launch stream, on one launch in TIMING_EVERY of each kernel (an event
    # record costs stream time), over more of the same back-to-back steps AFTER the timed region, so the kernel
    # averages rest on >= 20 launches of each kernel and `value` carries no instrumentation
    for e in _engines(eng, wl):
        e.set_option("timing_every", TIMING_EVERY)
        e.set_timing(True)
    for i in range(args.timing_steps):
        wl.step(args.steps + i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    for e in _engines(eng, wl):
        e.set_timing(False)
    timing = _read_timing(eng, wl)
    elapsed = t1 - t0
    saturation = None
    if sat0 is not None:
        sat = _saturated(eng, wl) - sat0
        if dist:
            t = torch.tensor([sat], dtype=torch.int64, device=dev if DIST_BACKEND == "nccl" else "cpu")
            dist.all_reduce(t)
            sat = int(t.item())
        tot = world * args.steps * args.batch
        saturation = {"transactions": sat, "of": tot, "frac": round(sat / tot, 8), "ring_k": wl.K,
                      "basis": "timed steps' transactions whose 24 h window held all ring_k prior events of the card "
                               "(engine counter window_saturated; their 24 h count / amount may be truncated at K)"}
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if DIST_BACKEND == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # loaded latency: the stream at the throughput operating point with a consumer's backpressure — at most
    # --loaded-inflight micro-batches submitted and not yet back (the host waits for batch i-D's results before it
    # submits batch i), each step's results copied to pinned host memory behind it on the output stream. A batch's
    # latency = its host submit -> its results in host memory, from GPU event timestamps relative to an event
    # recorded on the idle stream when the loop's host clock starts (offset: that event's launch, a few us)
    loaded = None
    if args.loaded_iters > 0 and hasattr(wl, "fetch"):
        D = max(1, args.loaded_inflight)
        # the events exist before the loop (a HIP event is created at its first record: that allocation is the
        # runtime's, not the stream's, and would stall the host mid-stream)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.loaded_iters)]
        for ev in evs:
            ev.record(stream)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        h0 = time.perf_counter()
        sub, host = [], []
        stall_trace = os.environ.get("FD_STALL_TRACE")  # diagnostics: the host stack of a submission > N ms
        if stall_trace:
            import faulthandler
        for i in range(args.loaded_iters):
            if i >= D:  # backpressure: batch i-D's results are back (a spin, as the isolated loop's wait)
                if spin:
                    while not evs[i - D].query():
                        pass
                else:
                    evs[i - D].synchronize()
            sub.append(time.perf_counter() - h0)
            if stall_trace:
                faulthandler.dump_traceback_later(float(stall_trace) / 1e3, exit=False)
            if hasattr(wl, "step_to_host"):
                wl.step_to_host(i, i)
            else:
                wl.step(i)
                wl.fetch(i)
            evs[i].record(stream)
            if stall_trace:
                faulthandler.cancel_dump_traceback_later()
            host.append(time.perf_counter() - h0 - sub[-1])
        torch.cuda.synchronize()
        h1 = time.perf_counter()
        ll = np.array([e0.elapsed_time(ev) - s_ * 1e3 for ev, s_ in zip(evs, sub)])
        worst = np.argsort(ll)[::-1][:5]
        loaded = {"p50_ms": round(float(np.percentile(ll, 50)), 4), "p99_ms": round(float(np.percentile(ll, 99)), 4),
                  "max_ms": round(float(ll.max()), 4), "samples": len(ll), "inflight": D,
                  "worst": [[int(j), round(float(ll[j]), 4), round(float(sub[j] * 1e3), 4)] for j in worst],
                  "host_submit_ms_max": round(max(host) * 1e3, 4),
                  "host_submit_ms_p50": round(float(np.percentile(host, 50)) * 1e3, 4),
                  "throughput_txn_per_s": round(args.loaded_iters * args.batch * world / (h1 - h0), 1),
                  "basis": f"back-to-back steps with at most {D} micro-batches in flight (backpressure), each "
                           "step's fraud_prob / confidence / decision / risk written to host-mapped pinned memory by the "
                           "engine's output kernel (workloads without that: a D2H to pinned memory); latency = host "
                           "submit -> results in host memory (GPU event timestamps)"}
        if dist:
            t = torch.tensor([loaded["p99_ms"]], dtype=torch.float64, device=dev if DIST_BACKEND == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            loaded["p99_ms"] = float(t.item())

    latency_split = {}
    lat, lat_ms, p99, lat_h2d, p99_h2d = latency_loops()

    # the same kernels one micro-batch at a time, nothing beside them (in the pipelined stream the next batch's
    # feature kernels share the CUs with the forests): each kernel's unshared duration
    timing_alone = None
    if args.alone_iters > 0:
        for e in _engines(eng, wl):
            e.set_option("timing_every", 1)
            e.set_timing(True)
        for i in range(args.alone_iters):
            wl.step(i)
            torch.cuda.synchronize()
        for e in _engines(eng, wl):
            e.set_timing(False)
        timing_alone = _read_timing(eng, wl)

    value = world * args.steps * args.batch / elapsed
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = wl.cpu_baseline(args.cpu_seconds)

    if rank == 0:
        try:
            roof = wl.roofline(timing)
        except ZeroDivisionError:  # no kernel timing samples (--timing-steps 0)
            roof = None
        if isinstance(roof, dict) and roof.get("unit") == "node-steps/s":  # the dominant kernel per pipeline step
            tp = roof["node_steps_per_launch"] / (elapsed / args.steps)
            roof["throughput_basis"] = {"achieved": round(tp, 1), "frac": round(tp / roof["peak"], 6),
                                        "basis": "node-steps per launch / ms_per_step (one launch per step; launches "
                                                 "of consecutive steps may overlap on the two pipeline streams)"}
        if timing_alone and isinstance(roof, dict):
            try:
                ra = wl.roofline(timing_alone)
                roof["alone"] = {"kernel_avg_us": ra.get("kernel_avg_us"), "achieved": ra.get("achieved"),
                                 "frac": ra.get("frac"), "basis": f"{args.alone_iters} steps one at a time, "
                                 "every launch timed (no other kernel on the CUs)"}
            except Exception as e:  # a workload whose roofline needs the timed region's kernels
                log(f"[rank {rank}] roofline.alone unavailable: {e!r}")
        line = {
            "metric": "scored transactions/sec (whole node)",
            "value": round(value, 1),
            "unit": "txn/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "host_submit_ms_per_step": round((t_sub - t0) / args.steps * 1e3, 5),
            "host_submit_breakdown": _host_breakdown(host0, host1, t_sub - t0, args.steps),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": wl.dtype,
            "data": "synthetic (seeded simulator-distribution stream / scoring vectors; random-init models in the "
                    "reference's file formats)",
            "config": dict(wl.config(world), **({"dist_backend": "gloo rehearsal (ranks share GPUs; not the metric)"}
                                               if world > 1 and DIST_BACKEND != "nccl" else {})),
            "p50_batch_latency_ms": round(float(np.percentile(lat_ms, 50)), 4),
            "p99_batch_latency_ms": round(p99, 4),
            "max_batch_latency_ms": round(float(lat_ms.max()), 4),
            "p99_batch_latency_with_h2d_ms": round(p99_h2d, 4) if lat_h2d else None,
            "p50_batch_latency_with_h2d_ms": (round(float(np.percentile(np.array(lat_h2d) * 1e3, 50)), 4)
                                              if lat_h2d else None),
            "latency_h2d_samples": len(lat_h2d),
            "latency_samples": len(lat),
            "latency_basis": "p50/p99/max: one micro-batch at a time (submit -> scores in host memory, then the next); "
                             "loaded_latency: at the throughput operating point",
            "latency_split": latency_split or None,
            "loaded_latency": loaded,
            "roofline": roof,
            "kernel_avg_us": wl.kernels(timing),
            "kernel_avg_us_alone": wl.kernels(timing_alone) if timing_alone else None,
            "kernel_timing": f"HIP events on the launch stream, 1 launch in {TIMING_EVERY} of each kernel, over "
                             f"{args.timing_steps} back-to-back steps after the timed region (none inside it)",
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
            "window_saturation": saturation,
            "step_launch": "direct kernel launches",
            "engine_options": dict(kv.split("=") for kv in args.engine_option) or None,
        }
        if blocks:
            line["diag_blocks_ms_per_step"] = blocks
        if hasattr(wl, "counter_groups"):
            line["counters"] = pmc_counters(wl.name, args.batch, wl.counter_groups(roof), line["kernel_avg_us"])
        if wl.name in ("config3", "config4", "config5"):
            per_gpu = value / world
            line["pipeline_hbm"] = {"bytes_per_txn": FUSED_BYTES_PER_TXN,
                                    "achieved_GBs_per_gpu": round(per_gpu * FUSED_BYTES_PER_TXN / 1e9, 3),
                                    "peak_GBs": HBM_PEAK_GBS,
                                    "frac": round(per_gpu * FUSED_BYTES_PER_TXN / 1e9 / HBM_PEAK_GBS, 6),
                                    "basis": "SURVEY §8(d) fused-pipeline algorithmic bytes x txn/s per GPU"}
        secondary = _secondary_list(args, world, wl.name)
        if secondary:
            # the line's own measurements are complete: free this process's GPU state (the config-4 card table is
            # ~160 GB of the card's 288) before the children allocate theirs
            wl = None
            eng.close()
            gc.unfreeze()
            gc.collect()
            torch.cuda.empty_cache()
            line["secondary_workloads"] = _run_secondaries(secondary)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


# BASELINE configs[4], [1], [2], and config 2's raw-JSON form (the Kafka codec ahead of the pipeline)
SECONDARY_DEFAULT = ("config5", "config2", "config3", "config3j")


def _secondary_list(args, world, name):
    if world != 1 or name != "config4" or os.environ.get("FD_BENCH_SECONDARY", "1") == "0":
        return []
    if args.secondary is None:
        return list(SECONDARY_DEFAULT)
    if args.secondary.strip().lower() in ("", "none"):
        return []
    return [w.strip() for w in args.secondary.split(",") if w.strip() in WORKLOADS and w.strip() != "config4"]


def _run_secondaries(names):
    """Each secondary workload as `python bench.py --workload W --steps 200 --warmup 20 --no-cpu-baseline` in a child
    process (started after this process freed its GPU state; never an exec), its JSON line parsed and summarised:
    the other BASELINE configurations measured by the same command the driver runs."""
    out = {}
    for w in names:
        cmd = [sys.executable, str(Path(__file__).resolve()), "--workload", w, "--steps", "200", "--warmup", "20",
               "--no-cpu-baseline", "--secondary", "none"]
        a = time.perf_counter()
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
            rows = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not rows:
                out[w] = {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-600:]}
                continue
            d = json.loads(rows[-1])
        except Exception as e:  # a failed secondary is reported, never fatal to the line
            out[w] = {"error": repr(e)}
            continue
        roof = d.get("roofline") or {}
        par = d.get("parity_vs_oracle") or {}
        out[w] = {
            "workload": (d.get("config") or {}).get("workload"),
            "metric": d.get("metric"), "value": d.get("value"), "unit": d.get("unit"),
            "ms_per_step": d.get("ms_per_step"), "steps": d.get("steps"), "warmup": d.get("warmup"),
            "p50_batch_latency_ms": d.get("p50_batch_latency_ms"), "p99_batch_latency_ms": d.get("p99_batch_latency_ms"),
            "p99_batch_latency_with_h2d_ms": d.get("p99_batch_latency_with_h2d_ms"),
            "dtype": d.get("dtype"),
            "roofline": {k: roof.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "kernel", "kernel_avg_us")
                         if k in roof} or None,
            "kernel_avg_us": d.get("kernel_avg_us"),
            "parity_vs_oracle": {k: v for k, v in par.items() if not isinstance(v, (list, dict))} or None,
            "parity_legs": {k: {q: u for q, u in v.items() if not isinstance(u, (list, dict))}
                            for k, v in par.items() if isinstance(v, dict)} or None,
            "wall_s": round(time.perf_counter() - a, 1),
        }
    return out


if __name__ == "__main__":
    main()
