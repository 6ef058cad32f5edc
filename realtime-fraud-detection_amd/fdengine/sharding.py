"""Card-hash sharded scoring across the GPUs of one node (BASELINE config 4).

The reference keys all per-card work by user id — Kafka partition key and Flink keyBy
(services/flink-jobs/.../FraudDetectionJob.java, WindowProcessor.java:45-64) — with the velocity state
in one Redis (RedisService.java:178-207). Here GPU r of G owns the cards with
shard_of(card_key, G) == r (fdengine.shard_of / fd_shard_of_host) and keeps their state resident in its
HBM. Models (≈2 MB) and the merchant table are replicated.

One micro-batch step, per rank (one process per GPU, torch.distributed: RCCL over xGMI on the GPU,
gloo in the CPU tests), in the serial form (`step(..., windows / sink)`, or a backend without the streaming hooks):
  1. fd_route_partition_device: group the ingested batch by owner (stable), 48-B records + counts;
  2. all_to_all of the per-owner counts (G int64), then both count vectors to the host (one sync:
     RCCL all-to-all needs host split sizes);
  3. all_to_all of the records (uneven splits);
  4. fd_score_records_device: features (this GPU's card state) -> XGBoost + IsolationForest -> blend;
  5. all_to_all of the 24-B result records back (splits reversed);
  6. fd_route_scatter_results_device: results in the ingest batch's original order.
Records from one source keep their arrival order and all_to_all concatenates sources in rank order,
so every card sees its transactions in (step, ingest rank, ingest index) order.

Streaming form (the scoring step of a backend with `start_partition`, i.e. EngineShardBackend): the same
exchanges, but nothing drains the device queue.
  * the partition and the count all-to-all run on a forward stream beside the scoring; the counts land in
    pinned host memory behind an event. Given `prefetch` (the next micro-batch), step s launches batch s+1's
    partition and count exchange, so step s+1 finds its split sizes already on the host (the one host wait is
    that event, which completed while the GPUs were still scoring);
  * the records all-to-all runs on the forward stream; the owner scores through fd_score_records_pipelined
    (its features wait for an event recorded after the records landed and overlap the previous batch's
    forests); the result all-to-all goes on a second communicator (`group_back`), queued behind the scoring
    on the engine stream, so a batch's returning results never hold up the next batch's records;
  * every rank makes the same calls in the same order (prefetch in the same steps on all ranks). With one shard (world 1)
the step is the fused hot path on the ingest batch itself (fd_score_batch_device): nothing to route.

The exchange logic is backend-agnostic: `EngineShardBackend` drives libfdengine.so (the product path);
the CPU tests plug an oracle-backed backend into the same `ShardedScorer` to check the protocol.

Keyed aggregates across shards (step(..., windows=True, sink=True)): the payment method and isFraud ride in
the transaction records; after scoring, each owner runs the Flink window aggregates (WindowProcessor, a5) and
the sink aggregates (RedisTransactionSink, f3) on the transactions it owns, with the ML fraud score as
Transaction.fraudScore. Cards are owned, so user windows are complete on their owner. Merchant-keyed state
spans shards: (1) ONE watermark — an all-reduce MAX of the ingest batches' largest event time, given to every
shard before its window step (fd_windows_observe), so all shards fire the same windows at the same step;
(2) each shard's fired merchant windows are exact-moment partials (counts, integer cents, cents^2, the
payment-method set; distinct users add because a card lives on one shard), all-gathered and merged with the
library's own finalisation (fd_merchant_windows_merge): bit-identical to an unsharded run. The sink's
hourly / daily / merchant-hour aggregates stay as per-shard integer partials and are summed at query time
(an all-reduce of counts and cents, `sink_query`). Nothing on the scoring path reads these aggregates
(merchant features come from the replicated merchant table), so no "as of batch start" snapshot is needed.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import _native as N
from .engine import FraudEngine, shard_of  # noqa: F401  (shard_of re-exported for callers)

REC = N.FD_ROUTE_RECORD_BYTES
RES = N.FD_RESULT_RECORD_BYTES
INT64_MIN = -(1 << 63)


class EngineShardBackend:
    """Steps 1, 4 and 6 on one GPU through the C-ABI (device tensors in, device tensors out)."""

    def __init__(self, eng: FraudEngine, params: N.fd_blend_params, slots: Sequence[int],
                 present: Optional[Sequence[int]] = None, pipelined: bool = False):
        """pipelined: one shard scores through fd_score_batch_pipelined (batch i+1's features overlap batch i's
        forests). The caller then guarantees each step's input tensors are complete when step() is called
        (resident in HBM, or pass `input_ready` to score_batch) and unchanged until its outputs are."""
        import torch
        self.torch = torch
        self.eng, self.params, self.slots, self.present = eng, params, list(slots), present
        self.pipelined = pipelined
        self._scorer = None
        self.device = torch.device("cuda", eng.device)
        # The engine's kernels and the collectives must be ordered on ONE stream: bind the engine to the
        # stream torch (and so RCCL's all_to_all and .cpu()) uses on this device.
        eng.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    # ---- the sharded step as one engine call over its own RCCL communicators (fd_comm_init / fd_sharded_step)
    native = False

    def init_comm(self, rank: int, world: int, group=None, rccl_path: Optional[str] = None, ids=None) -> None:
        """Collective over `group`: rank 0 makes the two RCCL unique ids, every rank joins the engine's communicators
        (forward: counts + records; back: results). RCCL is the process's own (torch's librccl.so) unless
        `rccl_path` names another library with the same API; `ids` (the two unique ids, made by the caller) skips
        the broadcast over `group` (ranks that are threads of one process: the loopback tests)."""
        path = rccl_path or rccl_library_path()
        if ids is None:
            import torch.distributed as dist
            box = [None]
            if rank == 0:
                from .engine import FraudEngine
                box = [(FraudEngine.comm_unique_id(path), FraudEngine.comm_unique_id(path))]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(box, src=src, group=group)
            ids = box[0]
        self.eng.comm_init(path, rank, world, ids[0], ids[1])
        self._sharded = self.eng.sharded_scorer(self.params, self.slots, self.present)
        self._prefetched = None  # (id, the prefetch tuple): kept alive until the call that scores or drops it
        self._next_id = 0
        self.native = True

    def sharded_step(self, txns: dict, n: int, input_ready=None, prefetch=None, out=None):
        """fd_sharded_step: outputs (fresh tensors on torch's current stream, written on the engine stream, or the
        caller's `out`, see _outputs) and the split sizes; prefetch = (next txns, next n[, next input_ready]).
        The prefetched batch is named to the engine by an id: this call passes the pending id only when `txns` is
        the very mapping (or the very tensors) given as the last prefetch, never by comparing addresses; the
        prefetch's tensors are referenced here until the call that consumes or drops them has returned."""
        res, (fp, conf, dec, risk) = self._outputs(n, out)
        pend = self._prefetched
        bid = pend[0] if pend is not None and int(pend[1][1]) == int(n) and _same_batch(pend[1][0], txns) else 0
        nxt, nn, nready, nid = None, 0, 0, 0
        if prefetch is not None:
            nxt = {f: prefetch[0][f].data_ptr() for f in N.TXN_FIELDS}
            nn = int(prefetch[1])
            nready = prefetch[2].cuda_event if len(prefetch) > 2 and prefetch[2] is not None else 0
            self._next_id += 1
            nid = self._next_id
        self._sharded({f: txns[f].data_ptr() for f in N.TXN_FIELDS}, n, fp, conf, dec, risk,
                      input_ready.cuda_event if input_ready is not None else 0, nxt, nn, nready,
                      batch_id=bid, next_id=nid)
        self._prefetched = (nid, prefetch) if prefetch is not None else None
        return res, self._sharded.split_sizes

    def close_comm(self) -> None:
        if self.native:
            self.eng.comm_destroy()
            self.native = False

    # ---- streaming sharded step (ShardedScorer._step_streaming)
    def _fwd(self):
        if getattr(self, "_x_fwd", None) is None:
            self._x_fwd = self.torch.cuda.Stream(self.device)
        return self._x_fwd

    def fwd_ctx(self):
        """the forward stream: partitions, count and record exchanges (torch's NCCL calls follow the current stream)"""
        return self.torch.cuda.stream(self._fwd())

    def start_partition(self, txns: dict, n: int, G: int, input_ready=None):
        """fd_route_partition_stream on the forward stream (call inside fwd_ctx); the input tensors are marked in
        use there, so freeing them on another stream cannot recycle them under the partition"""
        t, x = self.torch, self._fwd()
        if input_ready is not None:
            x.wait_event(input_ready)
        for v in txns.values():
            v.record_stream(x)
        rec = t.empty((n, REC), dtype=t.uint8, device=self.device)
        counts = t.empty(G, dtype=t.int64, device=self.device)
        self.eng.route_partition_stream({f: txns[f].data_ptr() for f in N.TXN_FIELDS}, None, n, G,
                                        rec.data_ptr() if n else 0, counts.data_ptr(), x.cuda_stream)
        return rec, counts

    def counts_to_host(self, counts, recv):
        """both count vectors to pinned host memory behind an event on the forward stream (inside fwd_ctx)"""
        t = self.torch
        G = counts.numel()
        h = t.empty(2 * G, dtype=t.int64, pin_memory=True)
        h[:G].copy_(counts, non_blocking=True)
        h[G:].copy_(recv, non_blocking=True)
        ev = t.cuda.Event()
        ev.record(self._fwd())
        return _HostCounts(h, ev, G)

    def forward_ready(self):
        """an event on the forward stream after the records landed (inside fwd_ctx)"""
        ev = self.torch.cuda.Event()
        ev.record(self._fwd())
        return ev

    def score_records_async(self, inbox, m: int, ready):
        """fd_score_records_pipelined: result records written on the engine stream (torch's current stream)"""
        t = self.torch
        res = t.empty((m, RES), dtype=t.uint8, device=self.device)
        if m:
            inbox.record_stream(t.cuda.current_stream(self.device))  # reused only after the engine stream passed
            self.eng.score_records_pipelined(self.params, self.slots, inbox.data_ptr(), m, res.data_ptr(),
                                             ready.cuda_event, self.present)
        return res

    def partition(self, txns: dict, n: int, G: int, extras: Optional[dict] = None):
        t = self.torch
        rec = t.empty((n, REC), dtype=t.uint8, device=self.device)
        counts = t.empty(G, dtype=t.int64, device=self.device)
        ptrs = {f: txns[f].data_ptr() for f in N.TXN_FIELDS}
        if extras:
            self.eng.route_partition_ex_device(ptrs, {k: v.data_ptr() for k, v in extras.items()}, n, G,
                                               rec.data_ptr() if n else 0, counts.data_ptr())
        else:
            self.eng.route_partition_device(ptrs, n, G, rec.data_ptr() if n else 0, counts.data_ptr())
        return rec, counts

    # ---- owner-side keyed aggregates (windows a5, sink f3)
    def unpack(self, rec, res, m: int) -> dict:
        """received records (+ result records) -> device columns for the window / sink kernels"""
        t = self.torch
        cols = {"card_key": t.empty(m, dtype=t.uint64, device=self.device),
                "ts_ms": t.empty(m, dtype=t.int64, device=self.device),
                "amount_cents": t.empty(m, dtype=t.int64, device=self.device),
                "merchant": t.empty(m, dtype=t.int32, device=self.device),
                "payment_method": t.empty(m, dtype=t.uint8, device=self.device),
                "is_fraud": t.empty(m, dtype=t.uint8, device=self.device),
                "fraud_score": t.empty(m, dtype=t.float64, device=self.device)}
        if m:
            self.eng.route_unpack_device(rec.data_ptr(), res.data_ptr() if res is not None else 0, m,
                                         {f: cols[f].data_ptr() for f in ("card_key", "ts_ms", "amount_cents",
                                                                          "merchant")},
                                         cols["payment_method"].data_ptr(), cols["is_fraud"].data_ptr(),
                                         cols["fraud_score"].data_ptr())
        return cols

    @staticmethod
    def _ins(cols):
        return {k: cols[k].data_ptr() for k in ("payment_method", "is_fraud", "fraud_score") if k in cols}

    def windows_observe(self, max_event_ts: int) -> None:
        self.eng.windows_observe(max_event_ts)

    def windows_step(self, cols: dict, m: int, flush: bool):
        return self.eng.windows_step_device({f: cols[f].data_ptr() for f in cols if f in N.TXN_FIELDS}, m,
                                            in_ptrs=self._ins(cols), flush=flush)

    def sink_update(self, cols: dict, m: int) -> None:
        if m:
            self.eng.sink_update_device({f: cols[f].data_ptr() for f in cols if f in N.TXN_FIELDS}, m,
                                        in_ptrs=self._ins(cols))

    def sink_query(self, kind: int, buckets, merchants=None):
        return self.eng.sink_query(kind, buckets, merchants)

    def score_records(self, rec, m: int):
        t = self.torch
        res = t.empty((m, RES), dtype=t.uint8, device=self.device)
        if m:
            self.eng.score_records_device(self.params, self.slots, rec.data_ptr(), m, res.data_ptr(), self.present)
        return res

    def _outputs(self, n: int, out):
        """caller-owned outputs (tensors or raw addresses; device memory or host-mapped pinned memory, which the
        engine's output kernel then writes over PCIe: no separate D2H) or fresh device tensors"""
        if out is not None:
            return tuple(out), [o if isinstance(o, int) else o.data_ptr() for o in out]
        t = self.torch
        o = (t.empty(n, dtype=t.float64, device=self.device), t.empty(n, dtype=t.float64, device=self.device),
             t.empty(n, dtype=t.uint8, device=self.device), t.empty(n, dtype=t.uint8, device=self.device))
        return o, [x.data_ptr() for x in o]

    def score_batch(self, txns: dict, n: int, input_ready=None, vectors=None, model_probs=None, out=None):
        """One shard: the whole hot path on the ingest GPU in arrival order (nothing to route).
        input_ready: optional torch.cuda.Event recorded once the input tensors were complete (pipelined).
        vectors / model_probs: optional device tensors (n x 64 f32 / n_models x n f64) that also receive the
        batch's scoring vectors / per-model probabilities.
        out: optional (fraud_prob f64, confidence f64, decision u8, risk u8) caller-owned buffers (see _outputs)."""
        res, (fp, conf, dec, risk) = self._outputs(n, out)
        if n:
            ptrs = {f: txns[f].data_ptr() for f in N.TXN_FIELDS}
            if self.pipelined:
                if self._scorer is None:
                    self._scorer = self.eng.pipelined_scorer(self.params, self.slots, self.present)
                self._scorer(ptrs, n, fp, conf, dec, risk, input_ready.cuda_event if input_ready is not None else 0,
                             vec_ptr=vectors.data_ptr() if vectors is not None else 0,
                             model_probs_ptr=model_probs.data_ptr() if model_probs is not None else 0)
            else:
                self.eng.score_batch_device(self.params, self.slots, ptrs, n, fp, conf, dec, risk,
                                            present=self.present,
                                            vec_ptr=vectors.data_ptr() if vectors is not None else 0,
                                            model_probs_ptr=model_probs.data_ptr() if model_probs is not None
                                            else 0)
        return res

    def snapshot(self, path: str, rank: int, world: int) -> int:
        return self.eng.state_snapshot(path, rank, world)

    def restore(self, path: str, rank: int, world: int) -> int:
        return self.eng.state_restore(path, rank, world, skip_windows=True, skip_sink=True)

    def scatter_results(self, res, n: int, sentinel: bool = False):
        """sentinel: pre-fill the outputs (NaN probability, decision/risk 255) so a row no result record
        reached (a mismatched exchange) cannot pass for a score."""
        t = self.torch
        if sentinel:
            fp = t.full((n,), float("nan"), dtype=t.float64, device=self.device)
            dec = t.full((n,), 255, dtype=t.uint8, device=self.device)
            risk = t.full((n,), 255, dtype=t.uint8, device=self.device)
        else:
            fp = t.empty(n, dtype=t.float64, device=self.device)
            dec = t.empty(n, dtype=t.uint8, device=self.device)
            risk = t.empty(n, dtype=t.uint8, device=self.device)
        conf = t.empty(n, dtype=t.float64, device=self.device)
        if n:
            self.eng.route_scatter_results_device(res.data_ptr(), n, fp.data_ptr(), conf.data_ptr(),
                                                  dec.data_ptr(), risk.data_ptr())
        return fp, conf, dec, risk


def _same_batch(a, b) -> bool:
    """the same input batch object: the same mapping, or the same tensor objects in every field"""
    return a is b or all(a[f] is b[f] for f in N.TXN_FIELDS)


class _HostCounts:
    """split sizes on their way to the host (pinned buffer + event)"""

    def __init__(self, h, ev, G):
        self.h, self.ev, self.G = h, ev, G

    def wait(self):
        if self.ev is not None:
            self.ev.synchronize()
        v = [int(c) for c in self.h.tolist()]
        return v[:self.G], v[self.G:]


class ShardedScorer:
    """One rank's side of the sharded hot path. `world == 1` runs the same kernels with no collective.
    streaming (default True): use the backend's streaming hooks when it has them (module docstring); the result
    all-to-all then runs on a second process group over the same ranks, created here (collectively)."""

    def __init__(self, backend, rank: int, world: int, group=None, streaming: bool = True, force_route: bool = False,
                 native: Optional[bool] = None, comm=None):
        """force_route: route even with one shard (partition, exchanges over a 1-rank process group, scatter) — the
        N > 1 step's own work measured / tested on one GPU (tools/route_overhead.py).
        native: the scoring step as one engine call over the engine's own RCCL communicators (fd_sharded_step);
        default: when the process group is RCCL ("nccl": one GPU per rank) and the backend supports it; else the
        streaming step in Python over torch.distributed (gloo groups: ranks sharing a GPU, CPU tests).
        comm: (library path, (id_fwd, id_back)) for the native step's communicators instead of torch's RCCL and a
        broadcast over `group` — ranks that are threads of one process (the loopback tests; no process group)."""
        self.be, self.rank, self.world, self.group = backend, int(rank), int(world), group
        self.last_counts = None  # (send, recv) split sizes of the last step, for diagnostics
        self.last_windows = None  # (user windows, merged merchant windows) fired by the last windows step
        self.route = self.world > 1 or bool(force_route)
        self.streaming = bool(streaming) and self.route and hasattr(backend, "start_partition")
        self.group_back = None
        self._pending = None
        self.native = False
        if self.streaming:
            import torch.distributed as dist
            if native is None:
                native = comm is not None or (hasattr(backend, "init_comm") and dist.get_backend(group) == "nccl")
            if native:
                if comm is not None:
                    backend.init_comm(self.rank, self.world, group, rccl_path=comm[0], ids=comm[1])
                else:
                    backend.init_comm(self.rank, self.world, group)
                self.native = True
            else:
                ranks = list(range(self.world)) if group is None else dist.get_process_group_ranks(group)
                self.group_back = dist.new_group(ranks=ranks)

    def _staged(self) -> bool:
        """gloo moves host memory only: device tensors are staged through the host (several ranks sharing one
        GPU in tests; RCCL — the product path — exchanges device memory directly)."""
        import torch.distributed as dist
        return dist.get_backend(self.group) == "gloo"

    def _a2a(self, out, inp, out_splits=None, in_splits=None, group="fwd"):
        import torch.distributed as dist
        g = self.group_back if group == "back" else self.group
        if self._staged() and (out.is_cuda or inp.is_cuda):
            o = out.cpu()
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=g)
            out.copy_(o)
            return
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=g)

    def _all_gather_records(self, arr: np.ndarray) -> list:
        """every rank's structured-array records (same dtype on all ranks), gathered as fixed-size tensors: the
        counts first (one int64 per rank), then each rank's records as bytes padded to the largest count — no
        pickled objects on the exchange"""
        import torch
        import torch.distributed as dist
        dev = "cpu" if self._staged() else self.be.device
        cnt = torch.tensor([len(arr)], dtype=torch.int64, device=dev)
        counts = [torch.empty_like(cnt) for _ in range(self.world)]
        dist.all_gather(counts, cnt, group=self.group)
        counts = [int(c.item()) for c in counts]
        rec = arr.dtype.itemsize
        top = max(1, max(counts))
        buf = np.zeros(top * rec, np.uint8)
        buf[:len(arr) * rec] = np.frombuffer(np.ascontiguousarray(arr).tobytes(), np.uint8)
        mine = torch.from_numpy(buf).to(dev)
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine, group=self.group)
        return [np.frombuffer(p.cpu().numpy().tobytes()[:c * rec], arr.dtype).copy() for p, c in zip(parts, counts)]

    def _allreduce_max(self, t):
        import torch.distributed as dist
        g = t.cpu() if self._staged() else t.clone()
        dist.all_reduce(g, op=dist.ReduceOp.MAX, group=self.group)
        return int(g.cpu()[0])

    def step(self, txns: dict, n: int, extras: Optional[dict] = None, windows: bool = False, sink: bool = False,
             flush: bool = False, input_ready=None, vectors=None, model_probs=None, prefetch=None, out=None):
        """txns: field -> tensor (n rows) on the backend's device, in arrival order.
        input_ready: optional torch.cuda.Event recorded once `txns` were complete (a pipelined backend's features
        wait for it instead of assuming resident inputs).
        -> (fraud_prob f64, confidence f64, decision u8, risk u8) tensors in the same order.
        extras: {"payment_method": u8, "is_fraud": u8} tensors (n rows) for the keyed aggregates.
        windows / sink: after scoring, run the Flink window aggregates / the sink aggregates on the owned
        transactions (module docstring); the fired windows are left in self.last_windows =
        (this shard's user windows, the node's merged merchant windows); flush: end of input.
        vectors / model_probs (world 1, backends with score_batch): optional device tensors that also receive the
        batch's scoring vectors (n x 64) / per-model probabilities (n_models x n).
        prefetch (world > 1, streaming): (next txns, next n[, next input_ready]) — the next micro-batch, whose
        partition and count exchange this step launches ahead; every rank must pass it in the same steps.
        out (world 1 with score_batch, or the native sharded step): caller-owned output buffers — tensors or raw
        addresses, device memory or host-mapped pinned memory the engine's output kernel writes over PCIe — that
        receive the results instead of fresh device tensors (returned as given)."""
        import torch
        G = self.world
        aux = windows or sink
        if not self.route:  # one shard owns every card: no partition, no exchange
            self.last_counts = ([n], [n])
            if hasattr(self.be, "score_batch"):
                kw = {k: v for k, v in (("input_ready", input_ready), ("vectors", vectors),
                                        ("model_probs", model_probs), ("out", out)) if v is not None}
                out = self.be.score_batch(txns, n, **kw)
                if aux:
                    cols = {f: txns[f] for f in ("card_key", "ts_ms", "amount_cents", "merchant")}
                    cols.update(extras or {})
                    cols["fraud_score"] = out[0]
                    self._aggregates(cols, n, None, windows, sink, flush)
                return out
            rec, _ = self.be.partition(txns, n, 1, extras) if aux else self.be.partition(txns, n, 1)
            res = self.be.score_records(rec, n)
            if aux:
                self._aggregates(self.be.unpack(rec, res, n), n, None, windows, sink, flush)
            return self.be.scatter_results(res, n)
        if self.native and not aux:
            res, split = self.be.sharded_step(txns, n, input_ready, prefetch, out)
            self.last_counts = (split[:G].tolist(), split[G:2 * G].tolist())
            return res
        if out is not None:
            raise ValueError("out= needs one shard (score_batch) or the native sharded step")
        if self.streaming and not aux:
            return self._step_streaming(txns, n, input_ready, prefetch)
        rec, counts = self.be.partition(txns, n, G, extras) if aux else self.be.partition(txns, n, G)
        recv_counts = torch.empty_like(counts)
        self._a2a(recv_counts, counts)
        both = torch.cat([counts, recv_counts]).cpu().tolist()
        send, recv = [int(c) for c in both[:G]], [int(c) for c in both[G:]]
        self.last_counts = (send, recv)
        m = sum(recv)
        inbox = torch.empty((m, REC), dtype=torch.uint8, device=rec.device)
        self._a2a(inbox, rec, recv, send)
        res = self.be.score_records(inbox, m)
        back = torch.empty((n, RES), dtype=torch.uint8, device=rec.device)
        self._a2a(back, res, send, recv)
        if aux:
            tmax = txns["ts_ms"].max().reshape(1) if n else torch.full((1,), INT64_MIN, dtype=torch.int64,
                                                                        device=rec.device)
            self._aggregates(self.be.unpack(inbox, res, m), m, tmax, windows, sink, flush)
        return self.be.scatter_results(back, n, sentinel=True)

    # ---------------------------------------------------------------- streaming exchange (module docstring)
    def _launch_counts(self, txns, n, input_ready):
        import torch
        be = self.be
        with be.fwd_ctx():
            rec, counts = be.start_partition(txns, n, self.world, input_ready)
            recv = torch.empty_like(counts)
            self._a2a(recv, counts)
            host = be.counts_to_host(counts, recv)
        # the batch itself (referenced: its tensors cannot be recycled while the prefetch is pending), matched by
        # identity — never by address, which torch's allocator reuses
        return {"txns": txns, "n": int(n), "rec": rec, "host": host}

    def _step_streaming(self, txns, n, input_ready, prefetch):
        import torch
        be = self.be
        p = self._pending
        self._pending = None
        if p is None or p["n"] != int(n) or not _same_batch(p["txns"], txns):
            # no prefetch, or another batch came instead of the prefetched one: its partition and count exchange
            # (issued on every rank alike) are dropped, this batch's are launched now
            p = self._launch_counts(txns, n, input_ready)
        send, recv = p["host"].wait()  # the step's one host wait: split sizes exchanged ahead
        self.last_counts = (send, recv)
        m = sum(recv)
        if prefetch is not None:  # the next batch's partition + counts first (as fd_sharded_step: DESIGN §7)
            nt, nn = prefetch[0], prefetch[1]
            self._pending = self._launch_counts(nt, nn, prefetch[2] if len(prefetch) > 2 else None)
        with be.fwd_ctx():
            inbox = torch.empty((m, REC), dtype=torch.uint8, device=p["rec"].device)
            self._a2a(inbox, p["rec"], recv, send)
            ready = be.forward_ready()
        res = be.score_records_async(inbox, m, ready)
        back = torch.empty((n, RES), dtype=torch.uint8, device=res.device)
        self._a2a(back, res, send, recv, group="back")
        return be.scatter_results(back, n, sentinel=True)

    def _aggregates(self, cols: dict, m: int, tmax, windows: bool, sink: bool, flush: bool):
        if windows:
            if tmax is not None:  # one watermark for the node: the largest event time of all ingest batches
                gmax = self._allreduce_max(tmax)
                if gmax != INT64_MIN:
                    self.be.windows_observe(gmax)
            uw, mw = self.be.windows_step(cols, m, flush)
            parts = self._all_gather_records(mw) if self.world > 1 else [mw]
            from .engine import merge_merchant_windows
            self.last_windows = (uw, merge_merchant_windows(parts))
        if sink:
            self.be.sink_update(cols, m)

    def sink_query(self, kind: int, buckets, merchants=None) -> np.ndarray:
        """RedisService.getAggregation over the whole node: this shard's integer partials summed over all
        shards (counts, distinct users — a card lives on one shard — and exact cents), then the reference's
        derived fields with the device's own operations (rate = fraud / count, avg = (cents / 100) / count)."""
        import torch
        import torch.distributed as dist
        a = self.be.sink_query(kind, buckets, merchants)
        if self.world == 1:
            return a
        cents = np.rint(a["total_amount"] * 100.0).astype(np.int64)  # exact: |cents| < 2^50
        ints = np.stack([a["total_count"], a["fraud_count"], a["high_risk_count"], a["unique_user_count"], cents,
                         a["found"].astype(np.int64)])
        t = torch.from_numpy(np.ascontiguousarray(ints))
        if not self._staged():
            t = t.to(self.be.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        tot = t.cpu().numpy()
        out = np.zeros(len(a), N.AGGREGATE_DTYPE)
        for i in range(len(a)):
            cnt, fr, hi, uu, c, found = (int(v) for v in tot[:, i])
            if found:
                total = c / 100
                out[i] = (cnt, fr, hi, uu, total, fr / cnt, total / cnt, 1, 0)
        return out

    # ------------------------------------------------------------------ checkpoint / rescale
    # Counterpart of Flink's externalized keyed-state checkpoints (fl/FraudDetectionJob.java:112-136):
    # every rank writes its key-addressed image, rank 0 writes the manifest after a barrier (the image set
    # is complete when the manifest exists). Restoring on any world size re-shards: each new rank reads every
    # old image and keeps the cards it owns.
    def checkpoint(self, directory: str, step: int) -> str:
        import json
        import os
        import torch.distributed as dist
        os.makedirs(directory, exist_ok=True)
        name = image_name(step, self.rank, self.world)
        nbytes = self.be.snapshot(os.path.join(directory, name), self.rank, self.world)
        sizes = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(sizes, nbytes, group=self.group)
        else:
            sizes = [nbytes]
        man = os.path.join(directory, f"checkpoint-{step:08d}.json")
        if self.rank == 0:
            doc = {"format": "fdsnap/1", "step": int(step), "world": self.world,
                   "images": [image_name(step, r, self.world) for r in range(self.world)], "bytes": sizes}
            tmp = man + ".tmp"
            with open(tmp, "w") as f:
                json.dump(doc, f)
            os.replace(tmp, man)
        if self.world > 1:
            dist.barrier(group=self.group)
        return man

    def restore(self, manifest: str) -> int:
        """Load a checkpoint written at any world size; returns the cards this rank now owns."""
        import json
        import os
        with open(manifest) as f:
            doc = json.load(f)
        if doc.get("format") != "fdsnap/1":
            raise ValueError(f"{manifest}: not an fdengine checkpoint manifest")
        base = os.path.dirname(manifest)
        return sum(self.be.restore(os.path.join(base, img), self.rank, self.world) for img in doc["images"])


def rccl_library_path() -> str:
    """the RCCL this process uses (torch's bundled librccl.so): the engine dlopens the same file"""
    import os

    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if not os.path.exists(p):
        raise RuntimeError(f"RCCL library not found at {p}")
    return p


def image_name(step: int, rank: int, world: int) -> str:
    return f"state-{step:08d}-{rank:03d}-of-{world:03d}.fdsnap"


def latest_checkpoint(directory: str) -> Optional[str]:
    """Manifest of the newest complete checkpoint in `directory` (None if there is none)."""
    import glob
    import os
    found = sorted(glob.glob(os.path.join(directory, "checkpoint-*.json")))
    return found[-1] if found else None


def owned_mask(keys, rank: int, world: int) -> np.ndarray:
    """Which cards (e.g. user profiles to load) this rank owns."""
    return shard_of(keys, world) == rank
