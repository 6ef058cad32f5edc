#!/usr/bin/env python3
"""The sharded step's own GPU work on one GPU: the direct pipelined step (ShardedScorer at world 1 ->
fd_score_batch_pipelined, what N = 1 runs) against the streaming routed step every rank runs at N > 1
(ShardedScorer(force_route=True) over a 1-rank RCCL process group: fd_route_partition_stream of the next batch one
step ahead, the count / record all-to-alls on the forward stream, fd_score_records_pipelined, the result all-to-all
on the second group, the scatter), config-4 shapes on a warm stream (CARDS env, default 10 M; 12 h of history).
Prints ms per 64 k step back to back for each, and the routed / direct ratio."""
import os
import socket
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import torch
import torch.distributed as dist

import bench
import fdengine
from fdengine import synth, synth_gpu
from fdengine.sharding import EngineShardBackend, ShardedScorer

B, CARDS, STEPS = 65536, int(os.environ.get("CARDS", 10_000_000)), int(os.environ.get("STEPS", 200))
dev = torch.device("cuda", 0)
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
xgb, ifm = bench.fit_models(0, 500, 8, 1, 16)
params, _, _ = bench.product_blend(["xgboost_primary", "isolation_forest"])
merch = synth.merchants_table(5000, seed=100)
cap = 1
while cap < int(CARDS * 1.6) + 65536:
    cap *= 2
result = {}
VARIANTS = os.environ.get("VARIANTS", "direct,native,streaming,serial").split(",")
for name in VARIANTS:
    name_v = name
    routed = name != "direct"
    eng = fdengine.FraudEngine(0)
    eng.state_init(cap, 1, 16)
    eng.load_merchants(merch["fraud_rate"], merch["risk_multiplier"])
    if os.environ.get("STREAM_PRIORITY"):
        eng.set_option("stream_priority", int(os.environ["STREAM_PRIORITY"]))
    if os.environ.get("COUNT_EXCHANGE"):  # the native step's count exchange: 1 all-gather, 0 point-to-point
        eng.set_option("count_exchange", int(os.environ["COUNT_EXCHANGE"]))
    sc = ShardedScorer(EngineShardBackend(eng, params, [0, 1], pipelined=True), 0, 1, force_route=routed,
                       streaming=name != "serial", native=name == "native")
    w = synth_gpu.warm_workload(eng, dev, CARDS, 0, 1, STEPS + 20, B, hours=12.0, keep_batches=0)
    eng.load_forest(0, xgb)
    eng.load_forest(1, ifm)
    parts = [{f: t[i * B:(i + 1) * B] for f, t in w["resident"].items()} for i in range(STEPS + 20)]

    def run(a, b):
        for i in range(a, b):
            pre = (parts[i + 1], B) if routed and i + 1 < b else None
            sc.step(parts[i], B, prefetch=pre)

    run(0, 20)
    torch.cuda.synchronize()
    PH = ("wait", "partition", "counts", "count_copy", "records", "score", "back", "scatter")
    c0 = {ph: eng.counter("sharded_host_ns_" + ph) for ph in PH} if name == "native" else None
    k0 = eng.counter("sharded_steps") if name == "native" else 0
    t0 = time.perf_counter()
    run(20, 20 + STEPS)
    t_host = time.perf_counter()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / STEPS * 1e3
    result[name_v] = ms
    print(f"{name_v}: {ms:.4f} ms/step back to back ({B / ms / 1e3:.1f} M txn/s), host submit "
          f"{(t_host - t0) / STEPS * 1e3:.4f} ms/step", flush=True)
    if name == "native":  # the timed steps only
        k = eng.counter("sharded_steps") - k0
        print("  host us/step inside fd_sharded_step: " + ", ".join(
            f"{ph} {(eng.counter('sharded_host_ns_' + ph) - c0[ph]) / k / 1e3:.1f}" for ph in PH), flush=True)
    if os.environ.get("PROFILE_HOST") and routed:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run(0, 20)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    eng.close()
    del w, parts
for k in result:
    if "direct" in result:
        print(f"{k} / direct = {result[k] / result['direct']:.3f}", flush=True)
dist.destroy_process_group()
