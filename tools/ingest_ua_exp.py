"""Ingest cost breakdown: the same 64k simulator messages with one group of members rewritten or removed
(kernel time per variant; stop_after=2 times staging + structure only)."""
import re
import sys
import time
sys.path[:0] = [".", "realtime-fraud-detection_amd"]
import torch
import fdengine
from fdengine import synth
from fdengine.ingest import IngestCodec, device_columns, pack
eng = fdengine.FraudEngine(0)
mids = [f"merchant_{i:08x}" for i in range(5000)]
codec = IngestCodec(eng, mids, synth.SIM_PAYMENT_METHODS, synth.SIM_TXN_TYPES, synth.SIM_CARD_TYPES)
B = 65536
base = synth.json_messages_fast(B, 10_000_000, mids, seed=1)


def sub(pat, rep):
    return [re.sub(pat, rep, m) for m in base]


variants = {
    "full": base,
    "short_ua": sub(rb'"user_agent": "[^"]*"', b'"user_agent": "x"'),
    "ua_110_ascii": sub(rb'"user_agent": "[^"]*"', b'"user_agent": "' + b"a" * 110 + b'"'),
    "ua_no_escapes": [m.replace(b"\\u00e9\\u4e2d", b"ee") for m in base],
    "no_locations": sub(rb', "(geolocation|merchant_location)": \{[^}]*\}', b''),
    "no_unknown": sub(rb', "(currency|card_last_four|device_id|fraud_type|processing_time_ms)": ("[^"]*"|null|\d+)', b''),
    "no_timestamp_str": sub(rb'"timestamp": "[^"]*"', b'"timestamp": "2025-09-05T00:00:00"'),
    "short_ids": sub(rb'"(transaction_id|device_fingerprint)": "[^"]*"', rb'"\1": "x"'),
}
for name, msgs in variants.items():
    for stop in (2, 0):
        eng.set_option("ingest_stop_after", stop)
        buf, off = pack(msgs)
        dbuf, doff = torch.from_numpy(buf.copy()).cuda(), torch.from_numpy(off).cuda()
        cols, ptrs = device_columns(B)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        for _ in range(3):
            codec.parse_device(dbuf.data_ptr(), doff.data_ptr(), B, ptrs)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            codec.parse_device(dbuf.data_ptr(), doff.data_ptr(), B, ptrs)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 10
        print(f"{name:18s} stop={stop}: {dt * 1e6:7.0f} us, {int(off[-1]) / B:.0f} B/msg", flush=True)
eng.set_option("ingest_stop_after", 0)
