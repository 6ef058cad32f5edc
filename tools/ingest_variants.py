"""Ingest kernel time per message shape (64 k simulator-format messages, full kernel): which members cost the
wave its time. Variants rewrite the same messages: locations null, score / amount short, unknown members
dropped, user agent short, timestamp without the fraction."""
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
VARIANTS = {
    "base": lambda m: m,
    "loc_null": lambda m: re.sub(rb'"(geolocation|merchant_location)": \{[^}]*\}', rb'"\1": null', m),
    "score_short": lambda m: re.sub(rb'"fraud_score": [0-9.e-]+', rb'"fraud_score": 0.5', m),
    "no_unknown": lambda m: re.sub(rb'"(currency|card_last_four|device_id|fraud_type|processing_time_ms)": '
                                   rb'("[^"]*"|null|[0-9]+), ?', b'', m),
    "ua_short": lambda m: re.sub(rb'"user_agent": "[^"]*"', rb'"user_agent": "curl/8"', m),
    "ts_nofrac": lambda m: re.sub(rb'("timestamp": "[0-9T:-]+)\.[0-9]+"', rb'\1"', m),
}
eng.set_stream(torch.cuda.current_stream().cuda_stream)
for name in [a for a in sys.argv[1:]] or list(VARIANTS):
    msgs = [VARIANTS[name](m) for m in base]
    buf, off = pack(msgs)
    dbuf, doff = torch.from_numpy(buf.copy()).cuda(), torch.from_numpy(off).cuda()
    cols, ptrs = device_columns(B)
    for _ in range(3):
        codec.parse_device(dbuf.data_ptr(), doff.data_ptr(), B, ptrs)
    torch.cuda.synchronize()
    st = cols["status"].cpu().numpy() if isinstance(cols, dict) and "status" in cols else None
    t = time.perf_counter()
    for _ in range(20):
        codec.parse_device(dbuf.data_ptr(), doff.data_ptr(), B, ptrs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    bad = "" if st is None else f", status!=0: {int((st != 0).sum())}"
    print(f"{name}: {dt * 1e6:.1f} us / 64k, {int(off[-1]) / B:.0f} B/msg{bad}", flush=True)
eng.close()
