import sys, time, re
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
variants = {
  "full": base,
  "short_ua": [re.sub(rb'"user_agent": "[^"]*"', b'"user_agent": "x"', m) for m in base],
  "no_ua_no_ids": [re.sub(rb'"(user_agent|transaction_id|device_id|device_fingerprint)": "[^"]*"', rb'"\1": "x"', m) for m in base],
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
        print(f"{name} stop={stop}: {dt*1e6:.0f} us, {int(off[-1])/B:.0f} B/msg", flush=True)
