"""Kafka JSON -> SoA ingest on the device: the drop-in for TransactionDeserializationSchema.deserialize
(services/flink-jobs/.../serialization/TransactionDeserializationSchema.java:28-49) over the simulator's wire
format (json.dumps(asdict(Transaction), default=str), services/data-simulator/src/main/python/simulator.py:186).

A micro-batch of raw message values (as a Kafka consumer hands them over) is packed into one byte buffer +
n+1 offsets and parsed by libfdengine.so (ingest.hip, one wavefront per message) into the engine's SoA columns:
fd_txn_batch (features / windows / routing), fd_txn_context (feature map / rule scores) and the window inputs.
Identities are fd_hash64 of the strings (card_key = hash64(user_id), device fingerprints likewise); merchants
and the payment / type / card vocabularies map to the engine's table indices.

Vocabulary growth is control plane: a string outside a vocabulary parses as FD_VOCAB_OTHER with status
FD_INGEST_UNKNOWN_VOCAB; `parse(..., grow_vocab=True)` then appends the new strings (first-occurrence order),
re-derives the engine's vocabulary flags (FeatureExtractor.isHighRiskPaymentMethod :486-493, the "refund"
equalsIgnoreCase test :377) and parses the batch again on the device.
"""
from __future__ import annotations

import ctypes as C
import json
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native as N

DTYPES = dict(N.INGEST_FIELDS)


def hash64(s) -> int:
    """fd_hash64 of a str (UTF-8) or bytes: the key the codec gives user ids / device fingerprints."""
    b = s.encode("utf-8", "surrogatepass") if isinstance(s, str) else bytes(s)
    arr = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    out = C.c_uint64()
    N.call("fd_hash64", C.c_void_p(arr.ctypes.data), len(b), C.byref(out))
    return out.value


def hash64_many(strings: Sequence) -> np.ndarray:
    return np.array([hash64(s) for s in strings], dtype=np.uint64)


def pack(messages: Sequence[bytes]):
    """-> (uint8 buffer, int64 offsets[n+1]) — the codec's batch layout."""
    lens = np.fromiter((len(m) for m in messages), dtype=np.int64, count=len(messages))
    offsets = np.zeros(len(messages) + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(messages), np.uint8) if len(messages) else np.zeros(0, np.uint8)
    return buf, offsets


def payment_high_risk(s: str) -> bool:
    """FeatureExtractor.isHighRiskPaymentMethod (FeatureExtractor.java:486-493)."""
    lo = s.lower()
    return any(w in lo for w in ("prepaid", "gift", "crypto", "wire"))


def is_refund(s: str) -> bool:
    """"refund".equalsIgnoreCase(transactionType) (FeatureExtractor.java:377)."""
    return s.lower() == "refund"


class IngestCodec:
    """Device JSON codec bound to one FraudEngine (its vocabularies and merchant table)."""

    def __init__(self, engine, merchant_ids: Sequence[str] = (), payment_methods: Sequence[str] = (),
                 transaction_types: Sequence[str] = (), card_types: Sequence[str] = ()):
        self.eng = engine
        self.vocab: List[List[str]] = [[], [], []]
        self.set_merchants(merchant_ids)
        for w, v in enumerate((payment_methods, transaction_types, card_types)):
            self.set_vocab(w, v)

    # ------------------------------------------------------------------ tables
    @staticmethod
    def _strings(strings):
        bs = [s.encode("utf-8", "surrogatepass") for s in strings]
        return pack(bs)

    def set_merchants(self, ids: Sequence[str]) -> None:
        buf, off = self._strings(ids)
        N.call("fd_ingest_set_merchants", self.eng.handle, C.c_void_p(buf.ctypes.data) if len(buf) else None,
               C.c_void_p(off.ctypes.data), len(ids))
        self.merchant_index = {s: i for i, s in reversed(list(enumerate(ids)))}

    def set_vocab(self, which: int, strings: Sequence[str]) -> None:
        strings = list(strings)
        if len(strings) > N.FD_VOCAB_OTHER:
            raise ValueError("a vocabulary holds at most 254 strings")
        buf, off = self._strings(strings)
        N.call("fd_ingest_set_vocab", self.eng.handle, int(which), C.c_void_p(buf.ctypes.data) if len(buf) else None,
               C.c_void_p(off.ctypes.data), len(strings))
        self.vocab[which] = strings

    def vocab_flags(self):
        """(payment code -> high risk, type code -> refund) flags for FraudEngine.load_vocab."""
        pay = np.zeros(256, np.uint8)
        ref = np.zeros(256, np.uint8)
        for i, s in enumerate(self.vocab[0]):
            pay[i] = payment_high_risk(s)
        for i, s in enumerate(self.vocab[1]):
            ref[i] = is_refund(s)
        return pay, ref

    def sync_engine_vocab(self) -> None:
        self.eng.load_vocab(*self.vocab_flags())

    # ------------------------------------------------------------------ parsing
    def parse(self, messages: Sequence[bytes], grow_vocab: bool = False) -> Dict[str, np.ndarray]:
        """Host messages -> host columns (staged through the device; synchronous)."""
        buf, off = pack(messages)
        cols = self._parse_packed(buf, off)
        if grow_vocab and (cols["status"] & N.FD_INGEST_UNKNOWN_VOCAB).any():
            if self._learn(messages, cols["status"]):
                self.sync_engine_vocab()
                cols = self._parse_packed(buf, off)
        return cols

    def _parse_packed(self, buf: np.ndarray, off: np.ndarray) -> Dict[str, np.ndarray]:
        n = len(off) - 1
        cols = {k: np.empty(n, dt) for k, dt in N.INGEST_FIELDS}
        out = N.fd_ingest_out(*[cols[k].ctypes.data for k, _ in N.INGEST_FIELDS])
        keep = buf if len(buf) else np.zeros(1, np.uint8)
        N.call("fd_ingest_json_host", self.eng.handle, C.c_void_p(keep.ctypes.data), C.c_void_p(off.ctypes.data), n,
               C.byref(out))
        return cols

    def parse_device(self, bytes_ptr: int, offsets_ptr: int, n: int, out_ptrs: Dict[str, int]) -> None:
        """HBM-resident batch -> HBM columns (device pointers; any column may be omitted). Asynchronous on
        the engine's stream."""
        out = N.fd_ingest_out(*[int(out_ptrs.get(k) or 0) or None for k, _ in N.INGEST_FIELDS])
        N.call("fd_ingest_json_device", self.eng.handle, C.c_void_p(bytes_ptr), C.c_void_p(offsets_ptr), int(n),
               C.byref(out))

    def _learn(self, messages: Sequence[bytes], status: np.ndarray) -> bool:
        """Append the unknown vocabulary strings of the flagged rows (first-occurrence order)."""
        keys = (("payment_method", "paymentMethod"), ("transaction_type", "transactionType"),
                ("card_type", "cardType"))
        grew = False
        for i in np.flatnonzero(status & N.FD_INGEST_UNKNOWN_VOCAB):
            try:
                doc = json.loads(messages[i])
            except ValueError:
                continue
            for w, names in enumerate(keys):
                v = None
                for k in names:
                    if k in doc:
                        v = doc[k]
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    v = json.dumps(v)
                elif isinstance(v, bool):
                    v = "true" if v else "false"
                if isinstance(v, str) and v not in self.vocab[w] and len(self.vocab[w]) < N.FD_VOCAB_OTHER:
                    self.vocab[w].append(v)
                    grew = True
        if grew:
            for w in range(3):
                self.set_vocab(w, self.vocab[w])
        return grew


def txn_batch_ptrs(cols: Dict[str, int]) -> Dict[str, int]:
    """The fd_txn_batch subset of parse_device's column pointers (FraudEngine.*_device takes it)."""
    return {k: cols[k] for k in N.TXN_FIELDS}


def context_ptrs(cols: Dict[str, int]) -> Dict[str, int]:
    return {k: cols[k] for k in N.CTX_FIELDS}


def device_columns(n: int, device: Optional[int] = None):
    """Allocate the codec's output columns as torch tensors on the GPU -> (tensors, pointers)."""
    import torch
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device())
    tmap = {"<u8": torch.int64, "<i8": torch.int64, "<i4": torch.int32, "u1": torch.uint8, "<f8": torch.float64}
    t = {k: torch.empty(n, dtype=tmap[dt], device=dev) for k, dt in N.INGEST_FIELDS}
    return t, {k: v.data_ptr() for k, v in t.items()}
