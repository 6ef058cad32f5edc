"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's cpu_baseline may import it; the product
never does). CPU restatement of the LSTM sequence head (realtime-fraud-detection_amd/csrc/lstm.hip) and of
the per-card event history the feature kernel keeps for it (csrc/features.hip, seq ring).

Reference: lstm_sequential (services/ml-models/src/utils/config.py:145-157, sequence_length 10,
hidden_units 128) predicted by ModelManager._predict_tensorflow (model_manager.py:313-319). The reference
has no model file and TensorFlow is absent, so the oracle is a plain PyTorch fp32 CPU forward of the same
architecture (torch.nn.LSTM + Linear, gate order i, f, g, o = Keras' i, f, c, o) — parity unpinned
against Keras itself; tolerance 1e-5 on probabilities.
"""
from __future__ import annotations

from collections import defaultdict, deque

import numpy as np

SEQ_INPUT = 16


def event_inputs(raw: np.ndarray) -> np.ndarray:
    """Bridged raw features [n, 16] f64 -> per-event LSTM inputs f32: NaN -> 0, sign(x) * log1p(|x|)."""
    r = np.asarray(raw, np.float64)
    a = np.log1p(np.abs(np.nan_to_num(r, nan=0.0)))
    return np.where(r < 0, -a, a).astype(np.float32)


class SequenceState:
    """Each card's last T events (oldest -> newest); sequences left-padded with zero events."""

    def __init__(self, T: int):
        self.T = T
        self.hist = defaultdict(lambda: deque(maxlen=T))

    def run(self, keys, raw) -> np.ndarray:
        ev = event_inputs(raw)
        n = len(ev)
        out = np.zeros((n, self.T, SEQ_INPUT), np.float32)
        for i in range(n):
            k = int(keys[i]) or 1
            h = self.hist[k]
            h.append(ev[i])
            m = len(h)
            out[i, self.T - m:] = np.stack(h)
        return out


def lstm_forward(w, seq: np.ndarray) -> np.ndarray:
    """PyTorch fp32 CPU forward. w: fdengine.lstm.LstmWeights-like; seq [n, T, >= input_size]."""
    import torch
    I, H, n_out = w.w_ih.shape[1], w.w_hh.shape[1], w.w_out.shape[0]
    x = torch.from_numpy(np.ascontiguousarray(np.asarray(seq, np.float32)[:, :, :I]))
    with torch.no_grad():
        m = torch.nn.LSTM(I, H, batch_first=True)
        m.weight_ih_l0.copy_(torch.from_numpy(np.asarray(w.w_ih, np.float32)))
        m.weight_hh_l0.copy_(torch.from_numpy(np.asarray(w.w_hh, np.float32)))
        m.bias_ih_l0.copy_(torch.from_numpy(np.asarray(w.b_ih if w.b_ih is not None else np.zeros(4 * H), np.float32)))
        m.bias_hh_l0.copy_(torch.from_numpy(np.asarray(w.b_hh if w.b_hh is not None else np.zeros(4 * H), np.float32)))
        _, (h, _) = m(x)
        z = h[0] @ torch.from_numpy(np.asarray(w.w_out, np.float32)).T
        if w.b_out is not None:
            z = z + torch.from_numpy(np.asarray(w.b_out, np.float32))
        p = torch.sigmoid(z[:, 0]) if n_out == 1 else torch.softmax(z, dim=1)[:, 1]
    return p.double().numpy()
