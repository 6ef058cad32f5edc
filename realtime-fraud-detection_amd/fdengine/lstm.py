"""The lstm_sequential head's weights (ml/utils/config.py:145-157: sequence_length 10, hidden_units 128)
in the engine's layout, and its loaders.

The reference loads a Keras model with tf.keras.models.load_model (ml/models/model_manager.py:162-165)
from models/tensorflow/lstm_fraud_model.h5 and takes predict(...)[:, 1] (or the flattened single
output, :313-319). The file does not exist in the reference and neither TensorFlow nor h5py is
available here, so the engine reads the same weights exported without TensorFlow:
  * Keras names  (.npz / .safetensors): lstm/kernel [I, 4H], lstm/recurrent_kernel [H, 4H],
    lstm/bias [4H], dense/kernel [H, n_out], dense/bias [n_out] (Keras gate order i, f, c, o);
  * PyTorch names: weight_ih_l0 [4H, I], weight_hh_l0 [4H, H], bias_ih_l0, bias_hh_l0 [4H],
    fc.weight [n_out, H], fc.bias [n_out] (gate order i, f, g, o — the same order).
A .h5 path is rejected with UnsupportedModel (h5py absent).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .forest import UnsupportedModel

HIDDEN = 128
SEQ_LEN = 10


@dataclass
class LstmWeights:
    w_ih: np.ndarray                 # [4H, I]
    w_hh: np.ndarray                 # [4H, H]
    b_ih: Optional[np.ndarray]       # [4H]
    b_hh: Optional[np.ndarray]       # [4H]
    w_out: np.ndarray                # [n_out, H]
    b_out: Optional[np.ndarray]      # [n_out]

    @property
    def input_size(self) -> int:
        return int(self.w_ih.shape[1])

    @property
    def hidden(self) -> int:
        return int(self.w_hh.shape[1])

    @property
    def n_out(self) -> int:
        return int(self.w_out.shape[0])

    def validate(self) -> "LstmWeights":
        H, I = self.hidden, self.input_size
        if self.w_ih.shape != (4 * H, I) or self.w_hh.shape != (4 * H, H) or self.w_out.shape[1] != H:
            raise UnsupportedModel(f"inconsistent LSTM weight shapes {self.w_ih.shape} {self.w_hh.shape} "
                                   f"{self.w_out.shape}")
        return self


def from_keras(kernel, recurrent_kernel, bias, dense_kernel, dense_bias) -> LstmWeights:
    return LstmWeights(np.asarray(kernel, np.float32).T.copy(), np.asarray(recurrent_kernel, np.float32).T.copy(),
                       None if bias is None else np.asarray(bias, np.float32), None,
                       np.asarray(dense_kernel, np.float32).T.copy(),
                       None if dense_bias is None else np.asarray(dense_bias, np.float32)).validate()


def from_state_dict(sd: dict) -> LstmWeights:
    g = lambda k: None if sd.get(k) is None else np.asarray(sd[k], np.float32)  # noqa: E731
    out_w = next((k for k in ("fc.weight", "head.weight", "linear.weight", "out.weight") if k in sd), None)
    if out_w is None:
        raise UnsupportedModel("no dense head weight (fc.weight) in the LSTM state dict")
    return LstmWeights(g("weight_ih_l0"), g("weight_hh_l0"), g("bias_ih_l0"), g("bias_hh_l0"), g(out_w),
                       g(out_w.replace("weight", "bias"))).validate()


def load_lstm_file(path: str) -> LstmWeights:
    if path.endswith(".h5"):
        raise UnsupportedModel("Keras .h5 needs h5py/TensorFlow (absent): export the weights to .safetensors "
                               "or .npz with Keras or PyTorch names")
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        d = load_file(path)
    else:
        with np.load(path, allow_pickle=False) as z:
            d = {k: z[k] for k in z.files}
    if "lstm/kernel" in d:
        return from_keras(d["lstm/kernel"], d["lstm/recurrent_kernel"], d.get("lstm/bias"), d["dense/kernel"],
                          d.get("dense/bias"))
    return from_state_dict(d)


def random_weights(input_size: int = 16, hidden: int = HIDDEN, n_out: int = 1, seed: int = 0) -> LstmWeights:
    """Random-init weights (PyTorch's U(-1/sqrt(H), 1/sqrt(H)); forget-gate bias 1 as Keras'
    unit_forget_bias) — no trained checkpoint exists for this head."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = 1.0 / np.sqrt(hidden)
    u = lambda *s: rng.uniform(-k, k, s).astype(np.float32)  # noqa: E731
    b_ih = u(4 * hidden)
    b_ih[hidden:2 * hidden] += 1.0
    return LstmWeights(u(4 * hidden, input_size), u(4 * hidden, hidden), b_ih, u(4 * hidden),
                       rng.uniform(-0.3, 0.3, (n_out, hidden)).astype(np.float32),
                       rng.uniform(-0.1, 0.1, n_out).astype(np.float32)).validate()


def save_npz(path: str, w: LstmWeights, keras: bool = True) -> None:
    if keras:
        b = (w.b_ih if w.b_ih is not None else 0) + (w.b_hh if w.b_hh is not None else 0)
        np.savez(path, **{"lstm/kernel": w.w_ih.T, "lstm/recurrent_kernel": w.w_hh.T,
                          "lstm/bias": np.asarray(b, np.float32), "dense/kernel": w.w_out.T,
                          "dense/bias": w.b_out if w.b_out is not None else np.zeros(w.n_out, np.float32)})
    else:
        np.savez(path, weight_ih_l0=w.w_ih, weight_hh_l0=w.w_hh, bias_ih_l0=w.b_ih, bias_hh_l0=w.b_hh,
                 **{"fc.weight": w.w_out, "fc.bias": w.b_out})
