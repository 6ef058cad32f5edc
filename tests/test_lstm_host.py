"""CPU: LSTM head host side — weight formats (Keras / PyTorch names, .npz / .safetensors) load to the same
model, .h5 is refused, the oracle's event history and inputs follow the declared rules, and the
registry resolves lstm_sequential's .h5 path to its exported sibling."""
import numpy as np
import pytest

from fdengine import lstm as L
from oracle import lstm_ref as R


def test_keras_and_torch_exports_are_the_same_model(tmp_path):
    w = L.random_weights(16, 128, 2, seed=3)
    seq = np.random.default_rng(1).normal(0, 1, (7, 10, 16)).astype(np.float32)
    ref = R.lstm_forward(w, seq)
    L.save_npz(str(tmp_path / "k.npz"), w, keras=True)
    L.save_npz(str(tmp_path / "t.npz"), w, keras=False)
    from safetensors.numpy import save_file
    save_file({"weight_ih_l0": w.w_ih, "weight_hh_l0": w.w_hh, "bias_ih_l0": w.b_ih, "bias_hh_l0": w.b_hh,
               "fc.weight": w.w_out, "fc.bias": w.b_out}, str(tmp_path / "t.safetensors"))
    for f in ("k.npz", "t.npz", "t.safetensors"):
        w2 = L.load_lstm_file(str(tmp_path / f))
        assert (w2.input_size, w2.hidden, w2.n_out) == (16, 128, 2)
        np.testing.assert_allclose(R.lstm_forward(w2, seq), ref, atol=1e-6)


def test_h5_is_refused(tmp_path):
    from fdengine.forest import UnsupportedModel
    p = tmp_path / "lstm_fraud_model.h5"
    p.write_bytes(b"\x89HDF\r\n")
    with pytest.raises(UnsupportedModel):
        L.load_lstm_file(str(p))


def test_bad_shapes_are_refused():
    from fdengine.forest import UnsupportedModel
    w = L.random_weights(16, 128, 1)
    with pytest.raises(UnsupportedModel):
        L.LstmWeights(w.w_ih[:, :8], w.w_hh[:100], w.b_ih, w.b_hh, w.w_out, w.b_out).validate()


def test_event_inputs_and_history():
    raw = np.array([[np.nan, -3.0, 0.0, 12.5] + [1.0] * 12, [2.0] * 16], np.float64)
    ev = R.event_inputs(raw)
    assert ev.dtype == np.float32
    assert ev[0, 0] == 0 and ev[0, 1] == np.float32(-np.log1p(3.0)) and ev[0, 2] == 0
    assert ev[0, 3] == np.float32(np.log1p(12.5))
    st = R.SequenceState(3)
    keys = np.array([5, 6, 5, 5, 5], np.uint64)
    r = np.arange(5 * 16, dtype=np.float64).reshape(5, 16)
    out = st.run(keys, r)
    e = R.event_inputs(r)
    assert (out[0, :2] == 0).all() and (out[0, 2] == e[0]).all()      # left-padded
    assert (out[2, 1] == e[0]).all() and (out[2, 2] == e[2]).all()     # card 5's 2 events
    assert (out[4] == e[[2, 3, 4]]).all()                              # window of the last 3
    out2 = st.run(np.array([6], np.uint64), r[:1])                     # history carried across batches
    assert (out2[0, 1] == e[1]).all() and (out2[0, 2] == e[0]).all()


def test_registry_resolves_h5_to_export(tmp_path):
    from fdengine.model_manager import _lstm_weight_file
    h5 = tmp_path / "tensorflow" / "lstm_fraud_model.h5"
    h5.parent.mkdir()
    assert _lstm_weight_file(str(h5)) is None
    L.save_npz(str(h5.with_suffix(".npz")), L.random_weights())
    assert _lstm_weight_file(str(h5)) == str(h5.with_suffix(".npz"))
