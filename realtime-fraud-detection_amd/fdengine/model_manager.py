"""Drop-in for the reference's model registry on the scoring path:
services/ml-models/src/models/model_manager.py (class ModelManager).

Same public surface — `load_all_models`, `predict(model_name, features) -> np.ndarray`,
`is_model_loaded`, `reload_model`, `reload_all_models`, `get_loaded_models`, `get_model_info`,
`cleanup` — and the same model files, but the two tree ensembles on the path run on the MI355X:

  model_type "xgboost"  unchanged XGBoost JSON (`_load_xgboost_model` :157-161) -> engine slot;
                        predict returns predict_proba(X)[:, 1] as float32 (`_predict_xgboost` :309-311)
  model_type "sklearn"  unchanged joblib IsolationForest (`_load_sklearn_model` :197-200) -> engine
                        slot; predict returns 1/(1+exp(decision_function)) (`_predict_sklearn` :338-346)

  model_type "tensorflow" lstm_sequential weights (`_load_tensorflow_model` :162-165) -> the engine's LSTM
                        head (fdengine/lstm.py formats; the .h5 path's .safetensors/.npz sibling);
                        predict takes [n, T, I] sequences (`_predict_tensorflow` :313-319); a flat
                        scoring vector raises as a Keras LSTM given a 2-D input does

Everything else keeps the reference's observable behaviour, so the ensemble above sees the same
model set: a missing model file yields the reference's random DummyModel (:115-118, 244-277);
its tensorflow / pytorch predict branches fail for a DummyModel exactly as the reference's do
(:313-331: `predict(..., verbose=0)` / `model(tensor)` raise TypeError) and the ensemble drops
them; "transformers" returns np.random (:332-336). Real tensorflow / pytorch / transformers model
files are outside this path and are rejected at load (logged, model not loaded).
"""
from __future__ import annotations

import asyncio
import logging
import os
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime
from typing import Any, Dict, Optional

import numpy as np

from .engine import FraudEngine
from .forest import UnsupportedModel, iforest_from_sklearn

log = logging.getLogger("fdengine.model_manager")


class DummyModel:
    """The reference's development stand-in for a missing model file (model_manager.py:248-277)."""

    def __init__(self, model_type: str, name: str):
        self.model_type = model_type
        self.name = name

    @staticmethod
    def _n(X) -> int:
        if isinstance(X, (list, tuple)):
            return len(X)
        if hasattr(X, "shape"):
            return X.shape[0] if len(X.shape) > 1 else 1
        return 1

    def predict(self, X):
        return np.random.random(self._n(X))

    def predict_proba(self, X):
        p = np.random.random((self._n(X), 2))
        return p / p.sum(axis=1, keepdims=True)


class EngineLstm:
    """The LSTM head resident in the engine (one per engine)."""

    def __init__(self, input_size: int, hidden: int, n_out: int, path: str):
        self.kind, self.input_size, self.hidden, self.n_out, self.path = "lstm", input_size, hidden, n_out, path


def _lstm_weight_file(path: str) -> Optional[str]:
    """The .h5 the registry names cannot be read without TensorFlow; its exported siblings can."""
    stem, ext = os.path.splitext(path)
    for cand in ([path] if ext in (".npz", ".safetensors") else []) + [stem + ".safetensors", stem + ".npz"]:
        if os.path.exists(cand):
            return cand
    return None


class EngineForest:
    """A forest resident in the engine (one slot)."""

    def __init__(self, slot: int, kind: str, num_feature: int, n_trees: int, depth: int):
        self.slot, self.kind, self.num_feature, self.n_trees, self.depth = slot, kind, num_feature, n_trees, depth


def _default_device() -> int:
    for k in ("FDENGINE_DEVICE", "LOCAL_RANK"):
        if os.environ.get(k, "").strip():
            return int(os.environ[k])
    return 0


class ModelManager:
    def __init__(self, config, device: Optional[int] = None, engine: Optional[FraudEngine] = None):
        self.config = config
        self.logger = log
        self.models: Dict[str, Any] = {}
        self.model_metadata: Dict[str, Dict[str, Any]] = {}
        self.model_load_times: Dict[str, datetime] = {}
        self.model_lock = asyncio.Lock()
        self.engine = engine if engine is not None else FraudEngine(_default_device() if device is None else device)
        # GPU round trips run off the event loop (uvicorn's single loop stays responsive). Calls that
        # stay on the loop's thread (predict_batch, loads, reloads) may overlap one in this worker: the library
        # serialises every entry point on one engine (a per-engine lock, include/fdengine.h), and an unload syncs
        # the engine's streams before freeing a forest (ctypes releases the GIL for each call's duration)
        self._executor = ThreadPoolExecutor(max_workers=1, thread_name_prefix="fdengine")
        names = list(config.models.keys())
        self._slot_of = {name: i for i, name in enumerate(names)}  # one engine slot per registry entry

    # ----------------------------------------------------------------------------- loading
    async def load_all_models(self) -> None:
        async with self.model_lock:
            enabled = self.config.get_enabled_models()
            results = await asyncio.gather(*(self._load_single_model(n, c) for n, c in enabled.items()),
                                           return_exceptions=True)
            ok = 0
            for name, r in zip(enabled.keys(), results):
                if isinstance(r, Exception):
                    self.logger.error(f"Failed to load model {name}: {r}")
                else:
                    ok += 1
            self.logger.info(f"Loaded {ok}/{len(enabled)} models successfully")

    async def _load_single_model(self, name: str, cfg) -> None:
        lstm_file = _lstm_weight_file(cfg.model_path) if cfg.model_type == "tensorflow" else None
        if lstm_file is not None:
            model = self._load_lstm(lstm_file)
        elif not os.path.exists(cfg.model_path):
            self.logger.warning(f"Model file not found: {cfg.model_path}. Creating dummy model.")
            model = DummyModel(cfg.model_type, name)
        else:
            model = self._load_by_type(name, cfg)
        self.models[name] = model
        self.model_load_times[name] = datetime.now()
        self.model_metadata[name] = {
            "type": cfg.model_type, "path": cfg.model_path, "weight": cfg.weight,
            "loaded_at": self.model_load_times[name].isoformat(),
            "hyperparameters": getattr(cfg, "hyperparameters", {}),
            "preprocessing_steps": getattr(cfg, "preprocessing_steps", []),
            "engine": (vars(model) if isinstance(model, (EngineForest, EngineLstm)) else None),
        }

    def _load_by_type(self, name: str, cfg):
        slot = self._slot_of.setdefault(name, len(self._slot_of))
        if cfg.model_type == "xgboost":  # the unchanged JSON file, parsed by the engine (fd_load_xgboost_json)
            self.engine.load_xgboost_file(slot, cfg.model_path)
            info = self.engine.forest_info(slot)
            return EngineForest(slot, "xgboost", info["num_feature"], info["n_trees"], info["depth"])
        if cfg.model_type == "sklearn":
            import joblib
            model = joblib.load(cfg.model_path)
            if type(model).__name__ != "IsolationForest":
                raise UnsupportedModel(f"sklearn model {type(model).__name__} is not on the engine path")
            return self._upload(slot, iforest_from_sklearn(model), "isolation_forest")
        raise UnsupportedModel(f"model_type {cfg.model_type!r} files are not served by the engine")

    def _load_lstm(self, path: str) -> EngineLstm:
        from .lstm import load_lstm_file
        w = load_lstm_file(path)
        self.engine.load_lstm(w)
        return EngineLstm(w.input_size, w.hidden, w.n_out, path)

    def _upload(self, slot: int, fa, kind: str) -> EngineForest:
        self.engine.load_forest(slot, fa)
        info = self.engine.forest_info(slot)
        return EngineForest(slot, kind, info["num_feature"], info["n_trees"], info["depth"])

    # ----------------------------------------------------------------------------- predict
    async def predict(self, model_name: str, features: np.ndarray) -> np.ndarray:
        if model_name not in self.models:
            raise ValueError(f"Model {model_name} not loaded")
        model = self.models[model_name]
        cfg = self.config.get_model_config(model_name)
        try:
            loop = asyncio.get_running_loop()
            return await loop.run_in_executor(self._executor, self.predict_sync, model_name, model, cfg.model_type,
                                              features)
        except Exception as e:
            self.logger.error(f"prediction failed: {e}", extra={"model_name": model_name, "model_type": cfg.model_type,
                                                                "features_shape": getattr(features, "shape", None)})
            raise

    def predict_sync(self, name: str, model, model_type: str, features: np.ndarray) -> np.ndarray:
        if isinstance(model, EngineLstm):
            X = np.asarray(features)
            if X.ndim != 3:  # Keras: an LSTM layer needs [batch, timesteps, features]
                raise ValueError(f"Input 0 of layer lstm is incompatible: expected ndim=3, found ndim={X.ndim}")
            return self.engine.lstm_predict(X).astype(np.float32)
        if isinstance(model, EngineForest):
            X = np.asarray(features)
            if X.ndim == 1:
                X = X.reshape(1, -1)
            if model.kind == "xgboost":
                if X.shape[1] > model.num_feature:  # XGBoost's Learner::ValidateDMatrix
                    raise ValueError(f"Feature shape mismatch, expected: {model.num_feature}, got {X.shape[1]}")
                return self.engine.predict(model.slot, X).astype(np.float32)
            if X.shape[1] != model.num_feature:  # sklearn's validate_data(reset=False) n_features_in_ check
                raise ValueError(f"X has {X.shape[1]} features, but IsolationForest is expecting "
                                 f"{model.num_feature} features as input.")
            return self.engine.predict(model.slot, X)
        # reference branches for the DummyModel stand-ins (model_manager.py:288-300, 313-336)
        if model_type == "xgboost":
            return model.predict_proba(features)[:, 1]
        if model_type == "tensorflow":
            predictions = model.predict(features, verbose=0)  # DummyModel: TypeError, as in the reference
            return predictions[:, 1] if predictions.shape[1] > 1 else predictions.flatten()
        if model_type == "pytorch":
            return model(features)  # DummyModel is not callable: TypeError, as in the reference
        if model_type == "transformers":
            return np.random.random(features.shape[0])
        if model_type == "sklearn":
            if hasattr(model, "predict_proba"):
                return model.predict_proba(features)[:, 1]
            return 1.0 / (1.0 + np.exp(model.decision_function(features)))
        return model.predict_proba(features)[:, 1]

    # ----------------------------------------------------------------------------- registry
    async def reload_model(self, model_name: str) -> None:
        if model_name not in self.config.models:
            raise ValueError(f"Model {model_name} not found in configuration")
        async with self.model_lock:
            cfg = self.config.get_model_config(model_name)
            if model_name in self.models:
                m = self.models.pop(model_name)
                self.model_metadata.pop(model_name, None)
                self.model_load_times.pop(model_name, None)
                self._unload(m)
            await self._load_single_model(model_name, cfg)

    async def reload_all_models(self) -> None:
        for name in list(self.models):
            self._unload(self.models[name])
        self.models.clear()
        self.model_metadata.clear()
        self.model_load_times.clear()
        await self.load_all_models()

    def get_loaded_models(self) -> Dict[str, Any]:
        return {n: {"type": self.model_metadata[n]["type"], "loaded_at": self.model_metadata[n]["loaded_at"],
                    "weight": self.model_metadata[n]["weight"]} for n in self.models}

    def get_model_info(self) -> Dict[str, Any]:
        return {"total_models": len(self.models), "models": self.model_metadata,
                "last_reload": max(self.model_load_times.values()).isoformat() if self.model_load_times else None}

    def is_model_loaded(self, model_name: str) -> bool:
        return model_name in self.models

    def _unload(self, m) -> None:
        if isinstance(m, EngineForest):
            self.engine.unload_forest(m.slot)
        elif isinstance(m, EngineLstm):
            self.engine.unload_lstm()

    def engine_slot(self, model_name: str) -> int:
        """Engine slot of a device-resident model (FD_SLOT_LSTM for the LSTM head), -1 otherwise."""
        m = self.models.get(model_name)
        if isinstance(m, EngineLstm):
            from ._native import FD_SLOT_LSTM
            return FD_SLOT_LSTM
        return m.slot if isinstance(m, EngineForest) else -1

    async def cleanup(self) -> None:
        async with self.model_lock:
            for name, m in list(self.models.items()):
                self._unload(m)
            self.models.clear()
            self.model_metadata.clear()
            self.model_load_times.clear()
