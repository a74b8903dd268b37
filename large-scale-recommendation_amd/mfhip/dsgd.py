"""Mirror of the reference's Flink-ML DSGD predictor, backed by libmfhip.

    sgd = DSGDforMF().setIterations(10).setNumFactors(10).setLearningRate(0.001).setBlocks(4)
    sgd.fit(ratings)                 # (user, item, rating) tuples or three arrays
    sgd.predict(pairs)               # inner join semantics: unknown ids are dropped
    sgd.empiricalRisk(labeled)
    users, items = sgd.factorsOption # lists of Factors(id, vector), ascending id

fl/mf/offline/DSGDforMF.scala:130-357 and fl/mf/offline/MatrixFactorization.scala:58-281.
Parameters and defaults follow MatrixFactorization.scala:201-223 and DSGDforMF.scala:163-169.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .context import Context
from .core import FactorVector

Factors = FactorVector


# --- flink-ml 1.3 LearningRateMethod --------------------------------------------------------
class LearningRateMethodTrait:
    code = 0
    arg = 0.0


class _Default(LearningRateMethodTrait):
    code, arg = 0, 0.0

    def __repr__(self):
        return "Default"


class _Constant(LearningRateMethodTrait):
    code, arg = 1, 0.0

    def __repr__(self):
        return "Constant"


@dataclass
class Bottou(LearningRateMethodTrait):
    optimalInit: float
    code = 2

    @property
    def arg(self):
        return self.optimalInit


@dataclass
class InvScaling(LearningRateMethodTrait):
    decay: float
    code = 3

    @property
    def arg(self):
        return self.decay


@dataclass
class Xu(LearningRateMethodTrait):
    decay: float
    code = 4

    @property
    def arg(self):
        return self.decay


class LearningRateMethod:
    Default = _Default()
    Constant = _Constant()
    Bottou = Bottou
    InvScaling = InvScaling
    Xu = Xu


def _columns(data) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    if isinstance(data, tuple) and len(data) == 3 and hasattr(data[0], "__len__") and not np.isscalar(data[0]):
        u, i, r = L.as_i32(data[0]), L.as_i32(data[1]), L.as_f64(data[2])
        L.same_length(u, i, r)
        return u, i, r
    arr = list(data)
    if not arr:
        return np.empty(0, np.int32), np.empty(0, np.int32), np.empty(0, np.float64)
    u = np.fromiter((t[0] for t in arr), np.int32, len(arr))
    i = np.fromiter((t[1] for t in arr), np.int32, len(arr))
    r = np.fromiter((t[2] for t in arr), np.float64, len(arr))
    return u, i, r


def _pairs(data) -> Tuple[np.ndarray, np.ndarray]:
    if isinstance(data, tuple) and len(data) == 2 and hasattr(data[0], "__len__") and not np.isscalar(data[0]):
        u, i = L.as_i32(data[0]), L.as_i32(data[1])
        L.same_length(u, i)
        return u, i
    arr = list(data)
    u = np.fromiter((t[0] for t in arr), np.int32, len(arr))
    i = np.fromiter((t[1] for t in arr), np.int32, len(arr))
    return u, i


class DSGDforMF:
    """DSGDforMF (fl/mf/offline/DSGDforMF.scala:130-155) on MI355X.

    mode="deterministic" replays the reference's exact per-block update order in f64 (same
    seed => bit-identical factors); mode="fast" runs the f32 conflict-free rotation schedule.
    devices: GPU ids for an in-process multi-GPU fit (numBlocks must be a multiple of their count).
    """

    def __init__(self, mode: str = "deterministic", devices: Optional[Sequence[int]] = None,
                 fast_waves: int = 0):
        self.mode = mode
        self.devices = list(devices) if devices is not None else None
        self.fast_waves = fast_waves
        self.parameters = {
            "NumFactors": 10, "Lambda": 1.0, "Iterations": 10, "Blocks": None, "Seed": 0,
            "TemporaryPath": None, "LearningRate": 0.001, "LearningRateMethod": LearningRateMethod.Default,
        }
        self.factorsOption: Optional[Tuple[List[Factors], List[Factors]]] = None
        self._ctx: Optional[Context] = None

    # fluent setters (MatrixFactorization.scala:71-125, DSGDforMF.scala:140-154)
    def setNumFactors(self, v: int): self.parameters["NumFactors"] = int(v); return self
    def setLambda(self, v: float): self.parameters["Lambda"] = float(v); return self
    def setIterations(self, v: int): self.parameters["Iterations"] = int(v); return self
    def setBlocks(self, v: int): self.parameters["Blocks"] = int(v); return self
    def setSeed(self, v: Optional[int]): self.parameters["Seed"] = None if v is None else int(v); return self
    def setTemporaryPath(self, v: str): self.parameters["TemporaryPath"] = v; return self
    def setLearningRate(self, v: float): self.parameters["LearningRate"] = float(v); return self
    def setLearningRateMethod(self, m): self.parameters["LearningRateMethod"] = m; return self

    def _params(self, overrides: Optional[dict] = None) -> L.mf_params:
        P = dict(self.parameters)
        if overrides:
            P.update(overrides)
        p = L.default_params()
        p.num_factors = P["NumFactors"]
        p.lambda_ = P["Lambda"]
        p.iterations = P["Iterations"]
        p.num_blocks = P["Blocks"] if P["Blocks"] is not None else 1  # getOrElse(1) (:270)
        p.has_seed = 0 if P["Seed"] is None else 1
        p.seed = 0 if P["Seed"] is None else P["Seed"]
        p.learning_rate = P["LearningRate"]
        m = P["LearningRateMethod"]
        p.lr_method = int(m.code)
        p.lr_arg = float(m.arg)
        p.mode = L.MODE_FAST_F32 if self.mode == "fast" else L.MODE_DETERMINISTIC_F64
        p.fast_waves = self.fast_waves
        return p

    # FitOperation (DSGDforMF.scala:262-357)
    def fit(self, input, fitParameters: Optional[dict] = None) -> "DSGDforMF":
        u, i, r = _columns(input)
        p = self._params(fitParameters)
        if self._ctx is not None:
            self._ctx.close()
        self._ctx = Context(p, devices=self.devices, n_devices=len(self.devices) if self.devices else 1)
        self._ctx.fit(u, i, r)
        self.factorsOption = self._unblock()
        path = self.parameters.get("TemporaryPath")
        if path:
            self.save(os.path.join(path, "userItem.npz"))
        return self

    def _unblock(self):
        uids, uvec = self._ctx.factors(L.SIDE_USER)
        iids, ivec = self._ctx.factors(L.SIDE_ITEM)
        return ([Factors(int(x), v) for x, v in zip(uids, uvec)],
                [Factors(int(x), v) for x, v in zip(iids, ivec)])

    def _require_fit(self):
        if self._ctx is None or self.factorsOption is None:
            raise RuntimeError("The MatrixFactorization model has not been fitted to data. "
                               "Prior to predicting values, it has to be trained on data.")

    # PredictDataSetOperation (MatrixFactorization.scala:239-274)
    def predict(self, input) -> List[Tuple[int, int, float]]:
        self._require_fit()
        u, i = _pairs(input)
        pred, found = self._ctx.predict(u, i)
        return [(int(a), int(b), float(c)) for a, b, c, f in zip(u, i, pred, found) if f]

    def predict_arrays(self, u, i):
        self._require_fit()
        return self._ctx.predict(u, i)

    def rmse(self, labeled) -> Tuple[float, int]:
        self._require_fit()
        u, i, r = _columns(labeled)
        return self._ctx.rmse(u, i, r)

    # MatrixFactorization.empiricalRisk (:133-192)
    def empiricalRisk(self, labeledData, riskParameters: Optional[dict] = None) -> float:
        if self._ctx is None:
            raise RuntimeError("The ALS model has not been fitted to data. "
                               "Prior to predicting values, it has to be trained on data.")
        lam = (riskParameters or {}).get("Lambda", self.parameters["Lambda"])
        u, i, r = _columns(labeledData)
        return self._ctx.empirical_risk(u, i, r, lam)

    # persistence of the unblocked factors (TemporaryPath, DSGDforMF.scala:291-296,346-349)
    def save(self, path: str) -> None:
        self._require_fit()
        uids, uvec = self._ctx.factors(L.SIDE_USER)
        iids, ivec = self._ctx.factors(L.SIDE_ITEM)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        np.savez(path, user_ids=uids, user_factors=uvec, item_ids=iids, item_factors=ivec,
                 superstep=np.int64(self._ctx.superstep))

    @property
    def context(self) -> Context:
        self._require_fit()
        return self._ctx

    @staticmethod
    def apply(**kw) -> "DSGDforMF":
        return DSGDforMF(**kw)
