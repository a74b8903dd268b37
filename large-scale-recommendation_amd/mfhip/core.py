"""Mirror of the reference's `core` types and updaters (core/src/main/scala/hu/sztaki/ilab/recom/core).

The scalar classes keep the reference's pure per-rating API (used by callers that want
the Scala semantics on single vectors); batches of ratings go to the GPU through
mfhip.online.OnlineMF, which applies the same arithmetic as hand-written HIP kernels.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import jvm

UserId = int
ItemId = int


@dataclass(frozen=True)
class Rating:
    """core/package.scala:15-19."""
    user: UserId
    item: ItemId
    rating: float

    @staticmethod
    def fromTuple(t: Tuple[int, int, float]) -> "Rating":
        return Rating(int(t[0]), int(t[1]), float(t[2]))


@dataclass
class FactorVector:
    """core/package.scala:21-23 (also MatrixFactorization.Factors, :232-234)."""
    id: int
    vector: np.ndarray

    def __repr__(self) -> str:
        return f"FactorVector({self.id}, [{','.join(repr(float(x)) for x in self.vector)}])"


Factors = FactorVector


@dataclass
class UserUpdate:
    vec: FactorVector


@dataclass
class ItemUpdate:
    vec: FactorVector


class FactorUpdater:
    """core/FactorUpdater.scala:3-19."""

    def nextFactors(self, rating: float, user, item):
        raise NotImplementedError

    def delta(self, rating: float, user, item):
        raise NotImplementedError


class MockFactorUpdater(FactorUpdater):
    """core/FactorUpdater.scala:21-33: identity."""

    def nextFactors(self, rating, user, item):
        return user, item

    def delta(self, rating, user, item):
        return user, item


class SGDUpdater(FactorUpdater):
    """core/FactorUpdater.scala:35-54: plain SGD, no regularisation."""

    def __init__(self, learningRate: float):
        self.learningRate = float(learningRate)

    @staticmethod
    def _err(rating, user, item) -> float:
        s = 0.0
        for x, y in zip(user, item):  # zip.map(x*y).sum: left fold from 0.0
            s = s + float(x) * float(y)
        return float(rating) - s

    def nextFactors(self, rating, user, item):
        e = self._err(rating, user, item)
        le = self.learningRate * e
        u = np.asarray(user, np.float64)
        i = np.asarray(item, np.float64)
        return u + le * i, i + le * u

    def delta(self, rating, user, item):
        e = self._err(rating, user, item)
        le = self.learningRate * e
        return le * np.asarray(item, np.float64), le * np.asarray(user, np.float64)


class FactorInitializer:
    """core/FactorInitializer.scala:5-7."""

    def nextFactor(self, id_: int) -> np.ndarray:
        raise NotImplementedError


class PseudoRandomFactorInitializer(FactorInitializer):
    """core/FactorInitializer.scala:23-27: new Random(id), numFactors x nextDouble."""

    def __init__(self, numFactors: int):
        self.numFactors = int(numFactors)

    def nextFactor(self, id_: int) -> np.ndarray:
        return jvm.random_factors(int(id_), self.numFactors)


class RandomFactorInitializer(FactorInitializer):
    """core/FactorInitializer.scala:17-21: a shared generator (not reproducible across runs)."""

    def __init__(self, numFactors: int, seed: int | None = None):
        self.numFactors = int(numFactors)
        self._rng = np.random.default_rng(seed)

    def nextFactor(self, id_: int) -> np.ndarray:
        return self._rng.random(self.numFactors)


class FactorInitializerDescriptor:
    """core/FactorInitializer.scala:9-21."""

    def __init__(self, factory):
        self._factory = factory

    def open(self) -> FactorInitializer:
        return self._factory()

    @staticmethod
    def apply(init) -> "FactorInitializerDescriptor":
        class _F(FactorInitializer):
            def nextFactor(self, id_):
                return np.asarray(init(id_), np.float64)
        return FactorInitializerDescriptor(_F)


def PseudoRandomFactorInitializerDescriptor(numFactors: int) -> FactorInitializerDescriptor:
    d = FactorInitializerDescriptor(lambda: PseudoRandomFactorInitializer(numFactors))
    d.numFactors = numFactors
    d.kind = "pseudo_random"
    return d


def RandomFactorInitializerDescriptor(numFactors: int) -> FactorInitializerDescriptor:
    d = FactorInitializerDescriptor(lambda: RandomFactorInitializer(numFactors))
    d.numFactors = numFactors
    d.kind = "random"
    return d
