"""The Python mirror of the reference API (no GPU needed for these checks)."""
import numpy as np
import pytest

import mf_oracle as O
import mfhip
from mfhip import DSGDforMF, LearningRateMethod, SGDUpdater, MockFactorUpdater, PseudoRandomFactorInitializer


def test_fluent_setters_and_params():
    s = (DSGDforMF().setNumFactors(7).setLambda(0.5).setIterations(3).setBlocks(4).setSeed(9)
         .setLearningRate(0.02).setLearningRateMethod(LearningRateMethod.InvScaling(0.5)))
    p = s._params()
    assert (p.num_factors, p.lambda_, p.iterations, p.num_blocks, p.seed, p.has_seed) == (7, 0.5, 3, 4, 9, 1)
    assert p.learning_rate == 0.02 and p.lr_method == 3 and p.lr_arg == 0.5
    p = DSGDforMF().setSeed(None)._params()
    assert p.has_seed == 0 and p.num_blocks == 1


def test_predict_before_fit_raises_runtime_error():
    with pytest.raises(RuntimeError, match="has not been fitted"):
        DSGDforMF().predict([(1, 2)])
    with pytest.raises(RuntimeError):
        DSGDforMF().empiricalRisk([(1, 2, 3.0)])


def test_sgd_updater_matches_reference_arithmetic():
    rng = np.random.default_rng(3)
    for _ in range(20):
        u, i = rng.random(6), rng.random(6)
        r = float(rng.random() * 5)
        nu, ni = SGDUpdater(0.01).nextFactors(r, u, i)
        ou, oi = O.sgd_next_factors(0.01, r, u.tolist(), i.tolist())
        assert nu.tolist() == ou and ni.tolist() == oi
        du, di = SGDUpdater(0.01).delta(r, u, i)
        odu, odi = O.sgd_delta(0.01, r, u.tolist(), i.tolist())
        assert du.tolist() == odu and di.tolist() == odi
    u, i = np.ones(3), np.zeros(3)
    assert MockFactorUpdater().nextFactors(1.0, u, i) == (u, i)


def test_pseudo_random_initializer():
    f = PseudoRandomFactorInitializer(5)
    for id_ in (0, 3, -4, 1000):
        assert f.nextFactor(id_).tolist() == O.pseudo_random_factor(id_, 5)


def test_rating_and_vector_types():
    r = mfhip.Rating.fromTuple((1, 2, 3.5))
    assert (r.user, r.item, r.rating) == (1, 2, 3.5)
    v = mfhip.FactorVector(4, np.array([1.0, 2.0]))
    assert repr(v) == "FactorVector(4, [1.0,2.0])"
