"""The oracle itself: JDK known-answer values, C vs Python restatements, golden fixtures."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import coracle
import mf_oracle as O
from conftest import GOLDEN, golden

# java.util.Random known answers (JDK 8 spec)
KAT = [
    ("nextInt", 42, None, -1170105035),
    ("nextInt", 0, None, -1155484576),
    ("nextDouble", 0, None, 0.730967787376657),
    ("nextDouble", 42, None, 0.7275636800328681),
    ("nextIntBound", 42, 10, 0),
]


@pytest.mark.parametrize("kind,seed,bound,expect", KAT)
def test_jdk_known_answers(kind, seed, bound, expect):
    r = O.JavaRandom(seed)
    if kind == "nextInt":
        assert r.nextInt() == expect
        assert coracle.next_int(seed, 1)[0] == expect
    elif kind == "nextDouble":
        assert r.nextDouble() == expect
        assert coracle.next_double(seed, 1)[0] == expect
    else:
        assert r.nextInt(bound) == expect
        assert coracle.next_int_bound(seed, bound, 1)[0] == expect


def test_rng_sequences_agree():
    for seed in (0, 1, -1, 42, 2**40 + 3, -(2**50)):
        r = O.JavaRandom(seed)
        assert [r.nextInt() for _ in range(50)] == coracle.next_int(seed, 50).tolist()
        for bound in (1, 2, 3, 7, 10, 64, 1000, 2**30 + 1, 2**31 - 1):
            r = O.JavaRandom(seed)
            assert [r.nextInt(bound) for _ in range(40)] == coracle.next_int_bound(seed, bound, 40).tolist()
        r = O.JavaRandom(seed)
        assert [r.nextDouble() for _ in range(30)] == coracle.next_double(seed, 30).tolist()


def test_shuffle_agrees_and_is_permutation():
    for seed in (0, 5, -3, 123456789):
        for n in (0, 1, 2, 3, 17, 1000):
            a = coracle.scala_shuffle(seed, n)
            b = O.scala_shuffle(O.JavaRandom(seed), range(n))
            assert a.tolist() == b
            assert sorted(b) == list(range(n))


def test_block_of_and_init():
    for id_ in (-5, 0, 1, 17, 2**31 - 1, -(2**31)):
        for seed in (0, 42, -1):
            for n in (1, 3, 8):
                assert coracle.block_of(id_, seed, n) == O.block_of(id_, seed, n)


def test_learning_rate_methods():
    for m, arg in ((0, 0.0), (1, 0.0), (2, 3.0), (3, 0.6), (4, 0.75)):
        for t in (1, 2, 10):
            assert coracle.learning_rate(m, 0.01, t, 0.5, arg) == O.learning_rate(m, 0.01, t, 0.5, arg)
    assert O.learning_rate(0, 0.001, 4, 1.0) == 0.001 / 2.0


def test_next_rating_block_rotation():
    # DSGDforMF.nextRatingBlock: user block p visits (p, p+s-1); item block q visits (q-(s-1), q)
    for n in (1, 2, 3, 5, 8):
        cu = {b: b * (n + 1) for b in range(n)}
        ci = dict(cu)
        for s in range(1, 3 * n + 1):
            for p in range(n):
                assert cu[p] == p * n + (p + s - 1) % n
            for q in range(n):
                assert ci[q] == ((q - (s - 1)) % n) * n + q
            cu = {b: O.next_rating_block(v, n)[0] for b, v in cu.items()}
            ci = {b: O.next_rating_block(v, n)[1] for b, v in ci.items()}


@pytest.mark.parametrize("nb,seed", [(1, 0), (2, 3), (3, -9), (5, 2**33)])
def test_c_oracle_equals_python_oracle(nb, seed):
    rnd = random.Random(nb * 31 + 1)
    R = [(rnd.randrange(-20, 60), rnd.randrange(35), rnd.random() * 5) for _ in range(700)]
    us, it = O.dsgd_fit(R, k=6, iterations=3, n_blocks=nb, seed=seed, lam=0.7, lr=0.01)
    m = coracle.dsgd_fit([a for a, _, _ in R], [b for _, b, _ in R], [c for _, _, c in R], k=6, iterations=3,
                         n_blocks=nb, seed=seed, lam=0.7, lr=0.01, threads=3)
    for side, ref in ((0, us), (1, it)):
        ids, vecs = m.factors(side)
        assert sorted(ref) == ids.tolist()
        assert np.array_equal(np.array([ref[x] for x in ids.tolist()]), vecs)


def test_golden_manifest():
    man = json.load(open(os.path.join(GOLDEN, "MANIFEST.json")))
    assert len(man) >= 11
    for name, sha in man.items():
        assert hashlib.sha256(open(os.path.join(GOLDEN, name), "rb").read()).hexdigest() == sha, name


@pytest.mark.parametrize("name", ["spark_example_dsgd_n1", "spark_example_dsgd_n2", "spark_example_dsgd_n3",
                                  "synthetic1k_dsgd_n3", "synthetic1k_dsgd_n4_seed_neg", "ml100k_like_dsgd_n4"])
def test_c_oracle_reproduces_golden(name):
    g = golden(name)
    m = coracle.dsgd_fit(g["u"], g["i"], g["r"], k=int(g["k"]), iterations=int(g["iterations"]),
                         n_blocks=int(g["n_blocks"]), seed=int(g["seed"]), lam=float(g["lam"]), lr=float(g["lr"]),
                         threads=2)
    ids, vecs = m.factors(0)
    assert np.array_equal(ids, g["user_ids"]) and np.array_equal(vecs, g["user_factors"])
    ids, vecs = m.factors(1)
    assert np.array_equal(ids, g["item_ids"]) and np.array_equal(vecs, g["item_factors"])
    if "test_u" in g:
        pred, found = m.predict(g["pred_u"], g["pred_i"])
        assert found.all() and np.array_equal(pred, g["pred"])


@pytest.mark.parametrize("name,flavour", [("spark_example_online_flink", "next"), ("spark_example_online_ps", "delta")])
def test_online_golden_restatements(name, flavour):
    """C online_apply (arrival order) == Python oracle, including PseudoRandom first-touch init."""
    g = golden(name)
    k, lr = int(g["k"]), float(g["lr"])
    uids = sorted(set(g["u"].tolist()))
    iids = sorted(set(g["i"].tolist()))
    U = np.array([O.pseudo_random_factor(x, k) for x in uids])
    I = np.array([O.pseudo_random_factor(x, k) for x in iids])
    urow = np.searchsorted(uids, g["u"])
    irow = np.searchsorted(iids, g["i"])
    coracle.online_apply(urow, irow, g["r"], U, I, k, lr)
    assert np.array_equal(U, g["user_factors"]) and np.array_equal(I, g["item_factors"])
