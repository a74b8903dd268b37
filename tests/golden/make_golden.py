"""Generates the golden fixtures under tests/golden/ from the pure-Python oracle.

TEST INFRASTRUCTURE ONLY.  The reference (Scala 2.11 on Flink/Spark) cannot run in this
container (no JVM), so the fixtures come from oracle/mf_oracle.py, the restatement of the
cited reference lines; its RNG is pinned by JDK known-answer values (tests/test_oracle.py).
Inputs:
  * SparkExample.data (sp/SparkExample.scala:54-104), the reference's only data fixture,
    restated as numbers below;
  * a seeded 1k-rating synthetic;
  * a MovieLens-100K-shaped synthetic (943 x 1682 x 100k, k=10, 10 iterations, n=4).
Run:  python tests/golden/make_golden.py   (writes *.npz and MANIFEST.json with sha256)
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mf_oracle as O  # noqa: E402

# sp/SparkExample.scala:54-104 (user, item, rating)
SPARK_EXAMPLE = [
    (2, 13, 534.3937734561154), (6, 14, 509.63176469621936), (4, 14, 515.8246770897443),
    (7, 3, 495.05234565105), (2, 3, 532.3281786219485), (5, 3, 497.1906356844367),
    (3, 3, 512.0640508585093), (10, 3, 500.2906742233019), (1, 4, 521.9189079662882),
    (2, 4, 515.0734651491396), (1, 7, 522.7532725967008), (8, 4, 492.65683825096403),
    (4, 8, 492.65683825096403), (10, 8, 507.03319667905413), (7, 1, 522.7532725967008),
    (1, 1, 572.2230209271174), (2, 1, 563.5849190220224), (6, 1, 518.4844061038742),
    (9, 1, 529.2443732217674), (8, 1, 543.3202505434103), (7, 2, 516.0188923307859),
    (1, 2, 563.5849190220224), (1, 11, 515.1023793011227), (8, 2, 536.8571133978352),
    (2, 11, 507.90776961762225), (3, 2, 532.3281786219485), (5, 11, 476.24185144363304),
    (4, 2, 515.0734651491396), (4, 11, 469.92049343738233), (3, 12, 509.4713776280098),
    (4, 12, 494.6533165132021), (7, 5, 482.2907867916308), (6, 5, 477.5940040923741),
    (4, 5, 480.9040684364228), (1, 6, 518.4844061038742), (6, 6, 470.6605085832807),
    (8, 6, 489.6360564705307), (4, 6, 472.74052954447046), (7, 9, 482.5837650471611),
    (5, 9, 487.00175463269863), (9, 9, 500.69514584780944), (4, 9, 477.71644808419325),
    (7, 10, 485.3852917539852), (8, 10, 507.03319667905413), (3, 10, 500.2906742233019),
    (5, 15, 488.08215944254437), (6, 15, 480.16929757607346),
]


def arrays(ratings):
    return (np.array([t[0] for t in ratings], np.int32), np.array([t[1] for t in ratings], np.int32),
            np.array([t[2] for t in ratings], np.float64))


def pack(d):
    return (np.array(sorted(d), np.int32), np.array([d[x] for x in sorted(d)], np.float64))


def dsgd_case(name, ratings, k, iterations, n_blocks, seed, lam=1.0, lr=0.001, test=None):
    users, items = O.dsgd_fit(ratings, k=k, iterations=iterations, lam=lam, lr=lr, n_blocks=n_blocks, seed=seed)
    u, i, r = arrays(ratings)
    uid, uf = pack(users)
    iid, itf = pack(items)
    out = dict(u=u, i=i, r=r, k=k, iterations=iterations, n_blocks=n_blocks, seed=seed, lam=lam, lr=lr,
               user_ids=uid, user_factors=uf, item_ids=iid, item_factors=itf)
    if test is not None:
        tu, ti, tr = arrays(test)
        pred = O.predict(users, items, list(zip(tu.tolist(), ti.tolist())))
        rm, cnt = O.rmse(users, items, test)
        out.update(test_u=tu, test_i=ti, test_r=tr, test_rmse=rm, test_matched=cnt,
                   pred_u=np.array([p[0] for p in pred], np.int32), pred_i=np.array([p[1] for p in pred], np.int32),
                   pred=np.array([p[2] for p in pred], np.float64),
                   risk=O.empirical_risk(users, items, test, lam))
    return name, out


def online_case(name, batches, k, lr, flavour, P=0):
    users, items = {}, {}
    for b in batches:
        if flavour == "spark":
            O.spark_sweep(b, users, items, k, lr, P)
        else:
            O.online_sequential(b, users, items, k, lr, "delta" if flavour == "ps" else "next")
    uid, uf = pack(users)
    iid, itf = pack(items)
    sizes = np.array([len(b) for b in batches], np.int64)
    u, i, r = arrays([t for b in batches for t in b])
    return name, dict(u=u, i=i, r=r, batch_sizes=sizes, k=k, lr=lr, partitions=P, user_ids=uid,
                      user_factors=uf, item_ids=iid, item_factors=itf)


def ml100k_like(seed=5):
    rng = np.random.default_rng(seed)
    nu, ni, n = 943, 1682, 100_000
    wu = (np.arange(nu) + 1.0 + 50) ** -0.8
    wi = (np.arange(ni) + 1.0 + 20) ** -1.0
    u = rng.choice(nu, n, p=wu / wu.sum())
    i = rng.choice(ni, n, p=wi / wi.sum())
    x = rng.normal(0, 0.5, (nu, 8))
    y = rng.normal(0, 0.5, (ni, 8))
    r = np.clip(np.rint(3.6 + np.sum(x[u] * y[i], 1) + rng.normal(0, 0.5, n)), 1, 5)
    test = rng.random(n) < 0.1
    tr = [(int(a), int(b), float(c)) for a, b, c, t in zip(u, i, r, test) if not t]
    te = [(int(a), int(b), float(c)) for a, b, c, t in zip(u, i, r, test) if t]
    return tr, te


def main(only=None):
    cases = []
    for nb in (1, 2, 3):
        cases.append(dsgd_case(f"spark_example_dsgd_n{nb}", SPARK_EXAMPLE, k=4, iterations=10, n_blocks=nb, seed=0,
                               test=SPARK_EXAMPLE[:10] + [(99, 1, 3.0), (1, 99, 2.0)]))
    rnd = random.Random(1)
    syn = [(rnd.randrange(60), rnd.randrange(40), float(rnd.randrange(1, 6))) for _ in range(1000)]
    syn += syn[:5]  # duplicates are rated independently
    cases.append(dsgd_case("synthetic1k_dsgd_n3", syn, k=8, iterations=5, n_blocks=3, seed=42, test=syn[:100]))
    cases.append(dsgd_case("synthetic1k_dsgd_n4_seed_neg", [(a - 30, b - 20, c) for a, b, c in syn], k=5,
                           iterations=3, n_blocks=4, seed=-7))
    batches = [SPARK_EXAMPLE[:20], SPARK_EXAMPLE[20:30], SPARK_EXAMPLE[30:]]  # SparkExample.scala:21-23
    cases.append(online_case("spark_example_online_flink", batches, 4, 0.01, "flink"))
    cases.append(online_case("spark_example_online_ps", batches, 4, 0.01, "ps"))
    for P in (1, 2, 4):
        cases.append(online_case(f"spark_example_online_spark_p{P}", batches, 4, 0.01, "spark", P))
    if only is None or "ml100k" in only:
        tr, te = ml100k_like()
        cases.append(dsgd_case("ml100k_like_dsgd_n4", tr, k=10, iterations=10, n_blocks=4, seed=0, test=te))
    manifest_path = os.path.join(HERE, "MANIFEST.json")
    manifest = json.load(open(manifest_path)) if os.path.exists(manifest_path) else {}
    for name, d in cases:
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        manifest[name + ".npz"] = hashlib.sha256(open(path, "rb").read()).hexdigest()
        print("wrote", name)
    json.dump(manifest, open(manifest_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
