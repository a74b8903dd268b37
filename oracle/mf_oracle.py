"""oracle/mf_oracle.py -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's DSGD and online-MF hot path.  It is the
independent second restatement that the C oracle (oracle/mf_oracle.c) is checked
against, and the generator of the committed golden fixtures under tests/golden/.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it;
the product (large-scale-recommendation_amd/) never does.

Parity pinning: the reference has no tests or fixtures and cannot run here (Scala,
no JVM).  The JVM RNG / Scala shuffle are pinned by JDK known-answer values; the
algorithm itself is unpinned beyond those (see DESIGN.md "Oracle").

All arithmetic is IEEE double in the JVM's evaluation order (Python floats are
binary64 and never fused), so results are bit-exact restatements.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

MASK48 = (1 << 48) - 1
MULT = 0x5DEECE66D


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def _i64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x & (1 << 63) else x


class JavaRandom:
    """java.util.Random (JDK 8 spec); scala.util.Random(seed) delegates to it."""

    def __init__(self, seed: int):
        self.seed = (_i64(seed) ^ MULT) & MASK48

    def next(self, bits: int) -> int:
        self.seed = (self.seed * MULT + 0xB) & MASK48
        return _i32(self.seed >> (48 - bits))

    def nextInt(self, bound: int | None = None) -> int:
        if bound is None:
            return self.next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        r = self.next(31)
        m = bound - 1
        if (bound & m) == 0:
            return _i32((bound * r) >> 31)
        u = r
        while True:
            r = u % bound  # u >= 0, so Python % == Java %
            if _i32(u - r + m) >= 0:
                return r
            u = self.next(31)

    def nextDouble(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))


def scala_shuffle(rng: JavaRandom, xs: Sequence) -> list:
    """scala.util.Random.shuffle, Scala 2.11: for n <- len to 2 by -1 {k = nextInt(n); swap(n-1, k)}."""
    buf = list(xs)
    for n in range(len(buf), 1, -1):
        k = rng.nextInt(n)
        buf[n - 1], buf[k] = buf[k], buf[n - 1]
    return buf


# ---------------------------------------------------------------------------
# flink-ml 1.3.0 LearningRateMethod (DSGDforMF.scala:10,383-386), restated.
# ---------------------------------------------------------------------------
LR_DEFAULT, LR_CONSTANT, LR_BOTTOU, LR_INVSCALING, LR_XU = range(5)


def learning_rate(method: int, lr: float, iteration: int, lam: float, arg: float = 0.0) -> float:
    if method == LR_CONSTANT:
        return lr
    if method == LR_BOTTOU:
        return 1.0 / (lam * (arg + iteration - 1))
    if method == LR_INVSCALING:
        return lr / math.pow(iteration, arg)
    if method == LR_XU:
        return lr * math.pow(1.0 + lam * lr * iteration, -arg)
    return lr / math.sqrt(iteration)


def ddot(x: Sequence[float], y: Sequence[float]) -> float:
    """netlib-java F2jBLAS.ddot: sequential left fold from 0.0."""
    acc = 0.0
    for a, b in zip(x, y):
        acc = acc + a * b
    return acc


def random_factors(k: int, rng: JavaRandom) -> List[float]:
    """MatrixFactorization.randomFactors (:278-280)."""
    return [rng.nextDouble() for _ in range(k)]


def block_of(id_: int, seed: int, n_blocks: int) -> int:
    """DSGDforMF.scala:531-533."""
    return JavaRandom(id_ ^ seed).nextInt(n_blocks)


def next_rating_block(current: int, n: int) -> Tuple[int, int]:
    """DSGDforMF.nextRatingBlock (:611-619)."""
    p_row = current // n
    q_row = current % n
    new_p = p_row * n + (current + 1) % n
    new_q = ((p_row + n - 1) % n) * n + q_row
    return new_p, new_q


def dsgd_update(p: List[float], q: List[float], r: float, eta: float, lam: float,
                omega_u: int, omega_i: int) -> Tuple[List[float], List[float]]:
    """The per-rating body of updateLocalFactors (DSGDforMF.scala:395-414)."""
    e = r - ddot(p, q)
    reg_u = lam / omega_u
    reg_i = lam / omega_i
    new_p = [pf - eta * (reg_u * pf - e * qf) for pf, qf in zip(p, q)]
    new_q = [qf - eta * (reg_i * qf - e * pf) for pf, qf in zip(p, q)]
    return new_p, new_q


def update_local_factors(ratings: Sequence[Tuple[float, int, int]], users: List[List[float]],
                         user_omegas: Sequence[int], items: List[List[float]],
                         item_omegas: Sequence[int], iteration: int, rating_block_id: int,
                         seed: int, lr: float, lr_method: int, lam: float, lr_arg: float = 0.0) -> None:
    """updateLocalFactors (DSGDforMF.scala:378-418); mutates users/items in place."""
    eta = learning_rate(lr_method, lr, iteration + 1, lam, lr_arg)
    order = scala_shuffle(JavaRandom((iteration ^ rating_block_id) ^ seed), range(len(ratings)))
    for x in order:
        rating, uidx, iidx = ratings[x]
        users[uidx], items[iidx] = dsgd_update(users[uidx], items[iidx], rating, eta, lam,
                                               user_omegas[uidx], item_omegas[iidx])


def dsgd_fit(ratings: Sequence[Tuple[int, int, float]], k: int = 10, iterations: int = 10,
             lam: float = 1.0, lr: float = 0.001, lr_method: int = LR_DEFAULT, lr_arg: float = 0.0,
             n_blocks: int = 1, seed: int = 0, max_supersteps: int | None = None
             ) -> Tuple[Dict[int, List[float]], Dict[int, List[float]]]:
    """DSGDforMF.fitSGD (:262-357) with a seed (deterministic mode). Returns (users, items)."""
    def init_side(ids: Sequence[int]):
        counts: Dict[int, int] = {}
        for x in ids:
            counts[x] = counts.get(x, 0) + 1
        blocks: Dict[int, List[int]] = {b: [] for b in range(n_blocks)}
        for x in sorted(counts):
            blocks[block_of(x, seed, n_blocks)].append(x)  # ids sorted within a block (:556)
        fac, omg, where = {}, {}, {}
        for b, ids_b in blocks.items():
            fac[b] = [random_factors(k, JavaRandom(x ^ seed)) for x in ids_b]  # :548-549
            omg[b] = [counts[x] for x in ids_b]
            for idx, x in enumerate(ids_b):
                where[x] = (b, idx)
        return blocks, fac, omg, where

    ublocks, ufac, uomg, uwhere = init_side([u for u, _, _ in ratings])
    iblocks, ifac, iomg, iwhere = init_side([i for _, i, _ in ratings])

    rblocks: Dict[int, list] = {}
    for pos, (u, i, r) in enumerate(ratings):
        ub, uidx = uwhere[u]
        ib, iidx = iwhere[i]
        rblocks.setdefault(ub * n_blocks + ib, []).append(((u, i, pos), (r, uidx, iidx)))
    for b in rblocks:  # sortBy((u,i)) when seeded (:319-323); stable => input order for ties
        rblocks[b].sort(key=lambda t: t[0])
        rblocks[b] = [t[1] for t in rblocks[b]]

    # Factor blocks travel with currentRatingBlock (initial b*(n+1), :562) and move with
    # nextRatingBlock; the coGroup matches them to the rating block of the same id (:448-450).
    cur_user = {b: b * (n_blocks + 1) for b in range(n_blocks)}
    cur_item = {b: b * (n_blocks + 1) for b in range(n_blocks)}
    total = iterations * n_blocks
    if max_supersteps is not None:
        total = min(total, max_supersteps)
    for superstep in range(1, total + 1):
        iteration = superstep // n_blocks  # getSuperstepNumber / numBlocks (:476)
        by_rb: Dict[int, list] = {}
        for b, rb in cur_user.items():
            by_rb.setdefault(rb, [None, None])[0] = b
        for b, rb in cur_item.items():
            by_rb.setdefault(rb, [None, None])[1] = b
        for rb, (ub, ib) in sorted(by_rb.items()):
            if rb in rblocks:
                update_local_factors(rblocks[rb], ufac[ub], uomg[ub], ifac[ib], iomg[ib],
                                     iteration, rb, seed, lr, lr_method, lam, lr_arg)
        for b in cur_user:
            cur_user[b] = next_rating_block(cur_user[b], n_blocks)[0]
        for b in cur_item:
            cur_item[b] = next_rating_block(cur_item[b], n_blocks)[1]

    users = {x: ufac[b][idx] for x, (b, idx) in uwhere.items()}  # unblock (:245-255)
    items = {x: ifac[b][idx] for x, (b, idx) in iwhere.items()}
    return users, items


def predict(users: Dict[int, List[float]], items: Dict[int, List[float]],
            pairs: Sequence[Tuple[int, int]]) -> List[Tuple[int, int, float]]:
    """predictRating (MatrixFactorization.scala:239-274): inner join on both ids, then ddot."""
    return [(u, i, ddot(users[u], items[i])) for u, i in pairs if u in users and i in items]


def rmse(users, items, labeled: Sequence[Tuple[int, int, float]]) -> Tuple[float, int]:
    """RMSE over the inner-joined labeled pairs (predictRating semantics; the reference has no RMSE)."""
    sse, cnt = 0.0, 0
    for u, i, r in labeled:
        if u in users and i in items:
            d = r - ddot(users[u], items[i])
            sse += d * d
            cnt += 1
    return (math.sqrt(sse / cnt) if cnt else float("nan")), cnt


def empirical_risk(users, items, labeled: Sequence[Tuple[int, int, float]], lam: float) -> float:
    """MatrixFactorization.empiricalRisk (:133-192).  The second join on (u,i) pairs every labeled
    row with every prediction of the same pair, so a pair occurring m times counts m times per row."""
    mult: Dict[Tuple[int, int], int] = {}
    for u, i, _ in labeled:
        mult[(u, i)] = mult.get((u, i), 0) + 1
    total = 0.0
    for u, i, r in labeled:
        if u in users and i in items:
            p, q = users[u], items[i]
            res = r - ddot(p, q)
            term = res * res + lam * (ddot(p, p) + ddot(q, q))
            for _ in range(mult[(u, i)]):
                total += term
    return total


# ---------------------------------------------------------------------------
# Online MF (core/FactorUpdater.scala, core/FactorInitializer.scala)
# ---------------------------------------------------------------------------
def pseudo_random_factor(id_: int, k: int) -> List[float]:
    """PseudoRandomFactorInitializer.nextFactor (core/FactorInitializer.scala:23-27): new Random(id)."""
    rng = JavaRandom(id_)
    return [rng.nextDouble() for _ in range(k)]


def sgd_next_factors(lr: float, rating: float, user: List[float], item: List[float]):
    """SGDUpdater.nextFactors (core/FactorUpdater.scala:37-45)."""
    s = 0.0
    for x, y in zip(user, item):
        s = s + x * y
    e = rating - s
    return ([u + lr * e * i for u, i in zip(user, item)],
            [i + lr * e * u for u, i in zip(user, item)])


def sgd_delta(lr: float, rating: float, user: List[float], item: List[float]):
    """SGDUpdater.delta (core/FactorUpdater.scala:47-53)."""
    s = 0.0
    for x, y in zip(user, item):
        s = s + x * y
    e = rating - s
    return [lr * e * i for i in item], [lr * e * u for u in user]


def online_sequential(ratings: Sequence[Tuple[int, int, float]], users: Dict[int, List[float]],
                      items: Dict[int, List[float]], k: int, lr: float, flavour: str = "next",
                      init=pseudo_random_factor, emitted: list | None = None) -> Tuple[List[int], List[int]]:
    """FlinkOnlineMF (fl/mf/online/FlinkOnlineMF.scala:52-137) under synchronous feedback: ratings
    applied in arrival order, each user FIFO (LockableStateWithQueue), first touch initialises.
    flavour "delta" is the PS path (PSOfflineOnlineMF.scala:167-180): vec + delta.
    emitted (optional list): per rating, the pair of vectors the operator emits --
    "next": (nextUserVector, nextItemVector), ItemOperator's out.collect (FlinkOnlineMF.scala:131-135);
    "delta": (userVec + deltaItemVec, deltaItemVec), the worker's ps.output (:176) with userVec the
    vector before this rating's update, and the vector pushed to the PS (:174).
    Returns the user / item ids touched, in first-touch order."""
    tu, ti = [], []
    for u, i, r in ratings:
        if u not in users:
            users[u] = init(u, k)
        if i not in items:
            items[i] = init(i, k)
        if flavour == "delta":
            du, di = sgd_delta(lr, r, users[u], items[i])
            if emitted is not None:
                emitted.append(([a + b for a, b in zip(users[u], di)], list(di)))
            users[u] = [a + b for a, b in zip(users[u], du)]
            items[i] = [a + b for a, b in zip(items[i], di)]
        else:
            users[u], items[i] = sgd_next_factors(lr, r, users[u], items[i])
            if emitted is not None:
                emitted.append((list(users[u]), list(items[i])))
        if u not in tu:
            tu.append(u)
        if i not in ti:
            ti.append(i)
    return tu, ti


def spark_sweep_order(ratings: Sequence[Tuple[int, int, float]], num_partitions: int,
                      iterations: int = 1) -> List[int]:
    """Sequential order of OfflineSpark.offlineDSGDWithCustomMap (sp/OfflineSpark.scala:115-207):
    users hash-partitioned (id % P), items in rating blocks abs(i) % P; in sub-epoch s (1-based)
    partition p holds item block (p - (s-1)) mod P; each cell is swept in insertion order."""
    P = num_partitions
    cells: Dict[Tuple[int, int], List[int]] = {}
    for pos, (u, i, _) in enumerate(ratings):
        cells.setdefault((u % P, abs(i) % P), []).append(pos)
    order: List[int] = []
    for _ in range(iterations):
        for s in range(1, P + 1):
            for p in range(P):
                order.extend(cells.get((p, (p - (s - 1)) % P), []))
    return order


def spark_sweep(ratings, users, items, k: int, lr: float, num_partitions: int, iterations: int = 1,
                init=pseudo_random_factor):
    """OfflineSpark.offlineDSGDUpdatesOnly on one micro-batch (OnlineSpark.scala:191-194)."""
    order = spark_sweep_order(ratings, num_partitions, iterations)
    return online_sequential([ratings[j] for j in order], users, items, k, lr, "next", init)
