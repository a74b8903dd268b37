"""Online micro-batch path on the GPU vs the oracle (SGDUpdater arithmetic, bit-exact in f64)."""
import os

import numpy as np
import pytest

import coracle
import mf_oracle as O
import mfhip
from conftest import set_knob, golden
from mfhip import _lib as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,flavour,P", [("spark_example_online_flink", "flink", 0),
                                            ("spark_example_online_ps", "ps", 0),
                                            ("spark_example_online_spark_p1", "spark", 1),
                                            ("spark_example_online_spark_p2", "spark", 2),
                                            ("spark_example_online_spark_p4", "spark", 4)])
def test_spark_example_batches_bit_exact(name, flavour, P):
    g = golden(name)
    model = mfhip.OnlineMF(int(g["k"]), float(g["lr"]), flavour=flavour, num_partitions=max(P, 1))
    start = 0
    for sz in g["batch_sizes"].tolist():
        sl = slice(start, start + sz)
        model.update((g["u"][sl], g["i"][sl], g["r"][sl]))
        start += sz
    ids, vecs = model.ctx.factors(L.SIDE_USER)
    assert np.array_equal(ids, g["user_ids"]) and np.array_equal(vecs, g["user_factors"])
    ids, vecs = model.ctx.factors(L.SIDE_ITEM)
    assert np.array_equal(ids, g["item_ids"]) and np.array_equal(vecs, g["item_factors"])


def test_large_batch_arrival_order_bit_exact():
    rng = np.random.default_rng(1)
    n, k = 60000, 48
    u = rng.integers(0, 3000, n).astype(np.int32)
    i = (rng.zipf(1.3, n) % 500).astype(np.int32)
    r = rng.integers(1, 6, n).astype(np.float64)
    model = mfhip.OnlineMF(k, 0.005)
    for s in range(0, n, 20000):
        model.update((u[s:s + 20000], i[s:s + 20000], r[s:s + 20000]))
    uids, iids = np.unique(u), np.unique(i)
    U = np.stack([O.pseudo_random_factor(int(x), k) for x in uids])
    I = np.stack([O.pseudo_random_factor(int(x), k) for x in iids])
    coracle.online_apply(np.searchsorted(uids, u), np.searchsorted(iids, i), r, U, I, k, 0.005)
    assert np.array_equal(model.ctx.factors(0)[1], U)
    assert np.array_equal(model.ctx.factors(1)[1], I)


def test_online_on_top_of_offline_model():
    """Combined path: DSGD fit, then online micro-batches on the same GPU-resident model."""
    from mfhip import synth
    d = synth.generate(500, 200, 10000, seed=3)
    p = L.default_params()
    p.num_factors, p.iterations, p.num_blocks, p.online_learning_rate = 8, 2, 2, 0.01
    ctx = mfhip.Context(p)
    ctx.fit(d.u, d.i, d.r)
    uids0, U0 = ctx.factors(0)
    iids0, I0 = ctx.factors(1)
    batch_u = np.array([d.u[0], 10**6, d.u[1]], np.int32)   # one unseen user
    batch_i = np.array([d.i[0], d.i[0], 10**6 + 1], np.int32)  # one unseen item
    batch_r = np.array([4.0, 2.0, 5.0])
    tu, ti = ctx.online_update(batch_u, batch_i, batch_r)
    assert (tu, ti) == (3, 2)
    users = {int(a): v.tolist() for a, v in zip(uids0, U0)}
    items = {int(a): v.tolist() for a, v in zip(iids0, I0)}
    O.online_sequential(list(zip(batch_u.tolist(), batch_i.tolist(), batch_r.tolist())), users, items, 8, 0.01)
    ids, vecs = ctx.factors(0)
    assert np.array_equal(vecs, np.array([users[x] for x in ids.tolist()]))
    ids, vecs = ctx.factors(1)
    assert np.array_equal(vecs, np.array([items[x] for x in ids.tolist()]))
    ctx.close()


@pytest.mark.gpu
def test_combined_offline_online_matches_oracle(tmp_path):
    """OnlineSpark.buildModelCombineOffline (sp/OnlineSpark.scala:26-162): online Spark sweeps per
    micro-batch, a from-scratch offlineDSGD over the whole history every offline_every-th batch;
    bit-exact against the oracle's composition of the same sweeps, snapshots written on schedule."""
    from mfhip import synth
    from mfhip.combined import OnlineOfflineSpark
    d = synth.generate(120, 60, 1800, seed=9)
    batches = [(d.u[x:x + 200], d.i[x:x + 200], d.r[x:x + 200]) for x in range(0, 1800, 200)]
    k, lr, P, every, iters = 6, 0.01, 3, 4, 3
    m = OnlineOfflineSpark(k, lr, num_partitions=P, offline_every=every, checkpoint_every=5, iterations=iters,
                           snapshot_dir=str(tmp_path))
    users, items, hist = {}, {}, []
    for b, (u, i, r) in enumerate(batches, start=1):
        rs = list(zip(u.tolist(), i.tolist(), r.tolist()))
        hist += rs
        uu, iu, offline = m.process(u, i, r)
        assert offline == (b % every == 0)
        if offline:
            users, items = {}, {}
            O.spark_sweep(hist, users, items, k, lr, P, iters)
            assert set(uu) == set(users) and set(iu) == set(items)
        else:
            O.spark_sweep(rs, users, items, k, lr, P, 1)
            assert set(uu) == set(u.tolist()) and set(iu) == set(i.tolist())
        for x, v in uu.items():
            assert np.array_equal(v, np.array(users[x])), (b, "user", x)
        for x, v in iu.items():
            assert np.array_equal(v, np.array(items[x])), (b, "item", x)
    assert sorted(os.listdir(tmp_path)) == ["model_000005.mfsnap"]
    m.close()


@pytest.mark.gpu
def test_ps_offline_online_matches_oracle():
    """PSOfflineOnlineMF.offlineOnlinePS (fl/mf/PSOfflineOnlineMF.scala:28-359), sequential
    serialisation: online delta updates in arrival order; a batch trigger clears the PS item
    vectors, keeps the worker's user vectors and replays the history `iterations` times in
    insertion order.  Bit-exact against the oracle's composition of the same delta updates."""
    from mfhip import synth
    from mfhip.combined import PSOfflineOnlineMF
    d = synth.generate(90, 50, 1500, seed=13)
    k, lr, iters = 5, 0.02, 3
    m = PSOfflineOnlineMF(k, lr, iterations=iters, emit_outputs=True)
    users, items, hist = {}, {}, []
    steps = ["o", "o", "b", "o", "o", "o", "b", "o"]
    x = 0
    for s in steps:
        if s == "o":
            u, i, r = d.u[x:x + 250], d.i[x:x + 250], d.r[x:x + 250]
            x += 250
            rs = list(zip(u.tolist(), i.tolist(), r.tolist()))
            hist += rs
            uu, iu = m.process(u, i, r)
            emitted = []
            O.online_sequential(rs, users, items, k, lr, "delta", emitted=emitted)
            assert set(uu) == set(u.tolist()) and set(iu) == set(i.tolist())
            assert np.array_equal(m.output[0], u)
        else:
            uu, iu = m.batch()
            items = {}
            emitted = []
            for _ in range(iters):
                O.online_sequential(hist, users, items, k, lr, "delta", emitted=emitted)
            assert set(uu) == set(users) and set(iu) == set(items)
        # the worker's per-rating stream, ps.output(user, userVec + deltaItemVec) (:176), bit-exact
        assert np.array_equal(m.output[1], np.array([a for a, _ in emitted])), s
        for a, v in uu.items():
            assert np.array_equal(v, np.array(users[a])), (s, "user", a)
        for a, v in iu.items():
            assert np.array_equal(v, np.array(items[a])), (s, "item", a)
    m.close()


@pytest.mark.parametrize("flavour,name", [(L.ONLINE_NEXT_FACTORS, "next"), (L.ONLINE_DELTA, "delta")])
def test_per_rating_outputs_bit_exact(flavour, name):
    """mf_online_update_out: the records the operators emit per rating -- Flink's ItemOperator
    (user', item') (FlinkOnlineMF.scala:131-135), the PS worker (userVec + deltaItemVec,
    deltaItemVec) (PSOfflineOnlineMF.scala:174-176) -- in arrival order over several dependency
    levels (repeated users and items), bit-exact against the oracle's sequential replay."""
    rng = np.random.default_rng(17)
    n, k, lr = 5000, 24, 0.004
    u = rng.integers(0, 300, n).astype(np.int32)
    i = (rng.zipf(1.4, n) % 120).astype(np.int32)
    r = rng.integers(1, 6, n).astype(np.float64)
    p = L.default_params()
    p.num_factors, p.online_learning_rate = k, lr
    with mfhip.Context(p) as ctx:
        uo, io = ctx.online_update_out(u[:3000], i[:3000], r[:3000], flavour)
        uo2, io2 = ctx.online_update_out(u[3000:], i[3000:], r[3000:], flavour)
        fu, fi = ctx.factors(0), ctx.factors(1)
    users, items, emitted = {}, {}, []
    O.online_sequential(list(zip(u.tolist(), i.tolist(), r.tolist())), users, items, k, lr, name, emitted=emitted)
    assert np.array_equal(np.concatenate([uo, uo2]), np.array([a for a, _ in emitted]))
    assert np.array_equal(np.concatenate([io, io2]), np.array([b for _, b in emitted]))
    assert np.array_equal(fu[1], np.array([users[x] for x in fu[0].tolist()]))
    assert np.array_equal(fi[1], np.array([items[x] for x in fi[0].tolist()]))
    with mfhip.Context(p) as ctx, pytest.raises(mfhip.MFError, match="touched rows"):
        ctx.online_update_out(u[:10], i[:10], r[:10], L.ONLINE_SPARK_SWEEP)


@pytest.mark.parametrize("mode,k", [(L.MODE_FAST_F32, 128), (L.MODE_DETERMINISTIC_F64, 200), (L.MODE_FAST_F32, 40),
                                    (L.MODE_DETERMINISTIC_F64, 128), (L.MODE_DETERMINISTIC_F64, 64),
                                    (L.MODE_DETERMINISTIC_F64, 256)])
def test_online_sweep_equals_level_replay(monkeypatch, mode, k):
    """The one-launch online sweep (the default: per-item waves, heavy items on waves of their own,
    per-user tickets, its wave lists and tickets built on the device by kernels_online.hip) gives the
    factors of the level-by-level replay (MFHIP_TEST online_kernel=level) bit for bit, including a
    hot item, repeated (user, item) pairs and ids first seen in a later batch.  f64 at k = 64 / 128 /
    256 runs on the deterministic split sweep (k_det_sweep_split with nextFactors' update); its
    predecessor k_online_sweep (online_kernel=ticket) is checked as well."""
    rng = np.random.default_rng(7)
    n = 120000
    u = rng.integers(0, 5000, n).astype(np.int32)
    i = (rng.zipf(1.2, n) % 2000).astype(np.int32)
    i[::37] = 3  # a hot item
    r = rng.integers(1, 6, n).astype(np.float64)
    res = {}
    # f32 "multi": every wave on k_online_f32's general path (online_single=0), none on the lean
    # single-item path the heavy items' waves take by default
    kerns = ("level", "sweep", "ticket") if mode == L.MODE_DETERMINISTIC_F64 else ("level", "sweep", "multi")
    for kern in kerns:
        set_knob(monkeypatch, "online_kernel", "sweep" if kern == "multi" else kern)
        set_knob(monkeypatch, "online_single", "0" if kern == "multi" else "1")
        p = L.default_params()
        p.num_factors, p.mode, p.online_learning_rate = k, mode, 0.01
        with mfhip.Context(p) as ctx:
            for s in range(0, n, 40000):
                ctx.online_update(u[s:s + 40000], i[s:s + 40000], r[s:s + 40000], L.ONLINE_NEXT_FACTORS)
            res[kern] = (ctx.factors(0), ctx.factors(1))
    for kern in kerns[1:]:
        for side in (0, 1):
            assert np.array_equal(res["level"][side][0], res[kern][side][0])
            assert np.array_equal(res["level"][side][1], res[kern][side][1])


# (f32, 64): every lane in use, the deferred-ticket instance; (f64, 64): the deterministic split sweep
@pytest.mark.parametrize("mode,k", [(L.MODE_FAST_F32, 32), (L.MODE_FAST_F32, 64), (L.MODE_DETERMINISTIC_F64, 64)])
@pytest.mark.parametrize("shape", ["one", "few", "one_user", "one_item", "spark"])
def test_online_sweep_edge_batches(monkeypatch, shape, mode, k):
    """Edge batches of the device-built sweep plan (kernels_online.hip) against the level replay,
    bit for bit: a single rating, fewer ratings than waves, one user across every wave (a ticket
    chain through all of them), one item (one wave holds the whole batch), and the Spark-sweep
    order (a permuted sequence)."""
    rng = np.random.default_rng(11)
    n = {"one": 1, "few": 37}.get(shape, 30000)
    u = rng.integers(0, 3000, n).astype(np.int32)
    i = rng.integers(0, 900, n).astype(np.int32)
    if shape == "one_user":
        u[:] = 42
    if shape == "one_item":
        i[:] = 7
    r = rng.integers(1, 6, n).astype(np.float64)
    flav = L.ONLINE_SPARK_SWEEP if shape == "spark" else L.ONLINE_NEXT_FACTORS
    res = {}
    for kern in ("level", "sweep"):
        set_knob(monkeypatch, "online_kernel", kern)
        p = L.default_params()
        p.num_factors, p.mode, p.online_learning_rate = k, mode, 0.01
        with mfhip.Context(p) as ctx:
            for s in range(0, n, 10000):
                bu, bi = u[s:s + 10000], i[s:s + 10000]
                if flav == L.ONLINE_SPARK_SWEEP:
                    tu, ti = ctx.online_update(bu, bi, r[s:s + 10000], flav, num_partitions=4)
                else:
                    tu, ti = ctx.online_update(bu, bi, r[s:s + 10000], flav)
                # touched rows (device-counted on the sweep path)
                assert (tu, ti) == (len(np.unique(bu)), len(np.unique(bi)))
            res[kern] = (ctx.factors(0), ctx.factors(1))
    for side in (0, 1):
        assert np.array_equal(res["level"][side][0], res["sweep"][side][0])
        assert np.array_equal(res["level"][side][1], res["sweep"][side][1])


@pytest.mark.parametrize("mode", [L.MODE_FAST_F32, L.MODE_DETERMINISTIC_F64])
def test_device_id_lookup_equals_host_lookup(monkeypatch, mode):
    """The online batch's id -> row lookup on the device (a mirror of each side's IdIndex, kept in
    step with the host table: whole after a rehash, else the slots written since) gives the rows of
    the host lookup (MFHIP_TEST online_lookup=host), bit for bit in the factors and the id lists:
    negative ids, an empty model at the start (every id new), new ids in every later batch (first
    touch order), and enough of them that both tables rehash between batches."""
    rng = np.random.default_rng(23)
    res = {}
    for where in ("host", "device"):
        set_knob(monkeypatch, "online_lookup", where)
        p = L.default_params()
        p.num_factors, p.mode, p.online_learning_rate = 64, mode, 0.01
        rng = np.random.default_rng(23)
        with mfhip.Context(p) as ctx:
            for b in range(6):
                n = 20000
                hi = 500 * 4 ** b  # the id ranges grow: each batch brings new ids, later batches force rehashes
                u = (rng.integers(-hi, hi, n)).astype(np.int32)
                i = (rng.integers(-hi // 4, hi // 4, n)).astype(np.int32)
                r = rng.integers(1, 6, n).astype(np.float64)
                tu, ti = ctx.online_update(u, i, r, L.ONLINE_NEXT_FACTORS)
                assert (tu, ti) == (len(np.unique(u)), len(np.unique(i)))
            res[where] = (ctx.factors(0), ctx.factors(1))
    for side in (0, 1):
        assert np.array_equal(res["host"][side][0], res["device"][side][0])
        assert np.array_equal(res["host"][side][1], res["device"][side][1])
