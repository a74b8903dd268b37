"""Host-side schedules (no GPU): dependency levels and the fast-mode rotation plan."""
import numpy as np
import pytest

import coracle
import mfhip
from mfhip import _lib as L
from mfhip import synth
import ctypes as C


def levels(u, i, order=None):
    u = np.ascontiguousarray(u, np.uint32)
    i = np.ascontiguousarray(i, np.uint32)
    out = np.empty(max(len(u), 1), np.int32)
    o = None if order is None else L.ptr(np.ascontiguousarray(order, np.int32), C.c_int32)
    L.check(L.lib().mf_debug_levels(u.ctypes.data_as(C.POINTER(C.c_uint32)), i.ctypes.data_as(C.POINTER(C.c_uint32)),
                                    o, len(u), L.ptr(out, C.c_int32)))
    return out[:len(u)]


def test_levels_are_conflict_free_and_replay_sequential_order():
    rng = np.random.default_rng(0)
    nu, ni, n, k = 40, 25, 3000, 5
    u = rng.integers(0, nu, n).astype(np.int32)
    i = (rng.zipf(1.6, n) % ni).astype(np.int32)
    r = rng.random(n) * 5
    order = coracle.scala_shuffle(77, n)
    lv = levels(u, i, order)
    uo, io, ro = u[order], i[order], r[order]
    for l in np.unique(lv):  # no two updates of a level share a row
        m = lv == l
        assert len(set(uo[m].tolist())) == m.sum() and len(set(io[m].tolist())) == m.sum()
    # replaying level by level (stable inside a level) == the sequential order, bit for bit
    U0 = rng.random((nu, k)); I0 = rng.random((ni, k))
    ru = np.full(nu, 0.1); ri = np.full(ni, 0.2)
    A_u, A_i = U0.copy(), I0.copy()
    coracle.dsgd_apply(uo, io, ro, A_u, A_i, ru, ri, k, 0.01)
    perm = np.argsort(lv, kind="stable")
    B_u, B_i = U0.copy(), I0.copy()
    coracle.dsgd_apply(uo[perm], io[perm], ro[perm], B_u, B_i, ru, ri, k, 0.01)
    assert np.array_equal(A_u, B_u) and np.array_equal(A_i, B_i)


def test_level_count_is_longest_row_chain_lower_bound():
    u = np.zeros(50, np.int32)            # one hot user: a pure chain
    i = np.arange(50, dtype=np.int32)
    assert levels(u, i).max() == 50
    assert levels(np.arange(50), np.arange(50)).max() == 1


def fast_plan_window(k):
    w = C.c_int32(0)
    L.check(L.lib().mf_fast_plan_window(k, C.byref(w)))
    return w.value


def fast_schedule(u, i, nb, seed, G, blocking=L.BLOCKING_REFERENCE, window=0, k=128):
    n = len(u)
    b = np.empty(n, np.int32); t = np.empty(n, np.int32); g = np.empty(n, np.int32); p = np.empty(n, np.int64)
    L.check(L.lib().mf_debug_fast_schedule(L.ptr(L.as_i32(u), C.c_int32), L.ptr(L.as_i32(i), C.c_int32), n, nb,
                                           seed, G, blocking, window, k, L.ptr(b, C.c_int32), L.ptr(t, C.c_int32), L.ptr(g, C.c_int32),
                                           L.ptr(p, C.c_int64)))
    return b, t, g, p


def fast_schedule_split(u, i, nb, seed, G, item_split, blocking=L.BLOCKING_REFERENCE, window=0, k=128):
    """fast_schedule plus the hot-item replica each rating updates (0 = the item's own row)."""
    n = len(u)
    b = np.empty(n, np.int32); t = np.empty(n, np.int32); g = np.empty(n, np.int32); p = np.empty(n, np.int64)
    r = np.empty(n, np.int32)
    L.check(L.lib().mf_debug_fast_split(L.ptr(L.as_i32(u), C.c_int32), L.ptr(L.as_i32(i), C.c_int32), n, nb,
                                        seed, G, blocking, window, k, item_split, L.ptr(b, C.c_int32),
                                        L.ptr(t, C.c_int32), L.ptr(g, C.c_int32), L.ptr(p, C.c_int64),
                                        L.ptr(r, C.c_int32)))
    return b, t, g, p, r


@pytest.mark.parametrize("nb,G,split", [(1, 8, 50), (2, 8, 30), (3, -64, 40), (2, 16, 7)])
def test_hot_item_replicas_split_and_stay_conflict_free(nb, G, split):
    """MFHIP_ITEM_SPLIT (experiment): an item with m > split ratings in a rating block is swept as
    R = ceil(m / split) chains of at most `split` ratings (round-robin), each chain its own
    physical row, and within a (stratum, sub-step) no physical row appears in two cells."""
    d = synth.generate(500, 200, 20000, seed=2)
    b, t, g, p, rep = fast_schedule_split(d.u, d.i, nb, 3, G, split)
    b0, t0, g0, p0 = fast_schedule(d.u, d.i, nb, 3, G)
    assert np.array_equal(b, b0)  # the blocking does not change
    assert rep.max() > 0  # some item was split
    for x in np.unique(b):
        m = b == x
        items, cnt = np.unique(d.i[m], return_counts=True)
        for it, c in zip(items.tolist(), cnt.tolist()):
            rr = rep[m & (d.i == it)]
            R = -(-c // split) if c > split else 1
            assert rr.max() == R - 1 and rr.min() == 0
            assert np.bincount(rr, minlength=R).max() <= split
    Gmax = int(g.max()) + 1
    for s in range(nb):
        in_stratum = ((b // nb + s) % nb) == (b % nb)
        for tt in np.unique(t[in_stratum]):
            m = in_stratum & (t == tt)
            cell = b[m].astype(np.int64) * Gmax + g[m]
            phys_item = d.i[m].astype(np.int64) * 4096 + rep[m]
            for ids in (d.u[m].astype(np.int64), phys_item):
                owner = {}
                for x, c in zip(ids.tolist(), cell.tolist()):
                    assert owner.setdefault(x, c) == c


@pytest.mark.parametrize("nb,G,window", [(1, 4, 0), (3, 8, 0), (4, 16, 0), (3, 8, 32), (2, 4, 16), (3, -64, 14),
                                         (2, -16, 14), (2, -16, 14 | (48 << 16)), (1, 16, 10 | (40 << 16))])
def test_fast_rotation_is_conflict_free(nb, G, window):
    """G < 0: the systolic sweep's per-rating-block groups for a budget of -G waves per superstep.
    window = w | (run_w << 16) (plan.hpp plan_window_pack): single-item cells keep every user
    run_w records apart, without forwarded repeats."""
    d = synth.generate(500, 200, 20000, seed=1)
    if window >> 16:  # a hot item, so that single-item cells exist
        rng = np.random.default_rng(2)
        hu = rng.integers(0, 500, 3000).astype(np.int32)
        d.u = np.concatenate([d.u, hu])
        d.i = np.concatenate([d.i, np.full(len(hu), 7, np.int32)])
        d.r = np.concatenate([d.r, np.ones(len(hu))])
    b, t, g, p = fast_schedule(d.u, d.i, nb, 3, G, window=window)
    if G < 0:
        Gb = {int(x): int(t[b == x].max()) + 1 for x in np.unique(b)}  # per block: t, g in [0, G_j)
        assert all(int(g[b == x].max()) < Gb[x] for x in Gb)
        assert all(v % 8 == 0 for v in Gb.values())
        for s in range(nb):  # the superstep's waves fit the budget
            assert sum(v for x, v in Gb.items() if (x // nb + s) % nb == x % nb) <= -G
        G = 1024
    win = (window & 0xFFFF) or 8
    run_win = window >> 16
    # blocks follow DSGD blocking of the reference
    ub = np.array([mfhip.jvm.block_of(int(x), 3, nb) for x in d.u])
    ib = np.array([mfhip.jvm.block_of(int(x), 3, nb) for x in d.i])
    assert np.array_equal(b, ub * nb + ib)
    # the stratum of superstep s holds blocks (p, p+s-1); within one (stratum, sub-step) no user or
    # item row appears in two different cells
    for s in range(nb):
        in_stratum = ((b // nb + s) % nb) == (b % nb)
        for tt in np.unique(t):
            m = in_stratum & (t == tt)
            cell = b[m].astype(np.int64) * G + g[m]
            for ids in (d.u[m], d.i[m]):
                owner = {}
                for x, c in zip(ids.tolist(), cell.tolist()):
                    assert owner.setdefault(x, c) == c
    # inside a cell every user and item row recurs either at the next position (forwarded in
    # registers: user / item runs) or at least `window` positions later (the kernel's prefetch
    # distance: 8 for kernels_fast.hip, lean_ring_depth(k) for kernels_lean.hip); item runs keep the item row in registers.  Padding records (the gaps)
    # carry the zero user row and the preceding record's item, so they extend an item run.
    key = b.astype(np.int64) * G * G + t.astype(np.int64) * G + g
    runs = single = 0
    for c in np.unique(key)[:300]:
        m = np.where(key == c)[0]
        pos = p[m]
        assert len(set(pos.tolist())) == len(m)  # distinct slots (gaps = no-op padding records)
        one_item = run_win and len(np.unique(d.i[m])) == 1
        single += bool(one_item)
        for side, ids in (("u", d.u[m]), ("i", d.i[m])):
            last, prev = {}, -1
            for x, y in sorted(zip(pos.tolist(), ids.tolist())):
                run = side == "i" and last.get(y) == prev  # only padding since this item's last record
                if one_item and side == "u":  # no repeat within run_win, not even adjacent
                    assert y not in last or x - last[y] >= run_win, (y, last.get(y), x)
                else:
                    assert y not in last or x - last[y] == 1 or x - last[y] >= win or run, (side, y, last.get(y), x)
                last[y] = prev = x
        items_in_order = d.i[m[np.argsort(pos)]]
        runs += int(np.sum(items_in_order[1:] == items_in_order[:-1]))
    assert runs > 0
    assert single > 0 or not run_win
