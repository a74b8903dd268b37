#!/usr/bin/env python3
"""Rank-mode (one process per GPU, RCCL ring) check against a single-process context.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
        tools/rank_check.py [--mode det|fast]

Every rank fits the same seeded synthetic in rank mode; rank 0 also fits it in a plain
single-device context and compares factors (det: bitwise) and RMSE.  Ranks beyond the
device count share devices (local_rank % device_count).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))


def row_hash(f):
    """One 64-bit hash per factor row (bitwise: any differing bit changes it)."""
    import numpy as np
    b = np.ascontiguousarray(f).view(np.uint64)
    mult = (np.arange(1, b.shape[1] + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1)
    with np.errstate(over="ignore"):
        return (b * mult).sum(axis=1, dtype=np.uint64)


def digest(ids, hashes):
    """Order-free 64-bit digest of (id, row) pairs: equal digests <=> (almost surely) equal rows per id."""
    with np.errstate(over="ignore"):
        h = hashes ^ (np.asarray(ids).astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F))
        return int(h.sum(dtype=np.uint64))


def stepwise(a, ctx, p, tu, ti, tr, rank, world, dist):
    from mfhip import _lib as L
    import mfhip
    steps = p.iterations * p.num_blocks
    trace = []
    for s in range(steps):
        ctx.run(1)
        ctx.sync()
        uids, uf = ctx.factors(L.SIDE_USER)
        iids, itf = ctx.factors(L.SIDE_ITEM)  # (an all-gather of the item blocks: every rank calls it)
        trace.append((uids, row_hash(uf), iids, row_hash(itf)))
    ctx.close()
    parts = [None] * world if rank == 0 else None
    dist.gather_object(trace, parts, dst=0)
    if rank == 0:
        ref = mfhip.Context(p, devices=[0] * world) if a.fast_waves < 0 else mfhip.Context(p)
        ref.prepare(tu, ti, tr)
        first = None
        for s in range(steps):
            ref.run(1)
            ref.sync()
            ruids, ruf = ref.factors(L.SIDE_USER)
            riids, ritf = ref.factors(L.SIDE_ITEM)
            rhu, rhi = dict(zip(ruids.tolist(), row_hash(ruf).tolist())), row_hash(ritf)
            du = {}
            for r in range(world):
                uids, hu, iids, hi = parts[r][s]
                du[r] = int(sum(1 for x, h in zip(uids.tolist(), hu.tolist()) if rhu[x] != h))
            iids, hi = parts[0][s][2], parts[0][s][3]
            assert np.array_equal(iids, riids)
            di = int(np.sum(hi != rhi))
            dv = [int(np.sum(parts[r][s][3] != hi)) for r in range(world)]
            print(f"superstep {s + 1}: differing user rows per rank {du}; differing item rows {di} "
                  f"(rank views differing from rank 0's: {dv})", flush=True)
            if first is None and (di or any(du.values())):
                first = s + 1
        ref.close()
        print(f"STEPWISE first differing superstep: {first}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="det")
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--fast-waves", type=int, default=0,
                    help="fast mode, -G: uniform groups; the reference is then an in-process context with one "
                         "virtual shard per rank (same plan), compared bitwise")
    ap.add_argument("--users", type=int, default=3000,
                    help="distinct users (3000: the reference's blocking puts every user into 2 of 4 blocks, so "
                         "one of 2 ranks holds no rating -- the empty-rank edge)")
    ap.add_argument("--k", type=int, default=32, help="rank (64 / 128 / 256: the pair sweep, whose ring overlaps)")
    ap.add_argument("--config", default=None,
                    help="a BASELINE-shaped synthetic instead (synth.CONFIGS: ML20M / NFLX / YAHOO) at --scale; "
                         "k and the block count default to the config's")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--fast-tol", type=float, default=5e-3,
                    help="fast mode with automatic groups: |rmse_rank - rmse_single| / rmse_single bound")
    ap.add_argument("--staged", action="store_true",
                    help="prepare + run + evaluate with no sync in between (the JNI dsgdPrepare / dsgdRun path): "
                         "evaluation must wait for the last superstep's overlapped launch and ring step itself")
    ap.add_argument("--stepwise", action="store_true",
                    help="run one superstep at a time (synced) and compare every rank's rows with the "
                         "single context after each: names the first superstep and rank that differ")
    ap.add_argument("--twice", action="store_true",
                    help="fit each side twice and report which side (rank ring / single context) repeats itself")
    ap.add_argument("--sync-each", action="store_true", help="host-sync after every superstep of the rank fits")
    ap.add_argument("--shared-data", default=None,
                    help="directory: rank 0 writes the split once (unless a previous step did), every rank "
                         "memory-maps it (large scales); the caller removes it")
    ap.add_argument("--no-ref", action="store_true",
                    help="rank fits only: print a DIGEST line (factors and RMSE) to compare with a --ref-only run")
    ap.add_argument("--ref-only", action="store_true",
                    help="one process: the single context only, same DIGEST line (full-size runs keep the two "
                         "sides in separate jobs so their host memory never adds up)")
    ap.add_argument("--ref-world", type=int, default=8, help="--ref-only with fast-waves < 0: virtual shards")
    ap.add_argument("--serial-prepare", action="store_true", help="ranks prepare one after another")
    ap.add_argument("--knobs", default=None, help="MFHIP_TEST for this run (e.g. device_plan=0)")
    ap.add_argument("--setenv", action="append", default=[], help="K=V set before the communicator exists")
    a = ap.parse_args()
    if a.knobs:
        os.environ["MFHIP_TEST"] = a.knobs
    for kv in a.setenv:
        os.environ[kv.split("=", 1)[0]] = kv.split("=", 1)[1]
    import torch.distributed as dist
    import mfhip
    from mfhip import _lib as L
    if os.environ.get("MFHIP_FAKE_HOSTS"):
        # several ranks on ONE device: RCCL refuses that on one host, so each rank claims its
        # own host id and the ranks talk over loopback sockets (a rehearsal of the ring)
        os.environ["NCCL_HOSTID"] = "mfhip-rank" + os.environ.get("RANK", "0")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", rank))
    import time
    k, nb = a.k, a.blocks
    if a.config:
        _, _, _, k, nb = mfhip.synth.CONFIGS[a.config]
        k = a.k if a.k != 32 else k
        nb = a.blocks if a.blocks != 4 else nb
    names = ("tu", "ti", "tr", "eu", "ei", "er")
    if a.shared_data:
        # rank 0 generates and splits once; every rank maps the same files (one copy in the page
        # cache instead of one per rank: the full-size rehearsal's host memory)
        if rank == 0 and not os.path.exists(os.path.join(a.shared_data, "er.npy")):  # (another step's split)
            os.makedirs(a.shared_data, exist_ok=True)
            data = mfhip.synth.config(a.config, a.scale) if a.config else mfhip.synth.generate(a.users, 800, 60000)
            for nm, arr in zip(names, [x for part in data.split() for x in part]):
                np.save(os.path.join(a.shared_data, nm + ".npy"), arr)
            del data
        dist.barrier()
        tu, ti, tr, eu, ei, er = [np.load(os.path.join(a.shared_data, nm + ".npy"), mmap_mode="r") for nm in names]
    else:
        data = mfhip.synth.config(a.config, a.scale) if a.config else mfhip.synth.generate(a.users, 800, 60000)
        (tu, ti, tr), (eu, ei, er) = data.split()
        del data
    p = L.default_params()
    p.num_factors, p.num_blocks, p.iterations, p.seed, p.has_seed = k, nb, a.iterations, 5, 1
    p.mode = L.MODE_DETERMINISTIC_F64 if a.mode == "det" else L.MODE_FAST_F32
    p.fast_waves = a.fast_waves
    if a.ref_only:
        ref = mfhip.Context(p, devices=[0] * a.ref_world) if a.fast_waves < 0 else mfhip.Context(p)
        t0 = time.time()
        ref.fit(tu, ti, tr)
        ref.sync()
        t_ref = time.time() - t0
        rrm, rcnt = ref.rmse(eu, ei, er)
        ruids, ruf = ref.factors(L.SIDE_USER)
        riids, ritf = ref.factors(L.SIDE_ITEM)
        ref.close()
        print(f"single context ({a.mode}, {a.config}@{a.scale:g}): prepare + {p.iterations} epoch(s) {t_ref:.1f} s",
              flush=True)
        print(f"DIGEST users {digest(ruids, row_hash(ruf)):016x} items {digest(riids, row_hash(ritf)):016x} "
              f"rmse {rrm:.12f} matched {rcnt}", flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    obj = [mfhip.Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    dev = local % max(1, mfhip.device_count())
    ctx = mfhip.Context(p, rank=(dev, world, rank, obj[0]))
    t0 = time.time()
    if a.serial_prepare:  # one rank at a time: the transient device blocking of every rank's copy of
        for r in range(world):  # all ratings does not add up on the one shared card
            if r == rank:
                ctx.prepare(tu, ti, tr)
                ctx.sync()
            dist.barrier()
    else:
        ctx.prepare(tu, ti, tr)
        ctx.sync()
    t_prep = time.time() - t0
    plan = np.zeros(2, np.uint64)
    if a.mode == "fast" and L.lib().mf_debug_plan_digest(ctx._h, plan.ctypes.data_as(L.C.POINTER(L.C.c_uint64))) != 0:
        plan[:] = 0  # (a rank without ratings, or a host-planned schedule, has no device plan digest)
    mem = np.zeros(2, np.int64)
    has_mem = hasattr(L.lib(), "mf_debug_device_bytes")  # (an older build, A/B runs)
    if has_mem:
        L.lib().mf_debug_device_bytes(mem.ctypes.data_as(L.C.POINTER(L.C.c_int64)))
    if a.stepwise:
        stepwise(a, ctx, p, tu, ti, tr, rank, world, dist)
        return
    t0 = time.time()
    if a.sync_each:
        for _ in range(p.iterations * p.num_blocks):
            ctx.run(1)
            ctx.sync()
    else:
        ctx.run(p.iterations * p.num_blocks)  # asynchronous: rmse / factors right behind it (staged)
    if not a.staged:
        ctx.sync()
    t_run = time.time() - t0
    rm, cnt = ctx.rmse(eu, ei, er)
    st = ctx.stats()
    mem2 = np.zeros(2, np.int64)
    if has_mem:
        L.lib().mf_debug_device_bytes(mem2.ctypes.data_as(L.C.POINTER(L.C.c_int64)))
    import resource
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20  # KiB -> GiB
    print(f"rank {rank}: updates {st['updates']} groups {st['groups']} pads {st['pads']} plan records {int(plan[1])} "
          f"device bytes after prepare {mem[0] / 2**30:.2f} GiB, peak {mem2[1] / 2**30:.2f} GiB; host max RSS "
          f"{rss:.1f} GiB; prepare {t_prep:.1f} s, {p.iterations} epoch(s) {t_run:.1f} s", flush=True)
    uids, uf = ctx.factors(L.SIDE_USER)
    iids, itf = ctx.factors(L.SIDE_ITEM)
    ctx.close()
    if a.twice:  # a second rank-mode fit on a fresh communicator: does the ring repeat itself?
        obj = [mfhip.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        with mfhip.Context(p, rank=(dev, world, rank, obj[0])) as c2:
            if a.sync_each:
                c2.prepare(tu, ti, tr)
                for _ in range(p.iterations * p.num_blocks):
                    c2.run(1)
                    c2.sync()
            else:
                c2.fit(tu, ti, tr)
            plan2 = np.zeros(2, np.uint64)
            if a.mode == "fast" and L.lib().mf_debug_plan_digest(c2._h, plan2.ctypes.data_as(L.C.POINTER(L.C.c_uint64))):
                plan2[:] = 0
            same = (np.array_equal(row_hash(c2.factors(L.SIDE_USER)[1]), row_hash(uf)),
                    np.array_equal(row_hash(c2.factors(L.SIDE_ITEM)[1]), row_hash(itf)),
                    f"plan {int(plan[0]):016x}" + ("" if plan2[0] == plan[0] else f" -> {int(plan2[0]):016x}"))
        flags = [None] * world if rank == 0 else None
        dist.gather_object(same, flags, dst=0)
        if rank == 0:
            print(f"rank-mode fit repeats itself (users, items, plan digest) per rank: {flags}", flush=True)
    if a.no_ref:
        du_ = [None] * world if rank == 0 else None
        dist.gather_object(digest(uids, row_hash(uf)), du_, dst=0)
        if rank == 0:
            tot = 0
            for x in du_:
                tot = (tot + x) % (1 << 64)
            print(f"DIGEST users {tot:016x} items {digest(iids, row_hash(itf)):016x} rmse {rm:.12f} matched {cnt}",
                  flush=True)
            print("RANK_CHECK_OK", flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    # users travel to rank 0 as one 64-bit hash per row (bitwise comparison) plus the row's
    # largest magnitude-free summary: the full slab would be 3.7 GB at YAHOO's full size
    parts = [None] * world if rank == 0 else None
    dist.gather_object((uids, row_hash(uf), uf.astype(np.float32)), parts, dst=0)
    del uf
    if rank == 0:
        owner = np.concatenate([np.full(len(x[0]), r, np.int32) for r, x in enumerate(parts)])
        uids = np.concatenate([x[0] for x in parts])
        uh = np.concatenate([x[1] for x in parts])
        uf32 = np.concatenate([x[2] for x in parts])
        del parts
        o = np.argsort(uids)
        uids, uh, uf32, owner = uids[o], uh[o], uf32[o], owner[o]
        ref = mfhip.Context(p, devices=[0] * world) if a.fast_waves < 0 else mfhip.Context(p)
        t0 = time.time()
        ref.fit(tu, ti, tr)
        ref.sync()
        t_ref = time.time() - t0
        rrm, rcnt = ref.rmse(eu, ei, er)
        ruids, ruf = ref.factors(L.SIDE_USER)
        riids, ritf = ref.factors(L.SIDE_ITEM)
        ref.close()
        if a.twice:
            with (mfhip.Context(p, devices=[0] * world) if a.fast_waves < 0 else mfhip.Context(p)) as r2:
                r2.fit(tu, ti, tr)
                print(f"single-context fit repeats itself: users "
                      f"{np.array_equal(row_hash(r2.factors(L.SIDE_USER)[1]), row_hash(ruf))} items "
                      f"{np.array_equal(row_hash(r2.factors(L.SIDE_ITEM)[1]), row_hash(ritf))}", flush=True)
        print(f"single context: prepare + {p.iterations} epoch(s) {t_ref:.1f} s", flush=True)
        assert np.array_equal(uids, ruids) and np.array_equal(iids, riids), "id sets differ"
        bad = uh != row_hash(ruf)
        du = float(np.max(np.abs(uf32[bad] - ruf[bad].astype(np.float32)))) if bad.any() else 0.0
        di = float(np.max(np.abs(itf - ritf)))
        if bad.any():  # which ranks' users differ, and how many rows
            per = {int(r): int(np.sum(bad & (owner == r))) for r in range(world)}
            print(f"differing user rows per rank: {per} of {len(uids)}", flush=True)
        if di != 0.0:
            print(f"differing item rows: {int(np.sum(np.any(itf != ritf, axis=1)))} of {len(iids)}", flush=True)
        print(f"world={world} mode={a.mode} config={a.config or 'small'}@{a.scale:g} k={k} n={nb} "
              f"rmse rank={rm:.6f} single={rrm:.6f} matched {cnt}/{rcnt} "
              f"max|dU|={du:.3g} max|dI|={di:.3g}", flush=True)
        if a.mode == "det" or a.fast_waves < 0:
            # factors bitwise; the RMSE's SSE is all-reduced over ranks (another summation order)
            assert du == 0.0 and di == 0.0 and abs(rm - rrm) <= 1e-12 * rrm, "rank mode is not bit-exact"
        else:
            assert abs(rm - rrm) / rrm < a.fast_tol, "rank-mode RMSE off"
        print("RANK_CHECK_OK", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
