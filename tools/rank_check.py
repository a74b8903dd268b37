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
    a = ap.parse_args()
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
        data = mfhip.synth.config(a.config, a.scale)
        _, _, _, k, nb = mfhip.synth.CONFIGS[a.config]
        k = a.k if a.k != 32 else k
        nb = a.blocks if a.blocks != 4 else nb
    else:
        data = mfhip.synth.generate(a.users, 800, 60000)
    (tu, ti, tr), (eu, ei, er) = data.split()
    del data
    p = L.default_params()
    p.num_factors, p.num_blocks, p.iterations, p.seed, p.has_seed = k, nb, a.iterations, 5, 1
    p.mode = L.MODE_DETERMINISTIC_F64 if a.mode == "det" else L.MODE_FAST_F32
    p.fast_waves = a.fast_waves
    obj = [mfhip.Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    dev = local % max(1, mfhip.device_count())
    ctx = mfhip.Context(p, rank=(dev, world, rank, obj[0]))
    t0 = time.time()
    ctx.prepare(tu, ti, tr)
    ctx.sync()
    t_prep = time.time() - t0
    plan = np.zeros(2, np.uint64)
    if a.mode == "fast" and L.lib().mf_debug_plan_digest(ctx._h, plan.ctypes.data_as(L.C.POINTER(L.C.c_uint64))) != 0:
        plan[:] = 0  # (a rank without ratings, or a host-planned schedule, has no device plan digest)
    mem = np.zeros(2, np.int64)
    L.lib().mf_debug_device_bytes(mem.ctypes.data_as(L.C.POINTER(L.C.c_int64)))
    t0 = time.time()
    ctx.run(p.iterations * p.num_blocks)  # asynchronous: rmse / factors right behind it (staged)
    if not a.staged:
        ctx.sync()
    t_run = time.time() - t0
    rm, cnt = ctx.rmse(eu, ei, er)
    st = ctx.stats()
    mem2 = np.zeros(2, np.int64)
    L.lib().mf_debug_device_bytes(mem2.ctypes.data_as(L.C.POINTER(L.C.c_int64)))
    import resource
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20  # KiB -> GiB
    print(f"rank {rank}: updates {st['updates']} groups {st['groups']} pads {st['pads']} plan records {int(plan[1])} "
          f"device bytes after prepare {mem[0] / 2**30:.2f} GiB, peak {mem2[1] / 2**30:.2f} GiB; host max RSS "
          f"{rss:.1f} GiB; prepare {t_prep:.1f} s, {p.iterations} epoch(s) {t_run:.1f} s", flush=True)
    uids, uf = ctx.factors(L.SIDE_USER)
    iids, itf = ctx.factors(L.SIDE_ITEM)
    ctx.close()
    parts = [None] * world if rank == 0 else None
    dist.gather_object((uids, uf), parts, dst=0)
    del uf
    if rank == 0:
        uids = np.concatenate([x[0] for x in parts])
        uf = np.concatenate([x[1] for x in parts])
        del parts
        o = np.argsort(uids)
        uids, uf = uids[o], uf[o]
        ref = mfhip.Context(p, devices=[0] * world) if a.fast_waves < 0 else mfhip.Context(p)
        t0 = time.time()
        ref.fit(tu, ti, tr)
        ref.sync()
        t_ref = time.time() - t0
        rrm, rcnt = ref.rmse(eu, ei, er)
        ruids, ruf = ref.factors(L.SIDE_USER)
        riids, ritf = ref.factors(L.SIDE_ITEM)
        ref.close()
        print(f"single context: prepare + {p.iterations} epoch(s) {t_ref:.1f} s", flush=True)
        assert np.array_equal(uids, ruids) and np.array_equal(iids, riids), "id sets differ"
        du = float(np.max(np.abs(uf - ruf)))
        di = float(np.max(np.abs(itf - ritf)))
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
