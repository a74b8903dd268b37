#!/usr/bin/env python3
"""DSGD throughput bench: SGD rating updates/s at rank 128 on the Netflix-shaped synthetic.

One step = one DSGD epoch (numBlocks supersteps, DSGDforMF.scala:341-344) over the training
split, fast f32 mode, factors and rating blocks resident in HBM before timing starts.

    python bench.py [--gpus N --steps K --warmup W] [--config NFLX|ML20M|...] [--mode fast|det]

N > 1 is launched by torch.distributed.run (one process per GPU).  Each rank owns
numBlocks/N user blocks; item blocks rotate between ranks over RCCL inside libmfhip
(mf_create_rank).  torch.distributed (gloo) carries only the control plane: the RCCL
unique id, the barriers around the timed region and the max/sum reductions.

Prints ONE JSON line on rank 0 with the contract fields plus "roofline" (dominant kernel,
HIP-event timed over the timed region) and "cpu_baseline" (oracle/ C restatement of the
reference, rank 0 at N=1 only, on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="NFLX")
    ap.add_argument("--mode", default="fast", choices=["fast", "det"])
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the synthetic (tests only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-supersteps", type=int, default=-1, help="oracle sample size (default: 1 epoch)")
    ap.add_argument("--fast-waves", type=int, default=0)
    ap.add_argument("--blocking", default="reference", choices=["reference", "balanced"],
                    help="fast-mode factor blocking (reference = new Random(id ^ seed).nextInt(n))")
    ap.add_argument("--traffic-json", default=None, help="rocprof PMC summary to fill roofline.traffic")
    ap.add_argument("--no-profile", action="store_true", help="skip the profiled replay (roofline = null)")
    ap.add_argument("--online-batches", type=int, default=5,
                    help="ONLINE leg (BASELINE config 5): 1M-rating micro-batches applied to the fitted model (0 = off)")
    ap.add_argument("--det-epochs", type=int, default=2,
                    help="deterministic-f64 leg (the reference's exact order) on the same data: timed epochs (0 = off)")
    ap.add_argument("--ml20m-epochs", type=int, default=9,
                    help="ML20M leg (BASELINE config 2, full size, fast f32, k=64) beside the NFLX line: timed "
                         "epochs (0 = off; only with --config NFLX on one GPU)")
    ap.add_argument("--block-update-reps", type=int, default=3,
                    help="deterministic leg: timed mf_block_update calls on one NFLX rating block (0 = off)")
    ap.add_argument("--item-split", type=int, default=0,
                    help="fast mode experiment: hot-item replicas (MFHIP_ITEM_SPLIT), max ratings per item chain "
                         "per rating block (0 = off)")
    return ap.parse_args()


class Dist:
    """Control plane over torch.distributed (gloo); a no-op at world size 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1 and os.environ.get("MFHIP_FAKE_HOSTS"):
            # rehearsal of the RCCL ring on ONE device: RCCL refuses two ranks on one GPU of one
            # host, so each rank claims its own host id and the ranks talk over loopback sockets
            os.environ["NCCL_HOSTID"] = f"mfhip-rank{self.rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def reduce(self, x: float, op: str) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


PMC_LAUNCH_TOL = 0.05  # a committed PMC summary must describe a launch this long (+-5%)


def pmc_traffic(a, k, groups, kernel, launch_us, tag=None):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 --pmc summary
    (tools/pmc_summary.py) of the same workload and kernel, or (None, None).  A summary whose
    rocprofv3 average launch differs from this run's event-timed launch (launch_us) by more than
    PMC_LAUNCH_TOL is stale -- it profiled another build of the kernel -- and is refused.
    tag: the summary's file-name suffix (profiles/r*_traffic_<config>_<tag>.json; default the mode)."""
    import glob
    tag = tag or a.mode
    paths = [a.traffic_json] if a.traffic_json and tag == a.mode else sorted(
        glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{a.config}_{tag}.json")))
    for path in reversed(paths):
        if not path or not os.path.exists(path):
            continue
        rec = json.load(open(path))
        if not (rec.get("rank") == k and rec.get("groups") in (groups, 0) and rec.get("kernel") == kernel
                and a.scale == 1.0):
            continue
        prof_us = rec.get("avg_ns", 0.0) / 1e3
        if not launch_us or abs(prof_us - launch_us) > PMC_LAUNCH_TOL * launch_us:
            print(f"[bench] {os.path.relpath(path, ROOT)}: profiled launch {prof_us:.1f} us vs this run's "
                  f"{launch_us} us: stale, not used", file=sys.stderr)
            return None, None
        return rec["bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


MALL_BYTES = 256 * 2**20  # MI355X_MICROARCH.md: 256-MiB Infinity Cache (MALL) on the die


def fetch_calibration():
    """The committed FETCH_SIZE / WRITE_SIZE calibration of the sweeps' access shape (512-B rows as
    64 lanes x 8 B, random rows of a slab past the MALL, sc1; tools/micro/fetch_calib.hip,
    tools/pmc_calib.py): {read_ratio, write_ratio, source} or None.  The ratio is raw counter bytes
    over known bytes, so the true bytes are counter / ratio."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_fetch_calib.json")))
    if not paths:
        return None
    rec = json.load(open(paths[-1]))
    cases = {c["case"]: c for c in rec.get("cases", [])}
    rd, wr = cases.get("read_sc1_3GiB"), cases.get("write_sc1_3GiB")
    if not rd or not wr or not rd.get("fetch_ratio_raw") or not wr.get("write_ratio_raw"):
        return None
    return {"read_ratio": rd["fetch_ratio_raw"], "write_ratio": wr["write_ratio_raw"],
            "source": os.path.relpath(paths[-1], ROOT)}


def traffic_level(k, users, dtype_bytes=4):
    """What the PMC bytes measure: FETCH_SIZE / WRITE_SIZE are the L2's memory-side (fabric)
    requests, Infinity-Cache (MALL) hits included (MI355X_MICROARCH.md, HBM section), so when the
    user slab fits the MALL the fraction is a fabric-traffic fraction, not an HBM one."""
    slab = (users + 2) * k * dtype_bytes
    return {"traffic_level": "l2-fabric (MALL hits included)", "user_slab_bytes": slab, "mall_bytes": MALL_BYTES,
            "user_slab_fits_mall": slab <= MALL_BYTES}


def fast_roofline(a, k, groups, st_p, prof_epochs, world, users):
    """Roofline of the fast sweep: a replay of prof_epochs epochs with a start/stop event pair on
    every sweep launch (on the library's stream; for the pair kernel recorded by the dispatch packet
    itself).  Headline: the committed PMC traffic of the same kernel (FETCH_SIZE x2 + WRITE_SIZE per
    launch) over the event-timed launch; beside it the bytes the kernel requests (mf_stats.moved_bytes,
    counted from the device plan), SURVEY 8d's per-update model (16k+20 B, which charges an item row
    per update the kernel keeps in registers through a run, so it can exceed 1) and the PMC bytes
    re-corrected with the measured calibration of this access shape (fetch_calibration)."""
    from mfhip import _lib as L
    if st_p["kernel_ms"] <= 0:
        return None
    bpu = 16 * k + 20 if a.mode == "fast" else 32 * k + 24
    launches = st_p["kernel_launches"]
    ksec = st_p["kernel_ms"] / 1e3
    achieved = st_p["moved_bytes"] / ksec / 1e9  # GB/s, this rank's sweep kernel
    kname = L.lib().mf_fast_kernel_name(k).decode() if a.mode == "fast" else det_kernel_name(k)
    launch_us = round(st_p["kernel_ms"] * 1e3 / max(launches, 1), 2)
    # the committed PMC summaries are one-GPU runs: a rank of an N-GPU ring runs other launches
    traffic, traffic_src = pmc_traffic(a, k, groups, kname, launch_us) if world == 1 else (None, None)
    launch_s = st_p["kernel_ms"] / max(launches, 1) / 1e3
    tr_gbs = traffic / launch_s / 1e9 if traffic else None
    alg_gbs = st_p["algorithmic_bytes"] / ksec / 1e9
    head = tr_gbs if tr_gbs is not None else achieved
    roof = {"bound": "hbm", "achieved": round(head, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(head / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kname,
            "achieved_source": "PMC traffic (FETCH_SIZE x2 + WRITE_SIZE) per launch / event-timed launch"
            if tr_gbs is not None else "requested bytes per launch / event-timed launch (no current PMC summary)",
            "bytes_per_launch": round(st_p["moved_bytes"] / max(launches, 1)),
            "bytes_source": "mf_stats.moved_bytes: in-range row loads/stores + schedule records of the device plan",
            "requested_achieved": round(achieved, 1), "requested_frac": round(achieved / HBM_PEAK_GBS, 4),
            "avg_launch_us": launch_us, "launches": launches, "profiled_epochs": prof_epochs,
            "traffic_source": traffic_src, "algorithmic_bytes_per_update": bpu,
            "algorithmic_achieved": round(alg_gbs, 1), "algorithmic_frac": round(alg_gbs / HBM_PEAK_GBS, 4),
            "algorithmic_note": "SURVEY 8d charges an item row read+write per update; the sweep keeps the item "
                                "row in registers through a run, so this can exceed 1 (not an HBM fraction)",
            "traffic_frac": round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs is not None else None,
            "kernel_ms_per_epoch": round(st_p["kernel_ms"] / max(prof_epochs, 1), 3)}
    roof.update(traffic_level(k, users, 4 if a.mode == "fast" else 8))
    cal = fetch_calibration()
    if traffic and cal:
        # the summary's bytes are FETCH_SIZE x2 + WRITE_SIZE; undo the x2 and divide each side by the
        # ratio measured for 8-B/lane random-row accesses
        rec = json.load(open(os.path.join(ROOT, traffic_src)))
        fetch_raw = rec["fetch_bytes_per_launch"] / 2.0
        corr = fetch_raw / cal["read_ratio"] + rec["write_bytes_per_launch"] / cal["write_ratio"]
        roof.update({"traffic_calibrated": round(corr), "calibrated_frac": round(corr / launch_s / 1e9 / HBM_PEAK_GBS, 4),
                     "calibration": cal})
    return roof


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(tu, ti, tr, k, nb, supersteps):
    """Oracle C restatement (f64, exact reference order), one thread per block of a stratum."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # checker / baseline only
    nproc = os.cpu_count() or 1
    # one thread per active rating block (the Flink-slot equivalent): a superstep has nb of them
    cores = min(nb, int(os.environ.get("OMP_NUM_THREADS", nproc)), nproc)
    m = coracle.dsgd_fit(tu, ti, tr, k=k, iterations=10, n_blocks=nb, seed=0, threads=cores,
                         max_supersteps=supersteps)
    v = m.updates / m.sweep_seconds if m.sweep_seconds > 0 else 0.0
    m.close()
    return {"value": v, "unit": "updates/s", "cores": cores, "kind": "port",
            "sample": f"{supersteps} superstep(s) of the training split ({m.updates} f64 updates, k={k}, "
                      f"n={nb}), oracle/mf_oracle.c, one thread per active block",
            "seconds": m.sweep_seconds, "nproc": nproc, "cpu_model": cpu_model(),
            "cores_note": f"threads = min(numBlocks {nb}, OMP_NUM_THREADS, nproc): the reference runs one "
                          "sequential sweep per active rating block"}


def rmse_reference(a, arrays):
    """The oracle's held-out RMSE after 10 epochs on exactly this data (tests/golden/rmse_ref.json,
    written by tools/rmse_parity.py; matched by the sha256 of the train/test arrays), or None."""
    path = os.path.join(ROOT, "tests", "golden", "rmse_ref.json")
    if a.mode != "fast" or not os.path.exists(path):
        return None
    rec = json.load(open(path)).get(f"{a.config}@{a.scale:g}")
    if not rec or rec.get("epochs") != 10:
        return None
    from mfhip import synth
    if synth.fingerprint(*arrays) != rec["data_sha256"]:
        print("[bench] rmse_ref fixture does not match this data (sha256); not used", file=sys.stderr)
        return None
    return rec


def det_kernel_name(k):
    """The persistent deterministic sweep the library picks (mfhip.cpp prepare_det_sweep): the
    split single-item chains (chain + helper wave) where k = 64 KPL, KPL in {1, 2, 4}, unless
    MFHIP_TEST det_split=0."""
    knobs = dict(x.split("=", 1) for x in os.environ.get("MFHIP_TEST", "").split(",") if "=" in x)
    if k in (64, 128, 256) and knobs.get("det_split") != "0":
        return f"k_det_sweep_split<{k // 64}, 0>"  # <KPL, 0>: the DSGD instance (<KPL, 1>: online f64)
    return "k_det_sweep2"


def det_roofline(a, k, sp):
    """The deterministic sweep against the HBM roofline: algorithmic bytes B_f64(k) = 32k+24 per
    update over its profiled launch time, and the committed PMC traffic of the same
    kernel (profiles/r*_traffic_<config>_det.json).  The kernel is bound by its per-item f64 chains
    (the sequential ddot fold), not by bytes: the fraction says how far from the roofline that is."""
    if sp["kernel_ms"] <= 0:
        return None
    launches = max(sp["kernel_launches"], 1)
    ksec = sp["kernel_ms"] / 1e3
    alg = sp["updates"] * (32 * k + 24) / ksec / 1e9
    da = argparse.Namespace(**{**vars(a), "mode": "det"})
    traffic, src = pmc_traffic(da, k, 0, det_kernel_name(k), round(sp["kernel_ms"] * 1e3 / launches, 2))
    tr_gbs = traffic / (ksec / launches) / 1e9 if traffic else None
    head = tr_gbs if tr_gbs is not None else alg
    return {"bound": "hbm", "achieved": round(head, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(head / HBM_PEAK_GBS, 4),
            "achieved_source": "PMC traffic per launch / launch time" if tr_gbs is not None
            else "algorithmic bytes / launch time (no current PMC summary)",
            "bytes_model": "algorithmic B_f64(k) = 32k+24 per update",
            "algorithmic_achieved": round(alg, 1), "algorithmic_frac": round(alg / HBM_PEAK_GBS, 4),
            "avg_launch_us": round(sp["kernel_ms"] * 1e3 / launches, 2), "traffic": traffic, "traffic_source": src,
            "traffic_frac": round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs is not None else None}


def block_update_bench(train, k, nb, det_launch_us, reps=3):
    """mf_block_update on one NFLX rating block (the Flink-resident updateLocalFactors,
    DSGDforMF.scala:378-418): the training ratings of users u % nb == 0 and items i % nb == 0 (a
    1/nb x 1/nb cell of the matrix, the size of one rating block), local indices, omegas counted over
    the whole training split, random factors.  Timed end to end (host shuffle + gather, H2D of the
    block's factor rows, one persistent split-sweep launch, D2H) and the launch alone (events);
    beside them the block's longest item chain, which bounds the launch, and the det superstep's
    per-block share (its launch over the nb blocks it runs at once)."""
    import numpy as np
    import mfhip
    from mfhip import _lib as L
    tu, ti, tr = train
    sel = (tu % nb == 0) & (ti % nb == 0)
    uu, uidx = np.unique(tu[sel], return_inverse=True)
    ii, iidx = np.unique(ti[sel], return_inverse=True)
    r = tr[sel]
    uom = np.bincount(tu)[uu].astype(np.int32)
    iom = np.bincount(ti)[ii].astype(np.int32)
    rng = np.random.default_rng(5)
    users, items = rng.random((len(uu), k)) * 0.1, rng.random((len(ii), k)) * 0.1
    p = L.default_params()
    p.num_factors = k
    walls, kms = [], []
    with mfhip.Context(p) as ctx:
        for rep in range(reps + 1):
            ctx.reset_stats()
            ctx.set_profiling(True)
            t0 = time.perf_counter()
            mfhip.block_update(r, uidx.astype(np.int32), iidx.astype(np.int32), users, uom, items, iom, k, rep, 0, 0,
                               0.001, 0, 0.0, 1.0, ctx=ctx)
            dt = time.perf_counter() - t0
            ctx.set_profiling(False)
            if rep:
                walls.append(dt)
                kms.append(ctx.stats()["kernel_ms"])
    chain = int(np.bincount(iidx).max())
    return {"ratings": int(len(r)), "users": int(len(uu)), "items": int(len(ii)), "k": k,
            "wall_ms_median": round(1e3 * float(np.median(walls)), 3),
            "kernel_ms_median": round(float(np.median(kms)), 3), "longest_item_chain": chain,
            "det_superstep_block_share_ms": round(det_launch_us / 1e3 / nb, 3) if det_launch_us else None,
            "note": "one persistent k_det_sweep_split launch per call, bitwise the oracle "
                    "(tests/test_gpu_dsgd.py test_block_update_1m_hot_block_bit_exact); the launch is bounded by "
                    "the block's longest item chain (its updates are sequential, DSGDforMF.scala:395-415)"}


def det_leg(a, k, nb, train, test, ref, stream):
    """The deterministic f64 mode on the same data: DSGDforMF.scala:378-418's exact update order
    (JVM shuffle, F2J ddot fold, no FMA), one persistent sweep per superstep.  Timed epochs after
    one warmup epoch (warm: a run takes over the first supersteps the previous run built on the
    host in the background), then a restarted 10-epoch fit -- cold: restart drops those builds,
    so it pays the first superstep's host build, reported as cold_fit_s -- whose held-out RMSE
    must equal the f64 oracle's on this data (tests/golden/rmse_ref.json) to the last bit of its
    printout; then the ONLINE leg in f64 on that model (the precision the bit-exact online tests
    cover)."""
    import mfhip
    from mfhip import _lib as L
    p = L.default_params()
    p.num_factors, p.num_blocks, p.seed, p.has_seed = k, nb, 0, 1
    p.iterations = 10
    p.mode = L.MODE_DETERMINISTIC_F64
    with mfhip.Context(p) as ctx:
        t0 = time.time()
        ctx.prepare(*train)
        ctx.sync()
        t_prep = time.time() - t0
        ctx.run(nb)
        ctx.sync()
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.run(a.det_epochs * nb)
        ctx.sync()
        el = time.perf_counter() - t0
        st = ctx.stats()
        ctx.reset_stats()
        ctx.set_profiling(True)
        ctx.run(nb)
        ctx.sync()
        ctx.set_profiling(False)
        sp = ctx.stats()
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.restart()
        ctx.run(10 * nb)
        ctx.sync()
        cold = time.perf_counter() - t0
        cold_updates = ctx.stats()["updates"]
        rmse, _ = ctx.rmse(*test)
        online = online_leg(ctx, stream, a) if stream is not None else None
    launch_us = sp["kernel_ms"] * 1e3 / max(sp["kernel_launches"], 1)
    blk = block_update_bench(train, k, nb, launch_us, a.block_update_reps) if a.block_update_reps > 0 else None
    return {"metric": "SGD rating updates/sec, deterministic f64 (the reference's exact update order)",
            "value": round(st["updates"] / el, 1), "unit": "updates/s", "dtype": "f64", "epochs": a.det_epochs,
            "ms_per_step": round(el * 1e3 / a.det_epochs, 3), "kernel": det_kernel_name(k),
            "avg_launch_us": round(sp["kernel_ms"] * 1e3 / max(sp["kernel_launches"], 1), 2),
            "roofline": det_roofline(a, k, sp),
            "launches_per_epoch": sp["kernel_launches"], "prepare_s": round(t_prep, 2),
            "cold_fit_s": round(cold, 4), "cold_fit_epochs": 10,
            "cold_value": round(cold_updates / cold, 1) if cold > 0 else None,
            "cold_note": "restart + 10 epochs + sync from a cold host pipeline (no superstep built ahead)",
            "rmse": round(rmse, 9), "rmse_ref": round(ref["oracle_rmse"], 9) if ref else None,
            "rmse_equal_to_ref": (abs(rmse - ref["oracle_rmse"]) <= 1e-12 * ref["oracle_rmse"]) if ref else None,
            "block_update": blk, "online": online}  # online: moved to the top-level "online" block by main()


def ml20m_leg(a):
    """BASELINE config 2 at full size beside the headline: ML20M-shaped synthetic (138k x 27k x 20M),
    fast f32, k = 64, numBlocks 8 (mfhip.synth.CONFIGS) on the same GPU, after the NFLX context is
    closed.  Timed epochs after one warmup epoch, the same profiled replay and roofline as the
    headline (PMC summary profiles/r*_traffic_ML20M_fast.json), and the held-out RMSE after exactly
    10 epochs against the f64 oracle's on the same data (tests/golden/rmse_ref.json)."""
    import mfhip
    from mfhip import _lib as L
    from mfhip import synth
    ma = argparse.Namespace(**{**vars(a), "config": "ML20M", "mode": "fast", "traffic_json": None})
    nu, ni, nr, k, nb = synth.CONFIGS["ML20M"]
    nu, ni, nr = max(1, int(nu * a.scale)), max(1, int(ni * a.scale)), max(1, int(nr * a.scale))
    (tu, ti, tr), (eu, ei, er) = synth.generate(nu, ni, nr).split()
    p = L.default_params()
    p.num_factors, p.num_blocks, p.seed, p.has_seed = k, nb, 0, 1
    p.iterations = 10
    p.mode = L.MODE_FAST_F32
    with mfhip.Context(p) as ctx:
        t0 = time.time()
        ctx.prepare(tu, ti, tr)
        ctx.sync()
        t_prep = time.time() - t0
        ctx.run(nb)
        ctx.sync()
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.run(a.ml20m_epochs * nb)
        ctx.sync()
        el = time.perf_counter() - t0
        st = ctx.stats()
        prof_epochs = min(a.ml20m_epochs, 2)
        ctx.reset_stats()
        ctx.set_profiling(True)
        ctx.run(prof_epochs * nb)
        ctx.sync()
        ctx.set_profiling(False)
        st_p = ctx.stats()
        ctx.restart()
        ctx.run(10 * nb)
        rmse, _ = ctx.rmse(eu, ei, er)
    ref = rmse_reference(ma, (tu, ti, tr, eu, ei, er))
    return {"metric": "SGD rating updates/sec, ML20M-shaped (BASELINE config 2), fast f32, rank 64, 1 GPU",
            "value": round(st["updates"] / el, 1), "unit": "updates/s", "dtype": "f32", "epochs": a.ml20m_epochs,
            "ms_per_step": round(el * 1e3 / a.ml20m_epochs, 3), "groups": st["groups"], "pad_records": st["pads"],
            "config": {"users": nu, "items": ni, "ratings": nr, "train_ratings": int(len(tr)), "rank": k,
                       "num_blocks": nb},
            "roofline": fast_roofline(ma, k, st["groups"], st_p, prof_epochs, 1, nu),
            "rmse": round(rmse, 6), "rmse_epochs": 10, "rmse_ref": round(ref["oracle_rmse"], 6) if ref else None,
            "rmse_rel": round((rmse - ref["oracle_rmse"]) / ref["oracle_rmse"], 5) if ref else None,
            "prepare_s": round(t_prep, 2)}


ONLINE_BATCH = 1_000_000


def online_stream(a, synth, nu, ni):
    """The ONLINE config's input (BASELINE config 5): 1M-rating micro-batches from the same
    generator (other seed), one untimed warmup batch plus a.online_batches timed ones."""
    return synth.generate(max(1, int(nu * a.scale)), max(1, int(ni * a.scale)),
                          ONLINE_BATCH * (a.online_batches + 1), seed=99, test_fraction=0.0)


def online_roofline(a, k, dtype, kernel, kernel_ms, batch):
    """The online sweep against the HBM roofline: algorithmic bytes per update B_f32(k) = 16k+20 /
    B_f64(k) = 32k+24 times the batch, over the median event-timed launch; frac is
    the committed PMC traffic of the same kernel over the same launch (profiles/r*_traffic_<config>_
    online_<dtype>.json, refused when stale), else the algorithmic figure."""
    if not kernel_ms or kernel_ms <= 0:
        return None
    bpu = 16 * k + 20 if dtype == "f32" else 32 * k + 24
    ksec = kernel_ms / 1e3
    alg = batch * bpu / ksec / 1e9
    launch_us = round(kernel_ms * 1e3, 2)
    traffic, src = pmc_traffic(a, k, 0, kernel, launch_us, tag=f"online_{dtype}")
    tr_gbs = traffic / ksec / 1e9 if traffic else None
    achieved = tr_gbs if tr_gbs is not None else alg
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
            "achieved_source": "PMC traffic per launch / launch time" if tr_gbs is not None
            else "algorithmic bytes / launch time (no current PMC summary)",
            "avg_launch_us": launch_us, "traffic_source": src,
            "algorithmic_bytes_per_update": bpu, "algorithmic_bytes_per_launch": batch * bpu,
            "algorithmic_achieved": round(alg, 1), "algorithmic_frac": round(alg / HBM_PEAK_GBS, 4),
            "traffic_frac": round(tr_gbs / HBM_PEAK_GBS, 4) if tr_gbs is not None else None}


def online_leg(ctx, stream, a, batch=ONLINE_BATCH):
    """BASELINE config 5: streaming micro-batches on top of the offline DSGD model just fitted.
    Each batch: SGDUpdater.nextFactors in arrival order with per-user FIFO (FlinkOnlineMF.scala:
    52-137; core/FactorUpdater.scala:37-45), unseen ids initialised on first touch; timed end to
    end.  The first batch is a warmup (it allocates the batch scratch and the pinned upload
    buffer once): reported as first_batch_s, not in the median."""
    import numpy as np
    from mfhip import _lib as L
    rates, launches, kms = [], [], []
    first = None
    ctx.set_profiling(True)  # a few launches per batch: one event pair each, noise against ~6 ms
    for b in range(a.online_batches + 1):
        s = slice(b * batch, (b + 1) * batch)
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.online_update(stream.u[s], stream.i[s], stream.r[s], L.ONLINE_NEXT_FACTORS)
        ctx.sync()
        dt = time.perf_counter() - t0
        if b == 0:
            first = dt
            continue
        rates.append(batch / dt)
        st = ctx.stats()
        launches.append(st["kernel_launches"])
        kms.append(st["kernel_ms"])
    ctx.set_profiling(False)
    dtype = "f64" if ctx.params.mode == L.MODE_DETERMINISTIC_F64 else "f32"
    k = ctx.params.num_factors
    kernel = ("k_online_f32" if k <= 256 else "k_online_sweep") if dtype == "f32" else \
        (f"k_det_sweep_split<{k // 64}, 1>" if k in (64, 128, 256) else "k_online_sweep")
    kms_med = float(np.median(kms))
    kms_mean = float(np.mean(kms))  # the roofline's launch time: rocprofv3's average is a mean too
    return {"metric": "online ratings/s (1M-rating micro-batches on the fitted model)",
            "value": round(float(np.median(rates)), 1), "unit": "ratings/s", "min": round(float(min(rates)), 1),
            "max": round(float(max(rates)), 1), "first_batch_s": round(first, 4),
            "batch": batch, "batches": a.online_batches, "launches_median": float(np.median(launches)),
            "kernel_ms_median": round(kms_med, 3), "kernel_ms_mean": round(kms_mean, 3),
            "flavour": "FlinkOnlineMF / SGDUpdater.nextFactors (lr 0.01)", "target": 10e6, "dtype": dtype,
            "kernel": f"{kernel} (one persistent launch per batch: per-item waves, per-user tickets)",
            "roofline": online_roofline(a, k, dtype, kernel, kms_mean if launches and max(launches) == 1 else None,
                                        batch),
            "timing": "end to end per micro-batch: host id lookup, H2D, device plan (kernels_online.hip), "
                      f"one {kernel} launch, sync; median over the timed batches after one warmup batch"}


def main():
    a = parse()
    D = Dist()
    import numpy as np
    import mfhip
    from mfhip import _lib as L
    from mfhip import synth

    nu, ni, nr, k, nb = synth.CONFIGS[a.config]
    t0 = time.time()
    data = synth.generate(max(1, int(nu * a.scale)), max(1, int(ni * a.scale)), max(1, int(nr * a.scale)))
    (tu, ti, tr), (eu, ei, er) = data.split()
    t_gen = time.time() - t0
    print(f"[bench] rank {D.rank}: generated {len(tr)} training ratings in {t_gen:.1f} s", file=sys.stderr, flush=True)

    p = L.default_params()
    p.num_factors, p.num_blocks, p.seed, p.has_seed = k, nb, 0, 1
    p.iterations = a.warmup + a.steps
    p.mode = L.MODE_FAST_F32 if a.mode == "fast" else L.MODE_DETERMINISTIC_F64
    p.fast_waves = a.fast_waves
    if a.item_split:
        os.environ["MFHIP_ITEM_SPLIT"] = str(a.item_split)
    p.fast_blocking = L.BLOCKING_BALANCED if a.blocking == "balanced" else L.BLOCKING_REFERENCE
    if D.world > 1:
        uid = D.bcast_bytes(mfhip.Context.unique_id() if D.rank == 0 else None)
        dev = D.local_rank % max(1, mfhip.device_count())  # identity on a full node
        ctx = mfhip.Context(p, rank=(dev, D.world, D.rank, uid))
    else:
        ctx = mfhip.Context(p)
    t0 = time.time()
    ctx.prepare(tu, ti, tr)
    ctx.sync()
    t_prep = time.time() - t0
    print(f"[bench] rank {D.rank}: prepared (blocking, plan, H2D) in {t_prep:.1f} s", file=sys.stderr, flush=True)

    ctx.run(a.warmup * nb)
    ctx.sync()
    ctx.reset_stats()
    ctx.set_profiling(False)  # per-launch timestamps cost ~15% of wall time: not in the timed region
    import torch
    have_torch_gpu = torch.cuda.is_available()
    D.barrier()
    if have_torch_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.run(a.steps * nb)
    ctx.sync()
    if have_torch_gpu:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.barrier()
    st = ctx.stats()
    elapsed = D.reduce(t1 - t0, "max")
    updates = D.reduce(float(st["updates"]), "sum")

    # Roofline: replay min(steps, 2) epochs of the same workload with a start/stop event pair on
    # every sweep launch (on the library's stream; for the pair kernel recorded by the dispatch
    # packet itself).  achieved = the bytes the sweep kernel requests per launch (its row loads
    # and stores with in-range offsets plus its schedule records: mf_stats.moved_bytes, counted
    # from the device plan) / its average launch time.  The SURVEY 8d per-update model
    # (16k+20 B) is reported beside it as algorithmic_frac: it charges an item row per update,
    # which this kernel keeps in registers through a run, so it overstates the bytes.
    prof_epochs = 0 if a.no_profile else min(a.steps, 2)
    st_p = {"kernel_ms": 0.0, "kernel_launches": 0, "algorithmic_bytes": 0.0, "moved_bytes": 0.0, "updates": 0}
    if prof_epochs:
        ctx.reset_stats()
        ctx.set_profiling(True)
        D.barrier()
        ctx.run(prof_epochs * nb)
        ctx.sync()
        ctx.set_profiling(False)
        st_p = ctx.stats()

    # RMSE after exactly 10 epochs (the metric's second half): the same prepared fit restarted
    # from its initial factors, 10 epochs, held-out RMSE; beside it the oracle's RMSE on the same
    # data (f64, reference order) when the committed fixture matches.
    t0 = time.time()
    ctx.restart()
    ctx.run(10 * nb)
    rmse, matched = ctx.rmse(eu, ei, er)
    t_eval = time.time() - t0
    ref = rmse_reference(a, (tu, ti, tr, eu, ei, er)) if D.rank == 0 else None

    value = updates / elapsed
    roof = fast_roofline(a, k, st["groups"], st_p, prof_epochs, D.world, int(nu * a.scale))

    online = None
    stream = online_stream(a, synth, nu, ni) if D.world == 1 and a.online_batches > 0 else None
    if stream is not None:
        online = {"f32": online_leg(ctx, stream, a)}
    det = None
    if D.world == 1 and a.mode == "fast" and a.det_epochs > 0:
        ctx.close()  # its HBM is not needed any more
        det = det_leg(a, k, nb, (tu, ti, tr), (eu, ei, er), ref, stream)
        if online is not None and det.get("online"):
            online["f64"] = det.pop("online")

    ml20m = None
    if D.world == 1 and a.config == "NFLX" and a.mode == "fast" and a.ml20m_epochs > 0:
        ctx.close()  # (closed already when the det leg ran)
        ml20m = ml20m_leg(a)

    cpu = None
    if D.rank == 0 and D.world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(tu, ti, tr, k, nb, a.cpu_supersteps if a.cpu_supersteps > 0 else nb)

    if D.rank == 0:
        out = {
            "metric": "SGD rating updates/sec (node) at rank 128, 1/2/4/8 GPU; RMSE after 10 epochs",
            "value": round(value, 1), "unit": "updates/s", "n_gpus": D.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / max(a.steps, 1), 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32" if a.mode == "fast" else "f64", "data": "synthetic (SURVEY.md 8d generator, seeds 42/1234/7)",
            "config": {"workload": f"{a.config}-shaped DSGD {'fast' if a.mode == 'fast' else 'deterministic'}",
                       "users": int(nu * a.scale), "items": int(ni * a.scale), "ratings": int(nr * a.scale),
                       "train_ratings": int(len(tr)), "rank": k, "num_blocks": nb, "lambda": 1.0, "lr": 0.001,
                       "lr_method": "Default", "blocking": a.blocking, "item_split": a.item_split, "groups": st["groups"], "pad_records": st["pads"],
                       "parallelism": f"dsgd-ring{D.world}"},
            "rmse": round(rmse, 6), "rmse_epochs": 10, "rmse_matched": matched,
            "rmse_ref": round(ref["oracle_rmse"], 6) if ref else None,
            "rmse_rel": round((rmse - ref["oracle_rmse"]) / ref["oracle_rmse"], 5) if ref else None,
            "rmse_ref_source": "tests/golden/rmse_ref.json (tools/rmse_parity.py, oracle f64, same data sha256)"
                               if ref else None,
            "roofline": roof, "cpu_baseline": cpu, "online": online, "deterministic": det, "ml20m": ml20m,
            "setup_s": {"generate": round(t_gen, 2), "prepare": round(t_prep, 2), "rmse_eval": round(t_eval, 3)},
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
