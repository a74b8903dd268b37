#!/usr/bin/env python3
"""Reference RMSE after N epochs: the C oracle (f64, the reference's exact update order,
DSGDforMF.scala:378-418) fitted on the bench's training split, scored on its held-out split
with predictRating inner-join semantics (MatrixFactorization.scala:239-274).

    python tools/rmse_parity.py --config NFLX [--scale 1.0] [--epochs 10] [--threads 8]

Writes the result into tests/golden/rmse_ref.json under "<config>@<scale>" together with the
sha256 of the generated train/test arrays (synth.fingerprint), so bench.py and the GPU RMSE
gates (tests/test_gpu_configs.py) compare against the oracle only when the data is identical.
The fast-mode RMSE it is compared with comes from the GPU (same generator, seeds and split).
Test infrastructure: imports oracle/.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-recommendation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
FIXTURE = os.path.join(ROOT, "tests", "golden", "rmse_ref.json")


def key(config: str, scale: float) -> str:
    return f"{config}@{scale:g}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="NFLX")
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    import coracle
    from mfhip import synth
    nu, ni, nr, k, nb = synth.CONFIGS[a.config]
    data = synth.generate(max(1, int(nu * a.scale)), max(1, int(ni * a.scale)), max(1, int(nr * a.scale)))
    (tu, ti, tr), (eu, ei, er) = data.split()
    sha = synth.fingerprint(tu, ti, tr, eu, ei, er)
    del data
    t0 = time.time()
    m = coracle.dsgd_fit(tu, ti, tr, k=k, iterations=a.epochs, n_blocks=nb, seed=0, threads=a.threads)
    fit_s = time.time() - t0
    rmse, matched = m.rmse(eu, ei, er)
    rec = {"config": a.config, "scale": a.scale, "rank": k, "num_blocks": nb, "epochs": a.epochs,
           "lambda": 1.0, "lr": 0.001, "lr_method": "Default", "seed": 0,
           "train_ratings": int(len(tr)), "test_ratings": int(len(er)), "data_sha256": sha,
           "oracle_rmse": rmse, "oracle_matched": matched, "oracle_fit_s": round(fit_s, 1),
           "oracle_updates_per_s": m.updates / max(m.sweep_seconds, 1e-9), "threads": a.threads,
           "source": "oracle/mf_oracle.c (f64, reference order), tools/rmse_parity.py"}
    fx = json.load(open(FIXTURE)) if os.path.exists(FIXTURE) else {}
    fx[key(a.config, a.scale)] = rec
    json.dump(dict(sorted(fx.items())), open(FIXTURE, "w"), indent=1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
