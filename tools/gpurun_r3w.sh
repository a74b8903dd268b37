#!/bin/bash
# Round-3: instruction-cache behaviour of the systolic sweep (its unrolled 56-pair chunk bodies are
# tens of KB): in situ (NFLX, ML20M) vs the one-wave chain.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3w
mkdir -p $O
cd /tmp
SQ="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU"
for tag in NFLX ML20M chain; do
  CMD=$([ $tag = chain ] && echo "$R/tools/chain_bench.py 128 100000 chain" || echo "$R/bench.py --config $tag --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0")
  timeout -s KILL 300 rocprofv3 --pmc $SQ -d $O/${tag} -o pmc --output-format csv -- python3 $CMD > $O/${tag}.log 2>&1 || { echo "$tag failed"; tail -5 $O/${tag}.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for tag in ("NFLX", "ML20M", "chain"):
    acc = collections.defaultdict(float)
    f = glob.glob(f"gpurun_out/r3w/{tag}/*counter_collection.csv")[0]
    for r in csv.DictReader(open(f)):
        if "k_sweep_pair" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    print(tag, {k: f"{v:.4g}" for k, v in sorted(acc.items())})
PY
