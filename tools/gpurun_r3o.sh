#!/bin/bash
# Round-3: vector-memory path counters of the systolic sweep in situ (NFLX) vs the one-wave chain.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3o
mkdir -p $O
cd /tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
TA="TA_BUSY_avr TA_BUFFER_TOTAL_CYCLES_sum"
for tag in insitu chain; do
  CMD=$([ $tag = insitu ] && echo "$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0" || echo "$R/tools/chain_bench.py 128 100000 chain")
  timeout -s KILL 300 rocprofv3 --pmc $SQ -d $O/${tag}_sq -o pmc --output-format csv -- python3 $CMD > $O/${tag}_sq.log 2>&1 || { echo "$tag sq failed"; tail -5 $O/${tag}_sq.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $TA -d $O/${tag}_ta -o pmc --output-format csv -- python3 $CMD > $O/${tag}_ta.log 2>&1 || { echo "$tag ta failed"; tail -5 $O/${tag}_ta.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for tag in ("insitu", "chain"):
    acc = collections.defaultdict(float)
    for part in ("sq", "ta"):
        f = glob.glob(f"gpurun_out/r3o/{tag}_{part}/*counter_collection.csv")[0]
        for r in csv.DictReader(open(f)):
            if "k_sweep_pair" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    print(tag, {k: f"{v:.4g}" for k, v in sorted(acc.items())})
PY
