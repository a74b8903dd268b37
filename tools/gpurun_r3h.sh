#!/bin/bash
# Round-3: instruction-fetch and issue-stall counters of the systolic pair sweep, in situ (NFLX
# bench, 656 waves) and for the one-wave hot chain alone (tools/chain_bench.py), one --pmc pass
# each (8 SQ counters).  Output under gpurun_out/r3h/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3h
mkdir -p $O
cd /tmp
PMC="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
timeout -s KILL 300 rocprofv3 --pmc $PMC -d $O/insitu -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/insitu.log 2>&1 || { echo "in-situ pmc failed"; tail -5 $O/insitu.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $PMC -d $O/chain -o pmc --output-format csv -- python3 $R/tools/chain_bench.py 128 100000 chain > $O/chain.log 2>&1 || { echo "chain pmc failed"; tail -5 $O/chain.log; exit 1; }
cd $R
python3 - <<'EOF'
import csv, glob, collections
for tag in ("insitu", "chain"):
    f = glob.glob(f"gpurun_out/r3h/{tag}/*counter_collection.csv")[0]
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "k_sweep_pair" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(tag, {k: f"{v:.4g}" for k, v in sorted(acc.items())}, "dispatches", max(n.values()) if n else 0)
    wc = acc.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"  {tag}: wait_inst_any {acc['SQ_WAIT_INST_ANY']/wc:.3f}  wait_any {acc['SQ_WAIT_ANY']/wc:.3f}  active_inst {acc['SQ_ACTIVE_INST_ANY']/wc:.3f}  "
          f"icache miss rate {acc['SQC_ICACHE_MISSES']/max(acc['SQC_ICACHE_MISSES']+acc['SQC_ICACHE_HITS'],1):.4f}  ifetch per wave-cycle {acc['SQ_IFETCH']/wc:.4f}")
EOF
