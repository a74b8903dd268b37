#!/bin/bash
# Full-size YAHOO strong-scaling inputs on the GPU box (its host has the memory): the plan probe at
# G = 1/2/4/8 (tools/probe/plan_probe ... scale) and a wave trace of one YAHOO epoch (experiments
# library) summarised by tools/sys_trace.py / tools/crowd_trace.py.  Outputs under gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:?out dir}
mkdir -p "$O"
(while sleep 30; do echo "[yahoo_scale] $(date +%T) still running"; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python tools/probe/dump_ratings.py YAHOO /tmp > "$O/dump.log" 2>&1 || { echo dump failed; exit 1; }
make -C tools/probe plan_probe > /dev/null || exit 1
timeout -k 10 900 tools/probe/plan_probe /tmp 8 256 1024 scale > "$O/yscale.txt" 2> "$O/probe.err" || { echo probe failed; tail -3 "$O/probe.err"; exit 1; }
rm -f /tmp/probe_u.bin /tmp/probe_i.bin /tmp/probe_r.bin
grep -v SCALE "$O/yscale.txt" | head -20
if [ -n "$2" ]; then
  MFHIP_LIB=$2 MFHIP_WAVE_TRACE=/tmp/yahoo.trace timeout -k 10 900 python bench.py --config YAHOO --steps 1 --warmup 1 \
    --no-cpu-baseline --online-batches 0 --det-epochs 0 --no-profile > "$O/yahoo_trace.json" 2> "$O/yahoo_trace.err" \
    || { echo trace bench failed; tail -3 "$O/yahoo_trace.err"; exit 1; }
  python tools/sys_trace.py /tmp/yahoo.trace > "$O/yahoo.sys.txt" && python tools/crowd_trace.py /tmp/yahoo.trace > "$O/yahoo.crowd.txt"
  rm -f /tmp/yahoo.trace
  head -4 "$O/yahoo.sys.txt"; cat "$O/yahoo.crowd.txt"
fi
