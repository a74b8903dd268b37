#!/bin/bash
# One parameterised GPU runner for gpurun (replaces the per-experiment gpurun_*.sh scripts):
#
#   gpurun -- bash tools/gpu.sh <out-dir-name> <step> [<step> ...]
#
# Steps run in order, each under its own time limit; the first failure ends the call (nothing more
# touches the GPU after a fault, an abort or a time limit).  Outputs go to gpurun_out/<out-dir-name>/.
#   test:<pytest args>                     pytest -m gpu (one process), log test_<n>.log (args are
#                                          shell-parsed: quote a -k expression)
#   smoke                                  __graft_entry__.smoke()
#   bench:<tag>:<bench.py args>            one bench line -> <tag>.json, summary printed
#   ab:<tag>:<reps>:<envA>|<envB>[|...]:<bench.py args>
#                                          alternating A/B of environment settings on the bench line
#   prof:<tag>:<kernel>:<cfg>:<mode>:<rank>:<bench.py args>   (<kernel> may be k1=sfx1;k2=sfx2;...:
#                                          one traffic_<cfg>_<sfx>.json per kernel of the same run)
#                                          rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE
#                                          and --pmc WRITE_SIZE passes, summarised per launch of <kernel>
#                                          (tools/pmc_summary.py) -> traffic_<tag>.json, stats_<tag>.csv
#   pmc:<tag>:<counters>:<bench.py args>   one rocprofv3 --pmc pass (counters space-separated, within one
#                                          pass's block budget) -> pmc_<tag>/ (tools/pmc_breakdown.py)
#   rank:<world>:<rank_check.py args>      rank mode (RCCL ring) rehearsal on one GPU: <world> ranks share
#                                          device 0 with distinct RCCL host ids (MFHIP_FAKE_HOSTS), checked
#                                          against a single-process context (tools/rank_check.py)
#   micro:<src.hip>[:<hipcc flags>]        build a tools/micro benchmark and run it
#   calib                                  FETCH_SIZE / WRITE_SIZE vs known bytes of 512-B row gathers and
#                                          scatters (tools/micro/fetch_calib.hip) -> fetch_calib.json
#   cmd:<shell command>                    anything else (300 s limit)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:?out dir}
shift
mkdir -p "$O"
cd "$R"
n=0
summ() {  # one-line summary of a bench JSON line
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
det = d.get("deterministic") or {}
on = d.get("online") or {}
s = f"{d['config']['workload']}: {d['value']/1e9:.3f} Gups {d['ms_per_step']} ms/step rmse {d.get('rmse')} rel {d.get('rmse_rel')}"
if r: s += f" | launch {r.get('avg_launch_us')} us frac {r.get('frac')} requested {r.get('requested_frac')} traffic_frac {r.get('traffic_frac')}"
if det: s += f" | det {det['value']/1e6:.1f} Mups {det['ms_per_step']} ms eq {det.get('rmse_equal_to_ref')} launch {det.get('avg_launch_us')} us cold {det.get('cold_fit_s')}"
for key, v in on.items():
    ro = v.get("roofline") or {}
    s += f" | online {key} {v['value']/1e6:.1f} M/s kernel {v.get('kernel_ms_median')} ms frac {ro.get('frac')} alg {ro.get('algorithmic_frac')}"
print(s)
EOF
}
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=${step#*:}
  echo "== step $n: $step"
  case $kind in
    test)
      eval "timeout -k 10 1100 python -u -m pytest $rest -m gpu -v --timeout 300 --timeout-method thread" > "$O/test_$n.log" 2>&1 \
        || { echo "pytest failed"; grep -E "FAILED|Error|Timeout" "$O/test_$n.log" | head -20; tail -3 "$O/test_$n.log"; exit 1; }
      tail -1 "$O/test_$n.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      tag=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 900 python bench.py $args > "$O/$tag.json" 2> "$O/$tag.err" \
        || { echo "bench $tag failed"; tail -5 "$O/$tag.err"; exit 1; }
      summ "$O/$tag.json" ;;
    ab)
      tag=${rest%%:*}; rest=${rest#*:}
      reps=${rest%%:*}; rest=${rest#*:}
      vars=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      IFS='|' read -ra VARS <<< "$vars"
      for rep in $(seq 1 "$reps"); do
        for v in "${VARS[@]}"; do
          t="${tag}_$(echo "$v" | tr ' =/' '_-_')_$rep"
          env $v timeout -k 10 600 python bench.py $args > "$O/$t.json" 2> "$O/$t.err" \
            || { echo "ab run [$v] failed"; tail -5 "$O/$t.err"; exit 1; }
          echo "[$v] $(summ "$O/$t.json")"
        done
      done ;;
    prof)
      IFS=':' read -r tag kern cfg mode rank args <<< "$rest"
      cd /tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/kt_$tag" -o kt --output-format csv -- python3 "$R/bench.py" $args \
        > "$O/prof_kt_$tag.log" 2>&1 || { echo "kernel trace $tag failed"; tail -5 "$O/prof_kt_$tag.log"; exit 1; }
      timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$tag" -o fetch --output-format csv -- python3 "$R/bench.py" $args \
        > "$O/prof_fetch_$tag.log" 2>&1 || { echo "fetch $tag failed"; tail -5 "$O/prof_fetch_$tag.log"; exit 1; }
      timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$tag" -o write --output-format csv -- python3 "$R/bench.py" $args \
        > "$O/prof_write_$tag.log" 2>&1 || { echo "write $tag failed"; tail -5 "$O/prof_write_$tag.log"; exit 1; }
      cd "$R"
      stats=$(ls "$O"/kt_$tag/*kernel_stats.csv | head -1)
      cp "$stats" "$O/stats_$tag.csv"
      # <kernel> may list several kernels of the same run, kernel=suffix;...: each is summarised to
      # traffic_<cfg>_<suffix>.json (mode = suffix); a bare kernel name writes traffic_<tag>.json.  A
      # kernel may carry its template arguments (k_det_sweep_split<2, 1>: that instance only)
      IFS=';' read -ra KS <<< "$kern"
      for ks in "${KS[@]}"; do
        kn=${ks%%=*}; sfx=${ks#*=}
        if [ "$sfx" = "$ks" ]; then out="$O/traffic_$tag.json"; md=$mode; else out="$O/traffic_${cfg}_$sfx.json"; md=$sfx; fi
        python3 tools/pmc_summary.py --stats "$stats" --fetch $(ls "$O"/fetch_$tag/*counter_collection.csv | head -1) \
          --write $(ls "$O"/write_$tag/*counter_collection.csv | head -1) --kernel "$kn" --config "$cfg" --mode "$md" \
          --rank "$rank" --out "$out" > /dev/null || { echo "pmc summary $tag $kn failed"; exit 1; }
        echo "traffic $kn: $(tr -d '\n ' < "$out" | cut -c1-260)"
      done
      rm -rf "$O/fetch_$tag" "$O/write_$tag"
      head -6 "$O/stats_$tag.csv" | cut -c1-150 ;;
    pmc)
      IFS=':' read -r tag ctrs args <<< "$rest"
      cd /tmp
      timeout -s KILL 400 rocprofv3 --pmc $ctrs -d "$O/pmc_$tag" -o pmc --output-format csv -- python3 "$R/bench.py" $args \
        > "$O/pmc_$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -5 "$O/pmc_$tag.log"; exit 1; }
      cd "$R"
      echo "pmc $tag: $(ls "$O"/pmc_$tag/*counter_collection.csv | head -1)" ;;
    rank)
      w=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      MFHIP_FAKE_HOSTS=1 MFHIP_DEVICE_SHARERS=$w NCCL_DEBUG=WARN timeout -k 10 1100 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$w" --master-addr 127.0.0.1 --master-port $((29500 + n)) tools/rank_check.py $args \
        > "$O/rank_$n.log" 2>&1
      rc=$?
      grep -E "world=|RANK_CHECK|rank [0-9]+:|differing|superstep|STEPWISE|repeats|DIGEST|single context" "$O/rank_$n.log" | head -60
      # a failed bitwise comparison lets the next step run; anything else (a fault, an abort, a
      # time limit) ends the call
      [ $rc -eq 0 ] || { echo "rank check failed ($rc)"; tail -5 "$O/rank_$n.log";
                         grep -q "AssertionError: rank mode is not bit-exact" "$O/rank_$n.log" || exit 1; } ;;
    micro)
      src=${rest%%:*}; flags=${rest#*:}; [ "$flags" = "$rest" ] && flags=""
      b=$(basename "$src" .hip)
      hipcc -O3 --offload-arch=gfx950 $flags -o "$O/$b" "$src" > "$O/$b.build.log" 2>&1 \
        || { echo "micro build failed"; tail -5 "$O/$b.build.log"; exit 1; }
      timeout -k 10 120 "$O/$b" > "$O/$b.txt" 2>&1 || { echo "micro $b failed"; tail -5 "$O/$b.txt"; exit 1; }
      cat "$O/$b.txt" ;;
    calib)  # FETCH_SIZE / WRITE_SIZE against known bytes (tools/micro/fetch_calib.hip, tools/pmc_calib.py)
      hipcc -O3 --offload-arch=gfx950 -o "$O/fetch_calib" tools/micro/fetch_calib.hip > "$O/fetch_calib.build.log" 2>&1 \
        || { echo "calib build failed"; tail -5 "$O/fetch_calib.build.log"; exit 1; }
      timeout -k 10 120 "$O/fetch_calib" > "$O/fetch_calib.txt" 2>&1 || { echo "calib run failed"; tail -5 "$O/fetch_calib.txt"; exit 1; }
      cd /tmp
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o f --output-format csv -- "$O/fetch_calib" \
        > "$O/calib_fetch.log" 2>&1 || { echo "calib fetch pass failed"; tail -5 "$O/calib_fetch.log"; exit 1; }
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o w --output-format csv -- "$O/fetch_calib" \
        > "$O/calib_write.log" 2>&1 || { echo "calib write pass failed"; tail -5 "$O/calib_write.log"; exit 1; }
      cd "$R"
      python3 tools/pmc_calib.py --cases "$O/fetch_calib.txt" --fetch $(ls "$O"/calib_fetch/*counter_collection.csv | head -1) \
        --write $(ls "$O"/calib_write/*counter_collection.csv | head -1) --out "$O/fetch_calib.json" || { echo "calib summary failed"; exit 1; }
      rm -rf "$O/calib_fetch" "$O/calib_write" ;;
    cmd)
      timeout -k 10 300 bash -c "$rest" > "$O/cmd_$n.log" 2>&1 || { echo "cmd failed"; tail -10 "$O/cmd_$n.log"; exit 1; }
      tail -20 "$O/cmd_$n.log" ;;
    *)
      echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
