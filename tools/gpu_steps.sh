#!/bin/bash
# GPU-box step runner (replaces the one-off per-experiment scripts).  Usage, from gpurun:
#   TAG=r4a bash tools/gpu_steps.sh ubench prof1 trace bench ...
# Each step has its own time limit; the first failure ends the call (no further GPU step after a fault).
# Outputs go to gpurun_out/$TAG/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-steps}
mkdir -p $OUT
BENCH="python3 -u bench.py"

summ() {   # one line from a bench JSON
  python3 - "$1" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline", {})
print(d.get("value"), "ZMWs/s", "gcups", d.get("gcups"), "ms/step", d.get("ms_per_step"),
      "dom", r.get("kernel"), "avg_ms", r.get("avg_launch_ms"), "frac", r.get("frac"), "in_flight", r.get("in_flight"))
EOF
}

step() {
  local s=$1
  case $s in
    ubench)   # chain-step variants (tools/ubench/chain_step.hip, built in-tree beforehand)
      timeout -k 10 120 tools/ubench/chain_step > $OUT/ubench.txt 2>&1 && cat $OUT/ubench.txt ;;
    tests)    # -v -u: each test's name reaches the log as it starts, so a hang names its test
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1; local rc=$?; tail -3 $OUT/pytest_gpu.log; return $rc ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log ;;
    evidence) # the round's committed inputs of the bench line, then the line: PMC traffic and VALU passes and the
              # single-slot run of the final sources copied to profiles/ under the names bench.py reads, then the
              # driver's command and the occupancy build's
      step traffic && for k in fill_tall fill score; do cp $OUT/traffic_$k.json profiles/r6_traffic_$k.json; done && \
        step valu && cp $OUT/valu_per_cell.json profiles/r6_valu_per_cell.json && \
        step binding && cp $OUT/binding_summary.json profiles/r6_binding_summary.json && \
        step occ && cp $OUT/bench_occ.json profiles/r6_occupancy_bench.json && \
        step bench1 && cp $OUT/bench_streams1.json profiles/r6_streams1_bench.json && step bench ;;
    apiccs)   # HIP API trace of the ccs stage (no counters): calls per API, e.g. no hipDeviceSynchronize in steady state
      timeout -k 10 500 rocprofv3 --hip-trace --stats -f csv -d $OUT/apiccs -o run -- $BENCH --stage ccs --steps 5 \
        --warmup 1 --cpu-sample 0 > $OUT/ccs_api.json 2> $OUT/ccs_api.err && \
        cp "$(find $OUT/apiccs -name '*hip_api_stats.csv' | head -1)" $OUT/ccs_hip_api_stats.csv && \
        grep -E "hipDeviceSynchronize|hipFree\"|hipMalloc\"|hipStreamSynchronize|hipMemcpyAsync" $OUT/ccs_hip_api_stats.csv | cut -c1-120 ;;
    bench2r)  # the headline on two self-launched ranks pinned to the one device (a rehearsal of --gpus N)
      PBCCS_BENCH_DEVICE=0 timeout -k 10 400 $BENCH --gpus 2 --steps 4 --warmup 1 --streams 4 > $OUT/bench_2ranks.json \
        2> $OUT/bench_2ranks.err && summ $OUT/bench_2ranks.json && \
        python3 -c "import json; d=json.load(open('$OUT/bench_2ranks.json')); print(d['n_gpus'], d['scaling'], d.get('parity_sample', {}).get('ok'))" ;;
    bench)    # the driver's command
      timeout -k 10 400 $BENCH --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && summ $OUT/bench.json ;;
    bench5)
      timeout -k 10 300 $BENCH --steps 5 --warmup 1 --cpu-sample 0 > $OUT/bench5.json 2> $OUT/bench5.err && summ $OUT/bench5.json ;;
    prof)     # rocprofv3 kernel summary of the driver's command
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- $BENCH --gpus 1 --steps 20 \
        --warmup 5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err && summ $OUT/bench_prof.json && \
        cp "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" $OUT/kernel_stats.csv ;;
    prof1)    # single slot: kernel durations that are not time-shared
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof1 -o run -- $BENCH --streams 1 --steps 5 \
        --warmup 1 --cpu-sample 0 > $OUT/bench_streams1_prof.json 2> $OUT/bench_streams1_prof.err && \
        summ $OUT/bench_streams1_prof.json && \
        cp "$(find $OUT/prof1 -name '*kernel_stats.csv' | head -1)" $OUT/streams1_kernel_stats.csv ;;
    bench1)   # single slot, no profiler
      timeout -k 10 300 $BENCH --streams 1 --steps 5 --warmup 1 > $OUT/bench_streams1.json \
        2> $OUT/bench_streams1.err && summ $OUT/bench_streams1.json ;;
    trace)    # per-round trace of the driver's command (phase walls per batch round, fill launch sets)
      PBCCS_ROUND_TRACE=1 PBCCS_FILL_PATHS=1 timeout -k 10 400 $BENCH --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 \
        > $OUT/trace.json 2> $OUT/trace.err && summ $OUT/trace.json ;;
    trace1)   # the same, single slot
      PBCCS_ROUND_TRACE=1 PBCCS_FILL_PATHS=1 timeout -k 10 300 $BENCH --streams 1 --steps 5 --warmup 1 --cpu-sample 0 \
        > $OUT/trace1.json 2> $OUT/trace1.err && summ $OUT/trace1.json ;;
    quiver)
      PBCCS_QUIVER_TRACE=1 timeout -k 10 300 $BENCH --stage quiver --steps 5 --warmup 2 > $OUT/quiver.json 2> $OUT/quiver.err && \
        python3 -c "import json; d=json.load(open('$OUT/quiver.json')); print('quiver', d['value'], 'warmup_call_ms', d.get('warmup_call_ms'), 'timed_call_ms', d.get('timed_call_ms'))" ;;
    poa)
      timeout -k 10 400 $BENCH --stage poa --steps 5 --warmup 1 > $OUT/poa.json 2> $OUT/poa.err && \
        python3 -c "import json; d=json.load(open('$OUT/poa.json')); print('poa', d['value'])" ;;
    ccs)
      PBCCS_CCS_TRACE=1 timeout -k 10 500 $BENCH --stage ccs --steps 5 --warmup 1 > $OUT/ccs.json 2> $OUT/ccs.err && \
        python3 -c "import json; d=json.load(open('$OUT/ccs.json')); print('ccs', d['value'], d['zmw_status'])" ;;
    prof10k)  # configs[2] at 2000 ZMWs through the work queue, rocprofv3 kernel summary
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof10k -o run -- $BENCH --workload 10kb \
        --steps 1 --zmws-per-step 2000 --warmup 0 > $OUT/bench_10kb.json 2> $OUT/bench_10kb.err && \
        summ $OUT/bench_10kb.json && \
        cp "$(find $OUT/prof10k -name '*kernel_stats.csv' | head -1)" $OUT/10kb_kernel_stats.csv ;;
    bench10k) # configs[2] at ZMWS10K ZMWs (default 10000), no profiler, progress on stderr
      timeout -k 10 1000 $BENCH --workload 10kb --steps 1 --zmws-per-step ${ZMWS10K:-10000} --warmup 0 \
        > $OUT/bench_10kb_big.json 2> $OUT/bench_10kb_big.err && summ $OUT/bench_10kb_big.json ;;
    mixed)    # configs[3] at 2000 ZMWs
      timeout -k 10 900 $BENCH --workload mixed --steps 1 --zmws-per-step 2000 --warmup 0 > $OUT/bench_mixed.json \
        2> $OUT/bench_mixed.err && summ $OUT/bench_mixed.json ;;
    abmixed)  # configs[3] at MIXN ZMWs under each "VAR=x VAR2=y" variant of VARIANTS (";"-separated), no profiler
      local k=0
      IFS=';' read -ra VS <<< "${VARIANTS:-NONE=1}"
      for v in "${VS[@]}"; do
        k=$((k+1))
        ( eval "export $v"; timeout -k 10 600 $BENCH --workload mixed --steps 1 --zmws-per-step ${MIXN:-1000} --warmup 0 \
          --streams ${MIXSTREAMS:-8} ${MIXARGS:-} ) > $OUT/abmixed_$k.json 2> $OUT/abmixed_$k.err || \
          { echo "variant $k ($v) failed"; tail -3 $OUT/abmixed_$k.err; return 1; }
        echo "[$v] $(summ $OUT/abmixed_$k.json) $(python3 -c "import json; d=json.load(open('$OUT/abmixed_$k.json')); print('polished', d['polished'], 'parity', d.get('parity_sample', {}).get('ok'))")"
      done ;;
    apimixed) # configs[3] HIP API trace: which calls block a slot thread between its kernels (tools/api_gaps.py)
      timeout -k 10 1000 rocprofv3 --hip-trace --kernel-trace --stats -f csv -d $OUT/apimixed -o run -- $BENCH \
        --workload mixed --steps 1 --zmws-per-step ${MIXN:-2000} --warmup 0 --streams 8 --cpu-sample 0 \
        > $OUT/bench_mixed_api.json 2> $OUT/bench_mixed_api.err && summ $OUT/bench_mixed_api.json && \
        python3 tools/api_gaps.py "$(find $OUT/apimixed -name '*hip_api_trace.csv' | head -1)" 200 > $OUT/api_gaps.json && \
        head -60 $OUT/api_gaps.json && rm -f "$(find $OUT/apimixed -name '*hip_api_trace.csv' | head -1)" ;;
    profmixed) # configs[3] at 2000 ZMWs on 8 slots under rocprofv3 (the line and its kernel summary in one run)
      timeout -k 10 1000 rocprofv3 --kernel-trace --stats -f csv -d $OUT/profmixed -o run -- $BENCH --workload mixed \
        --steps 1 --zmws-per-step 2000 --warmup 0 --streams 8 > $OUT/bench_mixed.json 2> $OUT/bench_mixed.err && \
        summ $OUT/bench_mixed.json && \
        cp "$(find $OUT/profmixed -name '*kernel_stats.csv' | head -1)" $OUT/mixed_kernel_stats.csv ;;
    cell2)    # configs[4]: two ranks sharing the one device (a rehearsal of the multi-rank queue), CELLN ZMWs
      PBCCS_BENCH_DEVICE=0 timeout -k 10 ${CELLTO:-1000} $BENCH --gpus 2 --workload smrtcell --steps 1 \
        --zmws-per-step ${CELLN:-10000} --warmup 0 --streams 4 > $OUT/bench_cell2.json 2> $OUT/bench_cell2.err && \
        summ $OUT/bench_cell2.json ;;
    ab_tall)  # interleaved A/B of the tall fill's layout: "G:rows" (PBCCS_TALL_G, PBCCS_TALL_ROWS), 10 steps each
      local k=0
      for v in ${VARIANTS:-64:2 64:1 64:2 64:1}; do
        k=$((k+1))
        PBCCS_TALL_G=${v%:*} PBCCS_TALL_ROWS=${v#*:} timeout -k 10 300 $BENCH --steps 10 --warmup 2 --cpu-sample 0 \
          > $OUT/ab_tall_$k.json 2> $OUT/ab_tall_$k.err || return 1
        echo "tall=$v $(summ $OUT/ab_tall_$k.json)"
      done ;;
    tests_sel)    # the GPU tests of the files in TESTS only
      timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 150 --timeout-method thread \
        > $OUT/pytest_sel.log 2>&1; local rc=$?; tail -3 $OUT/pytest_sel.log; return $rc ;;
    tests_fill)   # the fill / checkpoint parity tests only
      timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_ckpt_gpu.py -m gpu -x -q --timeout 300 \
        --timeout-method thread > $OUT/pytest_fill.log 2>&1; local rc=$?; tail -3 $OUT/pytest_fill.log; return $rc ;;
    pmc)      # SQ / GRBM counters, one rocprofv3 pass per group (counter limits per pass: MI355X_MICROARCH.md)
      local i=0
      for g in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
        i=$((i+1))
        timeout -s KILL 240 rocprofv3 --pmc $g -f csv -d $OUT/pmc$i -o pmc -- $BENCH --cpu-sample 0 --no-profile --steps 5 \
          --warmup 1 > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "pmc pass $i failed"; return 1; }
      done
      python3 tools/pmc_summary.py $(find $OUT/pmc1 $OUT/pmc2 -name '*counter_collection.csv') > $OUT/pmc_summary.txt && \
        head -60 $OUT/pmc_summary.txt ;;
    valu)     # VALU instructions per counted cell and LDS bank conflicts per kernel: one SQ pass with profiling on
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
        -f csv -d $OUT/valu -o pmc -- $BENCH --cpu-sample 0 --steps 5 --warmup 1 > $OUT/valu.json 2> $OUT/valu.err \
        || { echo "valu pass failed"; return 1; }
      python3 tools/valu_per_cell.py "$(find $OUT/valu -name '*counter_collection.csv' | head -1)" $OUT/valu.json \
        $OUT/valu_per_cell.json "$(python3 -c 'import bench; print(bench.kernel_source_digest())')" ;;
    binding)  # wave-cycle decomposition per kernel family (issuing / issue-stalled / parked), CU busy, L2 hit rate:
              # one pass of 8 SQ + 1 GRBM + 2 TCC counters (tools/binding.py)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY \
        SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum \
        -f csv -d $OUT/binding -o pmc -- $BENCH --cpu-sample 0 --steps 3 --warmup 1 > $OUT/binding.json \
        2> $OUT/binding.err || { echo "binding pass failed"; tail -5 $OUT/binding.err; return 1; }
      python3 tools/binding.py "$(find $OUT/binding -name '*counter_collection.csv' | head -1)" $OUT/binding_summary.json \
        "$(python3 -c 'import bench; print(bench.kernel_source_digest())')" ;;
    work)     # where the fills' computed cells go (PBCCS_FILL_WORK=1 in-kernel counters), the driver's shape, 5 steps
      PBCCS_FILL_WORK=1 timeout -k 10 300 $BENCH --steps 5 --warmup 1 --cpu-sample 0 > $OUT/work.json 2> $OUT/work.err && \
        python3 -c "import json; d=json.load(open('$OUT/work.json')); print(d['value'], json.dumps(d.get('fill_work')))" ;;
    traffic)  # HBM bytes of the fills and k_score: FETCH_SIZE and WRITE_SIZE passes (they do not fit one pass)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o pmc -- $BENCH --cpu-sample 0 --steps 5 \
        --warmup 1 > $OUT/fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; return 1; }
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o pmc -- $BENCH --cpu-sample 0 --steps 5 \
        --warmup 1 > $OUT/write.json 2> $OUT/write.err || { echo "write pass failed"; return 1; }
      local F W
      F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
      W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
      for k in k_fill_tall k_fill k_score; do
        python3 tools/pmc_traffic.py "$F" "$W" $OUT/fetch.json $OUT/traffic_${k#k_}.json $k > /dev/null || echo "no $k dispatches"
      done
      cat $OUT/traffic_fill_tall.json; gzip -f "$F" "$W" ;;
    ab_lib)   # interleaved A/B of two in-tree builds (PBCCS_LIB; LIBS="a b" paths), 10 steps each, plus k_score / fill ms
      local k=0
      for rep in 1 2; do
        for v in ${LIBS:-pbccs_amd/_lib/libpbccs_amd.so pbccs_amd/_lib_ab/libpbccs_amd.so} ; do
          k=$((k+1))
          PBCCS_LIB=$v timeout -k 10 300 $BENCH --steps 10 --warmup 2 --cpu-sample 0 ${ABARGS:-} > $OUT/ab_lib_$k.json \
            2> $OUT/ab_lib_$k.err || return 1
          echo "lib=$v $(summ $OUT/ab_lib_$k.json) $(python3 -c "import json; d=json.load(open('$OUT/ab_lib_$k.json')); print({n: round(v['device_ms']/max(1,v['launches']),2) for n,v in d['kernels'].items() if n in ('k_score','k_fill','k_fill_tall','k_suffix')})")"
        done
      done ;;
    occ)      # the driver's command on the occupancy build (wave stamps on: built by
              # AB_FLAGS="-DPBCCS_WAVE_STAMPS=1" AB_OUT=pbccs_amd/_lib_occ tools/build_ab.sh HEAD): roofline.occupancy
      PBCCS_LIB=pbccs_amd/_lib_occ/libpbccs_amd.so timeout -k 10 400 $BENCH --gpus 1 --steps 20 --warmup 5 \
        > $OUT/bench_occ.json 2> $OUT/bench_occ.err && summ $OUT/bench_occ.json && \
        python3 -c "import json; d=json.load(open('$OUT/bench_occ.json')); print(json.dumps(d['roofline'].get('occupancy')))" ;;
    ab_tree)  # interleaved A/B of whole trees (git worktrees of older revisions under _ab/, built in-tree): TREES="a b"
      local k=0
      for rep in 1 2; do
        for v in ${TREES:-. _ab/be29dbd}; do
          k=$((k+1))
          (cd $v && timeout -k 10 300 python3 -u bench.py --steps ${ABSTEPS:-10} --warmup 2 --cpu-sample 0 ${ABARGS:-}) \
            > $OUT/ab_tree_$k.json 2> $OUT/ab_tree_$k.err || return 1
          echo "tree=$v $(summ $OUT/ab_tree_$k.json)"
        done
      done ;;
    ab_env)   # interleaved A/B of environment settings: ENVS="A=1 A=0" (one KEY=VALUE per variant; "-" = none), 2 runs each
      local k=0
      for rep in 1 2; do
        for v in ${ENVS:-PBCCS_TALL_PRIO=1 PBCCS_TALL_PRIO=0}; do
          k=$((k+1))
          env ${v/#-/PBCCS_NONE=1} timeout -k 10 300 $BENCH --steps ${ABSTEPS:-10} --warmup 2 --cpu-sample 0 ${ABARGS:-} \
            > $OUT/ab_env_$k.json 2> $OUT/ab_env_$k.err || return 1
          echo "$v $(summ $OUT/ab_env_$k.json) $(python3 -c "import json; d=json.load(open('$OUT/ab_env_$k.json')); print({n: round(v['device_ms']/max(1,v['launches']),2) for n,v in d['kernels'].items() if n in ('k_score','k_fill','k_fill_tall')})")"
        done
      done ;;
    ab_args)  # interleaved A/B of bench arguments: ARGV="--streams 7;--streams 8" (';' between variants), 2 runs each
      local k=0
      IFS=';' read -ra VS <<< "${ARGV:---streams 8;--streams 7}"
      for rep in 1 2; do
        for v in "${VS[@]}"; do
          k=$((k+1))
          timeout -k 10 300 $BENCH --steps ${ABSTEPS:-20} --warmup 3 --cpu-sample 0 $v > $OUT/ab_args_$k.json \
            2> $OUT/ab_args_$k.err || return 1
          echo "[$v] $(summ $OUT/ab_args_$k.json)"
        done
      done ;;
    ab_ccs)   # interleaved A/B of the ccs stage's shape: CCSV="slots:chunk ..." (0 = the defaults), 2 runs each
      local k=0
      for rep in 1 2; do
        for v in ${CCSV:-0:0 8:1000}; do
          k=$((k+1))
          timeout -k 10 300 $BENCH --stage ccs --steps 5 --warmup 1 --cpu-sample 0 --streams ${v%:*} \
            --ccs-chunk ${v#*:} > $OUT/ab_ccs_$k.json 2> $OUT/ab_ccs_$k.err || return 1
          echo "ccs slots:chunk=$v $(python3 -c "import json; d=json.load(open('$OUT/ab_ccs_$k.json')); print(d['value'], d['config']['slots'], d['poa_wall_ms'], d['poa_device_ms'])")"
        done
      done ;;
    fillread) # per-launch slowest-read diagnostics (PBCCS_FILL_PATHS=2), single slot, per rows-per-lane setting
      local k=0
      for v in ${VARIANTS:-64:2 64:1}; do
        k=$((k+1))
        PBCCS_TALL_G=${v%:*} PBCCS_TALL_ROWS=${v#*:} PBCCS_FILL_PATHS=2 PBCCS_ROUND_TRACE=1 timeout -k 10 300 $BENCH \
          --streams 1 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/fillread_$k.json 2> $OUT/fillread_$k.err || return 1
        echo "tall=$v $(summ $OUT/fillread_$k.json)"; grep "path=2" $OUT/fillread_$k.err | tail -12
      done ;;
    *)
      echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  t0=$(date +%s)
  echo "== $s"
  step $s || { echo "step $s failed (rc $?)"; tail -20 $OUT/*.err 2>/dev/null | tail -40; exit 1; }
  echo "   ($(( $(date +%s) - t0 )) s)"
done
