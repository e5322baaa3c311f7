#!/bin/bash
# Round 6 GPU pass, parametrised: TAG names the output directory
# (gpurun_out/$TAG); DO lists what to run (tests bench pmc valu elect cmp tlb trace smoke ...).
#   TESTS   pytest selection (-k expression) for the tests step ("" = all -m gpu)
#   BENCH   extra bench.py arguments
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6_dev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for st in ${DO:-tests bench}; do
  case $st in
    tests)
      echo "== tests ${TESTS:-all}"
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; exit 1; } ;;
    bench)
      echo "== bench ${BENCH:-}"
      timeout -k 10 600 python3 -u bench.py ${BENCH:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; tail -4 "$OUT/bench.err"; [ $rc -eq 0 ] || exit 1
      python3 tools/summarize_bench.py "$OUT/bench.json" ;;
    bench2|bench3)
      # another bench line in the same call (A/B on the same box): BENCH2 / BENCH3 arguments
      eval "args=\${$(echo $st | tr a-z A-Z):-}"
      echo "== $st $args"
      timeout -k 10 600 python3 -u bench.py $args > "$OUT/$st.json" 2> "$OUT/$st.err"
      rc=$?; tail -2 "$OUT/$st.err"; [ $rc -eq 0 ] || exit 1
      python3 tools/summarize_bench.py "$OUT/$st.json" ;;
    abbench)
      # headline A/B of library variants (tools/variants/libmraft_hip_<tag>.so, ABLIBS tags) against
      # the in-tree library: interleaved bench lines without the secondary legs
      echo "== abbench ${ABLIBS:-}"
      for pass in 1 2 3; do
        for t in ${ABLIBS:-} in-tree; do
          if [ "$t" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$t.so; fi
          timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline ${BENCH:-} > "$OUT/ab_${t}_$pass.json" 2> "$OUT/ab_${t}_$pass.err" \
            || { tail -3 "$OUT/ab_${t}_$pass.err"; exit 1; }
          python3 -c "import json; d=json.loads(open('$OUT/ab_${t}_$pass.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$t', $pass, round(d['ms_per_step'], 4), r.get('frac'), r.get('kernel_ms_mean'))"
        done
      done
      unset MRAFT_LIB ;;
    deferred)
      # the deferred-heavy handle measurement alone (tools/bench_deferred.py)
      echo "== deferred"
      timeout -k 10 400 python3 tools/bench_deferred.py > "$OUT/deferred.json" 2> "$OUT/deferred.err" || { tail -5 "$OUT/deferred.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/deferred.json').read().strip().splitlines()[-1]); [print(k, round(v['ms_per_call'], 4), round(v['first_call_ms'], 3), round(v.get('vs_plain', 1.0), 3)) for k, v in d.items()]" ;;
    steady)
      # the steady-state ticks alone, full and light (tools/bench_steady.py)
      echo "== steady"
      timeout -k 10 400 python3 tools/bench_steady.py > "$OUT/steady.json" 2> "$OUT/steady.err" || { tail -5 "$OUT/steady.err"; exit 1; }
      python3 -c "import json; e=json.loads(open('$OUT/steady.json').read().strip().splitlines()[-1]); li=e['light']; print('full', round(e['tick_ms_steady'],4), 'light', round(li['tick_ms_steady'],4), 'x', round(li['speedup_tick_steady'],2), 'same', li['state_equals_full'], 'fb', li['fallback_groups_steps']); fu=e['fused']; print('per step: full start+tick', round(e['device_ms_per_step_steady'],4), 'light start+tick', round(li['device_ms_per_step_steady'],4), 'fused', round(fu['device_ms_per_step_steady'],4), 'same', fu['state_equals_full'])" ;;
    lighttests)
      # the whole tick-related GPU suite with every engine in MRAFT_TICK_LIGHT (tests/conftest.py)
      echo "== lighttests"
      MRAFT_TEST_TICK_MODE=light timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${LTESTS:-(tick or persist or ring or odd or index or snapshot or sim or multirank) and not mode_calls}" > "$OUT/pytest_light.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest_light.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$OUT/pytest_light.log" | head -20; exit 1; } ;;
    ktrace)
      # kernel trace + stats of a tool (KT_CMD, e.g. tools/bench_steady.py) -> $OUT/kt_<name>, per-kernel summary
      name=$(basename "${KT_CMD%% *}" .py)
      echo "== ktrace $KT_CMD"
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$name" -o kt -- python3 $KT_CMD \
        > "$OUT/kt_$name.json" 2> "$OUT/kt_$name.err" || { tail -5 "$OUT/kt_$name.err"; exit 1; }
      f=$(find "$OUT/kt_$name" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -25 "$f" | cut -d, -f1-8 ;;
    pmcsteady)
      # counters of the steady-state ticks (tools/bench_steady.py), one pass per group -> $OUT/steady_counters.json
      echo "== pmcsteady"
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" \
                 "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pst$i" -o p -- python3 tools/bench_steady.py \
          > "$OUT/pst$i.json" 2> "$OUT/pst$i.err" || { tail -5 "$OUT/pst$i.err"; exit 1; }
      done
      python3 tools/pmc_kernels.py "$OUT/steady_counters.json" "$OUT"/pst[0-9]* --kernels "k_tick_lite<5, false>;k_tick_lite<5, true>;k_tick_list<5>;k_tick_group<5, false>;k_tick_group<5, true>" | head -60 ;;
    abdeferred)
      # the deferred-heavy handle measurement per library variant (ABDEF_LIBS tags + in-tree)
      echo "== abdeferred ${ABDEF_LIBS:-}"
      for t in ${ABDEF_LIBS:-} in-tree; do
        if [ "$t" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$t.so; fi
        timeout -k 10 400 python3 tools/bench_deferred.py > "$OUT/abdef_$t.json" 2> "$OUT/abdef_$t.err" || { tail -5 "$OUT/abdef_$t.err"; exit 1; }
        python3 -c "import json; d=json.loads(open('$OUT/abdef_$t.json').read().strip().splitlines()[-1]); print('$t', {k: (round(v['first_call_ms'], 2), round(v['ms_per_call'], 4)) for k, v in d.items()})"
      done
      unset MRAFT_LIB ;;
    abmsg)
      # message path A/B of library variants (tools/build_variants.sh, VARIANTS="tag=DEFINES ...")
      echo "== abmsg ${VARIANTS:-prebuilt}"
      # (variants prebuilt here with tools/build_variants.sh travel in tools/variants/)
      [ -z "${VARIANTS:-}" ] || { (cd tools && eval "bash build_variants.sh $VARIANTS") > "$OUT/variants_build.log" 2>&1 || { tail -5 "$OUT/variants_build.log"; exit 1; }; }
      for pass in 1 2; do
        for lib in ${ABMSG_LIBS-tools/variants/*.so} in-tree; do
          [ "$lib" = in-tree ] || [ -e "$lib" ] || continue  # no variants built: in-tree only
          if [ "$lib" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/$lib; fi
          timeout -k 10 300 python3 tools/ab_message_path.py >> "$OUT/abmsg.jsonl" 2>> "$OUT/abmsg.err" || { tail -5 "$OUT/abmsg.err"; exit 1; }
        done
      done
      unset MRAFT_LIB; cat "$OUT/abmsg.jsonl" ;;
    abtick)
      # tick A/B with FETCH/WRITE passes (tools/ab_tick_pmc.sh; LIBS = variant tags)
      echo "== abtick ${LIBS:-all}"
      TAG=$TAG/abtick bash tools/ab_tick_pmc.sh > "$OUT/abtick.log" 2>&1; rc=$?
      tail -40 "$OUT/abtick.log"; [ $rc -eq 0 ] || exit 1 ;;
    tracemsg)
      # message-path device timeline (tools/timeline.py): busy / idle / overlap per gated section
      echo "== tracemsg"
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/msgkt" -o msgkt -- python3 tools/ab_message_path.py \
        > "$OUT/msgkt.json" 2> "$OUT/msgkt.err" || { tail -5 "$OUT/msgkt.err"; exit 1; }
      python3 tools/timeline.py "$OUT/msgkt" "$OUT/timeline.json" > /dev/null && python3 -c "import json; [print({k: v for k, v in s.items() if k != 'per_kernel'}) for s in json.load(open('$OUT/timeline.json'))]" ;;
    pmcmsg)
      # message-path HBM bytes per kernel (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_msg.py)
      echo "== pmcmsg"
      for c in FETCH_SIZE WRITE_SIZE; do
        SHARDS=2 timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$OUT/msgpmc_$c" -o p -- python3 tools/ab_message_path.py \
          > "$OUT/msgpmc_$c.json" 2> "$OUT/msgpmc_$c.err" || { tail -5 "$OUT/msgpmc_$c.err"; exit 1; }
      done
      python3 tools/pmc_msg.py "$OUT/msgpmc_FETCH_SIZE" "$OUT/msgpmc_WRITE_SIZE" "$OUT/msgpmc.json" ;;
    pmc)
      # FETCH_SIZE / WRITE_SIZE passes of the bench (BENCH_EXTRA) + calibration -> profiles/pmc_traffic*.json
      echo "== pmc ${BENCH_EXTRA:-}"
      rm -rf gpurun_out/prof
      BENCH_EXTRA="--no-secondary ${BENCH_EXTRA:-}" bash tools/profile_round.sh > "$OUT/profile.log" 2>&1 || { tail -5 "$OUT/profile.log"; exit 1; }
      python3 tools/pmc_summary.py "$TAG" > "$OUT/pmc_summary.log" 2>&1 || { tail -5 "$OUT/pmc_summary.log"; exit 1; }
      mkdir -p "$OUT/pmc"; cp profiles/pmc_traffic*.json profiles/${TAG}_*.csv "$OUT/pmc/" 2>/dev/null
      grep -E '"(hbm_bytes_per_step|traffic_over_algorithmic|shards|groups)"' "$OUT/pmc_summary.log" ;;
    valu)
      # SQ counters of the election storm (config #5) -> profiles/pmc_valu_config5.json
      echo "== valu"
      timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/valu" -o valu -- python3 bench_election.py --no-cpu-baseline --steps 5 \
        > "$OUT/valu_bench.json" 2> "$OUT/valu_bench.err" || { tail -5 "$OUT/valu_bench.err"; exit 1; }
      timeout -k 10 300 python3 bench_election.py --no-cpu-baseline > "$OUT/election_bench.json" 2> "$OUT/election_bench.err" || exit 1
      python3 tools/pmc_valu.py "$TAG" "$OUT/valu" "$OUT/election_bench.json" | tee "$OUT/pmc_valu.log" | grep -E "frac|busy|SQ_INSTS_VALU"
      cp profiles/pmc_valu_config5.json "$OUT/" ;;
    elect)
      # where the election storm's issue slots go: stall and LDS counters of
      # k_election_rounds<7>, one pass per counter group
      echo "== elect"
      i=0
      for grp in "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
                 "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/elect$i" -o e -- python3 bench_election.py --no-cpu-baseline --steps 5 \
          > "$OUT/elect$i.json" 2> "$OUT/elect$i.err" || { tail -5 "$OUT/elect$i.err"; exit 1; }
      done
      python3 tools/pmc_kernels.py "$OUT/elect_counters.json" "$OUT"/elect1 "$OUT"/elect2 --kernels "k_election_rounds<7>" | head -40 ;;
    abelect)
      # election storm A/B of library variants (tools/variants/libmraft_hip_<tag>.so, ABELECT_LIBS tags)
      echo "== abelect ${ABELECT_LIBS:-}"
      for pass in 1 2 3; do
        for t in ${ABELECT_LIBS:-} in-tree; do
          if [ "$t" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$t.so; fi
          timeout -k 10 200 python3 bench_election.py --no-cpu-baseline > "$OUT/abelect_${t}_$pass.json" 2> "$OUT/abelect_${t}_$pass.err" \
            || { tail -3 "$OUT/abelect_${t}_$pass.err"; exit 1; }
          python3 -c "import json; d=json.loads(open('$OUT/abelect_${t}_$pass.json').read().strip().splitlines()[-1]); print('$t', $pass, round(d['ms_per_step'], 4), d['roofline'].get('frac'))"
        done
      done
      unset MRAFT_LIB ;;
    cmp)
      # the tick and the handler on the same state copy, counters per kernel
      echo "== cmp"
      timeout -k 10 300 python3 tools/cmp_tick_handler.py > "$OUT/cmp_times.json" 2> "$OUT/cmp_times.err" || { tail -5 "$OUT/cmp_times.err"; exit 1; }
      cat "$OUT/cmp_times.json"
      i=0
      for grp in "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
                 "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE" "WRITE_SIZE" \
                 "TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL" \
                 "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"; do
        i=$((i+1))
        REPS=3 timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/cmp$i" -o c -- python3 tools/cmp_tick_handler.py \
          > "$OUT/cmp$i.json" 2> "$OUT/cmp$i.err" || { tail -5 "$OUT/cmp$i.err"; exit 1; }
      done
      python3 tools/pmc_kernels.py "$OUT/cmp_counters.json" "$OUT"/cmp[0-9]* --kernels "k_tick_group<5, false>;k_handle_set<4, 0>;k_handle_deferred;k_gather_args;k_claim_ae" > /dev/null
      python3 tools/cmp_summary.py "$OUT" "$OUT/cmp_summary.json" | head -60 ;;
    tlb)
      # address-translation counters of the message path's kernels: are the gather's and the
      # fold's dependent round trips stretched by UTCL1 misses? k_handle_set
      # (row streams) is the comparison
      echo "== tlb"
      i=0
      for grp in "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE" \
                 "TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum"; do
        i=$((i+1))
        SHARDS=1 timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/tlb$i" -o t -- python3 tools/ab_message_path.py \
          > "$OUT/tlb$i.json" 2> "$OUT/tlb$i.err" || { tail -5 "$OUT/tlb$i.err"; exit 1; }
      done
      python3 tools/pmc_kernels.py "$OUT/tlb_counters.json" "$OUT"/tlb1 "$OUT"/tlb2 \
        --kernels "k_gather_args;k_fold<5>;k_handle_set<4, 0>;k_claim_zero;k_claim_ae;k_fold_tail<5>" | head -80 ;;
    ctest)
      echo "== ctest"
      make -s -C tests/c_host && timeout -k 10 120 tests/c_host/mraft_host_tick tests/golden/tick_vectors.bin 0 | tee "$OUT/c_host.txt" ;;
    trace)
      # kernel trace + stats of the bench (BENCH) -> $OUT/kt
      echo "== trace ${BENCH:-}"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py ${BENCH:-} \
        > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || { tail -5 "$OUT/kt_bench.err"; exit 1; }
      python3 tools/summarize_bench.py "$OUT/kt_bench.json" ;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1; rc=$?; tail -2 "$OUT/smoke.txt"; [ $rc -eq 0 ] || exit 1 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done $TAG"
