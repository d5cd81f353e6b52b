# Round 6's GPU calls, one case per call (gpurun runs it from the repository root):
#   bash tools/gpu/round6.sh NAME
# The A/B cases compare the in-tree build with tools/probe/*.so builds of the code
# they name (DESIGN.md records each result); kept so every number cited there has
# its command. final_evidence_a / final_evidence_b / final_stress are the final
# build's evidence (suite, stress, rocprofv3 profiles, bench line).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# a GPU step that timed out, aborted or faulted ends the call
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
case "$1" in
crash_race)
  # round 6: crash-mode parity + the GPU suite, then the phase-O race without its
  # per-pass store wait (diagnostics build, LNW_DEBUG_SKIP bit 25) with every wrong
  # block dumped for the offline source attribution (tools/race_chunks.py)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_crash_modes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/crash.log 2>&1
  rc=$?; tail -5 gpurun_out/crash.log; fatal $rc && exit $rc
  bash tools/gpu/tests.sh; rc=$?; fatal $rc && exit $rc
  RACE_REF_NOSPLIT=1 RACE_SKIP_BITS=33554432 RACE_DUMP=gpurun_out/race_dump.npz \
    LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so \
    timeout -k 10 600 python -u tools/contact_race.py 10 1 > gpurun_out/race_r06.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/race_r06.log | grep "^run\|dumped" | head -12
  exit $rc
  ;;
race_nowait)
  # round 6, second call: the phase-O race on the shipped code minus its store
  # wait (tools/probe/liblnw_nowait.so, -DLNW_PROBE_NO_OBS_WAIT) with every wrong
  # block dumped; the GPU suite; config 5's per-launch PMC; the default bench line
  RACE_REF_NOSPLIT=1 RACE_DUMP=gpurun_out/race_dump_nowait.npz LNW_LIB=$PWD/tools/probe/liblnw_nowait.so \
    timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_nowait.log 2>&1
  rc=$?; echo "no-wait race: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_nowait.log) of 60"
  grep "dumped" gpurun_out/race_nowait.log; fatal $rc && exit $rc
  bash tools/gpu/tests.sh; rc=$?; fatal $rc && exit $rc
  bash tools/gpu/c5_pmc.sh r06_config5; rc=$?; fatal $rc && exit $rc
  timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06b.json 2> gpurun_out/bench_r06b.err
  rc=$?; tail -c 600 gpurun_out/bench_r06b.json; exit $rc
  ;;
race_nowait_nt)
  # round 6, third call: the phase-O fault's dependence on write-through stores
  # (the no-wait probe with LNW_NO_STORE_WT: non-temporal global stores instead of
  # buffer_store ... sc1), the shipped build repeated, and the policy tile
  # read-back probe (13) beside the fault's reproduction (probe 10)
  LNW_NO_STORE_WT=1 RACE_REF_NOSPLIT=1 RACE_DUMP=gpurun_out/race_dump_nowait_nt.npz LNW_LIB=$PWD/tools/probe/liblnw_nowait.so \
    timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_nowait_nt.log 2>&1
  rc=$?; echo "no-wait, non-temporal stores: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_nowait_nt.log) of 60"; fatal $rc && exit $rc
  timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_prod.log 2>&1
  rc=$?; echo "shipped (wait, write-through): clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_prod.log) of 60"; fatal $rc && exit $rc
  : > gpurun_out/det_p13.log
  for d in 10 13; do
    POLICY_LIB=tools/probe/actor_disturb$d.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_p13.log 2>&1
    rc=$?; fatal $rc && exit $rc
  done
  grep "^lib\|mismatching\|probe stage" gpurun_out/det_p13.log
  ;;
policy_probe14)
  # round 6, fourth call: policy probe 14 (inside the victim MLP: its fc1
  # operands, its head outputs and per-row outputs against a rerun), then the
  # rollout tests and config 5's kernel trace on the build with the critic's fc1
  # loads all in flight
  POLICY_LIB=tools/probe/actor_disturb14.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed > gpurun_out/det_p14.log 2>&1
  rc=$?; grep "^lib\|mismatching\|probe stage" gpurun_out/det_p14.log; fatal $rc && exit $rc
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout_fullsize.py tests/test_gpu_obs_options.py > gpurun_out/ro_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/ro_tests.log; [ $rc -ne 0 ] && exit $rc
  bash tools/gpu/c5_trace.sh c5_post
  ;;
policy_probe15_16)
  # round 6: policy probes 15 (layers per row tile vs a rerun) and 16 (fc1 split terms, pre-activation)
  POLICY_LIB=tools/probe/actor_disturb16.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 20 packed > gpurun_out/det_p16.log 2>&1
  rc=$?; grep "^lib\|mismatching\|probe stage" gpurun_out/det_p16.log; exit $rc
  ;;
policy_probe16_c4fetch)
  # round 6: policy probe 16, then config 4's fetch attribution (tools/gpu/c4_fetch.sh)
  bash tools/gpu/round6.sh policy_probe15_16 || exit 1
  bash tools/gpu/c4_fetch.sh > gpurun_out/c4_fetch.txt 2>&1; rc=$?; cat gpurun_out/c4_fetch.txt; exit $rc
  ;;
policy_fence)
  # round 6: the policy fault against the split-before-MFMA fence: probe 10's
  # schedule (the partner's head beside each MLP) and the overlapped schedule
  # (each wave's MLP right after its own head) with and without the fence, then
  # the timing of base / fence / overlap+fence (tools/policy_probe.py)
  : > gpurun_out/det_fence.log
  for v in disturb10 disturb10_fence overlap overlap_fence fence; do
    POLICY_LIB=tools/probe/actor_$v.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_fence.log 2>&1 || exit 1
  done
  grep "^lib\|mismatching" gpurun_out/det_fence.log
  timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_base.so tools/probe/actor_fence.so tools/probe/actor_overlap_fence.so tools/probe/actor_base.so tools/probe/actor_fence.so tools/probe/actor_overlap_fence.so 2>&1 | grep "so {" 
  ;;
policy_tail_quads)
  # round 6: lnw_policy_act with the tail loaded as float4 quads (actor_tq) against
  # the per-value tail loads (actor_base): timing (tools/policy_probe.py, A/B/A/B)
  # and determinism of the new build
  timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_base.so tools/probe/actor_tq.so tools/probe/actor_base.so tools/probe/actor_tq.so tools/probe/actor_base.so tools/probe/actor_tq.so 2>&1 | grep "so {" || exit 1
  POLICY_LIB=tools/probe/actor_tq.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided,critic > gpurun_out/det_tq.log 2>&1 || exit 2
  grep "mismatching" gpurun_out/det_tq.log
  ;;
c4_rows_batched)
  # round 6: config 4's rows with batched window loads: A/B against the previous
  # build (tools/probe/liblnw_prev.so), then the group-kernel parity tests
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so littoral-naval-warfare-marl_amd/lnw/liblnw.so "--workload config4" || exit 1
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_fullsize.py tests/test_gpu_crash_modes.py tests/test_gpu_state.py > gpurun_out/grp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/grp_tests.log; exit $rc
  ;;
shard_timelines)
  # round 6: LNW_PROF timelines of the small shards (production build)
  bash tools/gpu/timeline.sh sh8192 "--global-envs 8192" || exit $?
  bash tools/gpu/timeline.sh sh4096 "--global-envs 4096" || exit $?
  ;;
quiet_columns_upfront)
  # round 6: quiet path with its LDS columns read up front (quiet test, rewards,
  # cog sums) against the previous build: interleaved A/B at the small shards and
  # the headline, the quiet/shard/units/parity tests, the new build's timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
  bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet workgroups|grid:|sh8192n"
  ;;
quiet_pairs_packed)
  # round 6: the quiet test's pair loop on packed 16-bit pairs (+ phase-Q stamps)
  # against the previous build: interleaved A/B, the quiet-path tests, timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
  bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
  ;;
quiet_only_probe)
  # round 6: the quiet path compiled without phase S (timing probe,
  # LNW_PROBE_QUIET_ONLY) against the production build, and its timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 2 $L tools/probe/liblnw_qonly.so "--global-envs 8192" "--global-envs 4096" "" || exit $?
  LNW_LIB=$PWD/tools/probe/liblnw_qonly.so bash tools/gpu/timeline.sh qonly8192 "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|qonly"
  ;;
quiet_test_spread)
  # round 6: the quiet test's pair loop on spread over (ship, env) lanes in small workgroups
  # against the previous build: interleaved A/B, the quiet-path tests, timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
  bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
  ;;
counters_at_launch)
  # round 6: env and draw counters loaded at launch in small quiet workgroups
  # against the previous build: interleaved A/B, the quiet-path tests, timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
  bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
  ;;
counters_knob)
  # round 6: small quiet workgroups' env / draw counters loaded at launch, A/B of
  # the knob (LNW_DEBUG_SKIP bit 29 = loaded in phase Q) at the shard sizes of
  # N = 16 / 8 / 4 GPUs, then the quiet-path tests and the 4 096-env timeline
  bash tools/gpu/ab_env.sh LNW_DEBUG_SKIP=536870912 3 "--global-envs 4096" "--global-envs 8192" "--global-envs 16384" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
  bash tools/gpu/timeline.sh sh4096n "--global-envs 4096" 2>&1 | grep -E "quiet|grid:|sh4096n"
  LNW_DEBUG_SKIP=536870912 bash tools/gpu/timeline.sh sh4096q "--global-envs 4096" 2>&1 | grep -E "quiet|grid:|sh4096q"
  ;;
evidence_first_a)
  # round 6 evidence, part A: the GPU suite + smoke(), then the rocprofv3 evidence
  # of the headline, the 8 192-env shard and config 2 (prof_all.sh part 1)
  bash tools/gpu/tests.sh || exit $?
  bash tools/gpu/prof_all.sh r06 1 || exit $?
  ;;
evidence_first_b)
  # round 6 evidence, part B: rocprofv3 evidence of melee, config 4 and config 5
  # (prof_all.sh part 2), then the default bench line
  bash tools/gpu/prof_all.sh r06 2 || exit $?
  timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06r.json 2> gpurun_out/bench_r06r.err
  rc=$?; tail -c 300 gpurun_out/bench_r06r.json; exit $rc
  ;;
sincos_probe)
  # round 6: what phase M's double sincos costs (timing probe with an f32
  # __sincosf in its place, results change) at the headline and the shard sizes
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 $L tools/probe/liblnw_fastsc.so "" "--global-envs 8192" "--global-envs 4096" || exit $?
  ;;
sincos_certified)
  # round 6: float32 move rows' sin / cos from a certified fast kernel
  # (sincos_f32_cert, library sincos when uncertain) against the previous build,
  # then the whole GPU suite
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 4096" "--spawns melee" || exit $?
  bash tools/gpu/tests.sh || exit $?
  ;;
move_cell_fast)
  # round 6: float32 move rows: target cell from float polynomials when its rounding
  # is certain (move_cell_f32_fast; the double sincos otherwise) against the
  # previous build, then the whole GPU suite
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 4096" "--spawns melee" || exit $?
  bash tools/gpu/tests.sh || exit $?
  ;;
store_wt_knob)
  # round 6: the small shards' row stores without write-through (LNW_NO_STORE_WT:
  # plain stores), interleaved A/B of the knob
  bash tools/gpu/ab_env.sh LNW_NO_STORE_WT 3 "--global-envs 8192" "--global-envs 4096" "" || exit $?
  ;;
no_phase_q_barrier)
  # round 6: small quiet workgroups without the phase-Q barrier (wave 1 commits
  # every move itself, wave 0 takes the final cells from the phase-M columns)
  # against the previous build, the whole GPU suite, the 8 192-env timeline
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "--global-envs 16384" || exit $?
  bash tools/gpu/tests.sh || exit $?
  bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
  ;;
counters_removed)
  # round 6: the launch-time counter loads removed (they put 52 B/lane of scratch
  # into the contact kernels and 28 B into the small-shard kernel) against the
  # previous build; the GPU suite
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" "--spawns melee" || exit $?
  bash tools/gpu/tests.sh || exit $?
  ;;
counters_noncontact)
  # round 6: the launch-time counter loads kept in the non-contact kernels only
  # (the contact variants scratch-free again) against the previous build
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--spawns melee" "" || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py tests/test_gpu_rollout.py tests/test_gpu_rollout_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; exit $rc
  ;;
policy_tail_address)
  # the policy: timing of two actor builds (tools/probe: actor_prev = HEAD, actor_new = the tree), then determinism, rollout parity
  timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_prev.so tools/probe/actor_new.so tools/probe/actor_prev.so tools/probe/actor_new.so 2>&1 | grep -v amdgpu || exit 1
  timeout -k 10 300 python -u tools/policy_determinism.py 32768 48 critic,strided,packed > gpurun_out/det_w.log 2>&1 || { tail -20 gpurun_out/det_w.log; exit 2; }
  grep "mismatching" gpurun_out/det_w.log
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_fullsize.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py tests/test_gpu_obs_options.py $(ls tests/test_gpu_*polic*.py tests/test_gpu_*actor*.py 2>/dev/null) > gpurun_out/w_tests.log 2>&1 || { tail -20 gpurun_out/w_tests.log; exit 3; }
  tail -1 gpurun_out/w_tests.log
  ;;
final_evidence_a)
  # round 6 final evidence, part A: the GPU suite + smoke(), the stress runs
  # (split contact rows 30x, policy / critic determinism), the rocprofv3 evidence
  # of the headline, the 8 192-env shard and config 2
  bash tools/gpu/tests.sh || exit $?
  bash tools/gpu/stress.sh 30 48 || exit $?
  bash tools/gpu/prof_all.sh r06 1 || exit $?
  ;;
final_evidence_b)
  # round 6 final evidence, part B: rocprofv3 evidence of melee, config 4 and config 5
  # (prof_all.sh part 2), then the default bench line
  bash tools/gpu/prof_all.sh r06 2 || exit $?
  timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06bb.json 2> gpurun_out/bench_r06bb.err
  rc=$?; tail -c 300 gpurun_out/bench_r06bb.json; exit $rc
  ;;
critic_prefetch)
  # the critic launch: 256-bound instantiation with the whole fc1 row prefetched (actor_new) vs HEAD (actor_prev), then determinism, rollout parity
  timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_prev.so tools/probe/actor_new.so tools/probe/actor_prev.so tools/probe/actor_new.so 2>&1 | grep -v amdgpu || exit 1
  timeout -k 10 300 python -u tools/policy_determinism.py 32768 48 critic,strided,packed > gpurun_out/det_w.log 2>&1 || { tail -20 gpurun_out/det_w.log; exit 2; }
  grep "mismatching" gpurun_out/det_w.log
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_fullsize.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py tests/test_gpu_obs_options.py $(ls tests/test_gpu_*polic*.py tests/test_gpu_*actor*.py 2>/dev/null) > gpurun_out/w_tests.log 2>&1 || { tail -20 gpurun_out/w_tests.log; exit 3; }
  tail -1 gpurun_out/w_tests.log
  ;;
final_stress)
  # round 6: final-build repetition evidence: split contact rows 60 runs, policy /
  # critic 150 repetitions (tools/gpu/stress.sh), then the GPU suite a second time
  bash tools/gpu/stress.sh 60 150 || exit $?
  bash tools/gpu/tests.sh || exit $?
  ;;
quiet_likely)
  # round 6: the quiet branch marked likely (block placement) against the previous
  # build: interleaved A/B at the headline and the shard sizes
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 4096" || exit $?
  ;;
scale_shapes)
  # round 6: the per-GPU shapes of N = 2 and N = 4 (32 768 and 16 384 envs) timed,
  # with their LNW_PROF timelines
  bash tools/gpu/timeline.sh sh32768 "--global-envs 32768" 2>&1 | grep -E "wg=|quiet|grid:|sh32768" || exit 1
  bash tools/gpu/timeline.sh sh16384 "--global-envs 16384" 2>&1 | grep -E "wg=|quiet|grid:|sh16384" || exit 1
  ;;
epw_shapes)
  # round 6: envs per workgroup at the N = 2 / 4 per-GPU shapes (LNW_EPW_RT
  # overrides choose_epw): 16384 and 32768 envs at 16 / 32 / 64 envs per workgroup
  for a in "16384 16" "16384 32" "32768 16" "32768 32" "32768 64"; do
    set -- $a
    LNW_EPW_RT=$2 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 \
      --global-envs $1 > gpurun_out/epw.json 2>gpurun_out/epw.err || { tail -5 gpurun_out/epw.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/epw.json')); print('envs $1 epw $2', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
  done
  ;;
slab_rows)
  # round 6: quiet workgroups of 32 envs write their rows in two 16-env slabs
  # (step_qdirect) against the previous build and the LNW_NO_SLAB knob, then the
  # shard / parity / full-size / units / state tests
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 16384" "--global-envs 8192" "--global-envs 4096" "" || exit $?
  LNW_LIB=$PWD/$L bash tools/gpu/ab_env.sh LNW_NO_SLAB 2 "--global-envs 16384" || exit $?
  timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_units.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; exit $rc
  ;;
units2)
  # round 6: two-unit workgroups (LNW_UNITS2) at the N = 2 and N = 4 per-GPU shapes,
  # interleaved A/B of the knob; the units / shard tests with it on (the knob and
  # its kernel were removed after this measured slower: DESIGN.md)
  bash tools/gpu/ab_env.sh LNW_UNITS2 3 "--global-envs 32768" "--global-envs 16384" || exit $?
  LNW_UNITS2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; exit $rc
  ;;
epw8)
  # round 6: 8 envs per workgroup at config 2 (4 096 envs: 512 workgroups instead of
  # 256 of 16) and at 8 192, interleaved with the default choice
  for r in 1 2 3; do
    for a in "4096 0" "4096 8" "8192 0" "8192 8"; do
      set -- $a
      if [ "$2" = 0 ]; then unset LNW_EPW_RT; else export LNW_EPW_RT=$2; fi
      timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 \
        --global-envs $1 > gpurun_out/epw.json 2>gpurun_out/epw.err || { tail -5 gpurun_out/epw.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/epw.json')); print('r$r envs $1 epw ${2/#0/default}', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
    done
  done
  ;;
loud_call)
  # round 6: the units kernel's loud units behind a call (step_loud_unit) against
  # the previous build, headline and shard shapes, then the units / parity tests
  L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
  bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 16384" "--spawns melee" || exit $?
  timeout -k 10 900 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; exit $rc
  ;;
*)
  echo "usage: bash tools/gpu/round6.sh {loud_call|epw8|units2|slab_rows|scale_shapes|epw_shapes|crash_race|race_nowait|race_nowait_nt|policy_probe14|policy_probe15_16|policy_probe16_c4fetch|policy_fence|policy_tail_quads|c4_rows_batched|shard_timelines|quiet_columns_upfront|quiet_pairs_packed|quiet_only_probe|quiet_test_spread|counters_at_launch|counters_knob|evidence_first_a|evidence_first_b|sincos_probe|sincos_certified|move_cell_fast|store_wt_knob|no_phase_q_barrier|counters_removed|counters_noncontact|policy_tail_address|final_evidence_a|final_evidence_b|critic_prefetch|final_stress|quiet_likely}"
  exit 2
  ;;
esac
