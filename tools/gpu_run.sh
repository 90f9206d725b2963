#!/bin/bash
# The one GPU-box runner (via gpurun): named steps, in the order given, each under its own time limit,
# stdout / stderr of step <name> in gpurun_out/<name>_<TAG>.out / .err.  The script stops at the first failing step, so nothing touches the GPU
# after a timeout, abort or fault.
#
#   tools/gpu_run.sh smoke tests bench            # the round trip
#   TAG=r06 tools/gpu_run.sh bench kprof profile  # round evidence (then: python tools/pmc_summary.py r06)
#   AB="ab/base.so ab/new.so" tools/gpu_run.sh ab # in-process A/B of two builds (tools/build_variant.sh)
#
# Steps (environment knobs in brackets):
#   smoke      __graft_entry__.smoke()
#   tests      pytest -m gpu, one process, per-test limits                       [PYTEST_ARGS]
#   bench      the default bench line                                            [BENCH_ARGS]
#   kprof      instrumented counts of one 100-spp config-4 frame, wave- and lane-level per region
#              (tools/kprofile.py; then here: python tools/region_table.py <kprof.json>)  [KPROF_ARGS]
#   profile    rocprofv3 kernel trace + separate PMC passes (tools/profile.sh)
#   ab         tools/ab_libs.py on config 4's whole frame (ring mode) and rank 0 of 8 (direct)  [AB SPP ROUNDS]
#   ab_ch9     the same on chapter 9 (config 2)                                  [AB ROUNDS]
#   pmc_ab     PMC passes over an in-process A/B (tools/pmc_ab.sh)               [AB ARGS]
#   ranksim    every rank's rows in bench.py's N > 1 frame pipeline (tools/rank_sim.py)  [NS PIPE RANKSIM_ARGS]
#   configs    every BASELINE config (tools/configs_bench.py)
#   dropin     the drop-in's one-shot cost per fresh process (tools/dropin_cold.py)  [DROPIN_CONFIGS]
#   peak       event-timed VALU peak and issue-cost table (tools/bin/peak_rates, built beforehand)
#   diag       bounds-checked builds through tools/diag_modes.py (ab/bounds*.so)
#   uselib     copy $LIB (an ab/*.so build) over the in-tree librtzig.so for the steps after it (on the
#              box's copy of the tree only)                                     [LIB]
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-run}
AB=${AB:-"ab/base.so ab/new.so"}

run() {  # run <name> <seconds> <command...>: stdout to gpurun_out/<name>_<tag>.out, stderr to .err;
         # stop on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$T.out" 2> "gpurun_out/${name}_$T.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 1500 "gpurun_out/${name}_$T.out"; echo; tail -3 "gpurun_out/${name}_$T.err"
  [ $rc -eq 0 ] || exit $rc
}

for step in "$@"; do
  case $step in
    smoke)   run smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)   run gputest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread $PYTEST_ARGS ;;
    bench)   run bench 300 python3 -u bench.py $BENCH_ARGS ;;
    kprof)   run kprof 200 python3 -u tools/kprofile.py --spp 100 --variants bvh --out "gpurun_out/kprof_$T.json" $KPROF_ARGS ;;
    profile) TAG=$T bash tools/profile.sh || exit $? ;;
    ab)      run ab_full 300 python3 -u tools/ab_libs.py $AB --spp ${SPP:-100} --rounds ${ROUNDS:-7}
             run ab_r8 300 python3 -u tools/ab_libs.py $AB --spp 500 --row-step 8 --rounds ${ROUNDS:-7} ;;
    ab_ch9)  run ab_ch9 200 python3 -u tools/ab_libs.py $AB --scene ch9 --width 400 --aspect 1.7777777777777777 --spp 100 --rounds ${ROUNDS:-9} ;;
    pmc_ab)  TAG=$T AB="$AB" bash tools/pmc_ab.sh || exit $? ;;
    ranksim) run ranksim 300 python3 -u tools/rank_sim.py --ns ${NS:-1 2 4 8} --reps 2 --pipe-frames 8 --pipe-mode ${PIPE:-deferred} $RANKSIM_ARGS ;;
    configs) run configs 300 python3 -u tools/configs_bench.py --out "gpurun_out/configs_$T.json" ;;
    dropin)  run dropin 300 python3 -u tools/dropin_cold.py --runs 3 --configs ${DROPIN_CONFIGS:-2,4,5} ;;
    peak)    run peak 300 ./tools/bin/peak_rates ${PEAK_MS:-60} ${PEAK_MODE:-2} ;;
    diag)    run diag 300 python3 -u tools/diag_modes.py raytracing-with-zig_amd/librtzig.so ab/bounds.so --oracle-row ;;
    uselib)  cp "$LIB" raytracing-with-zig_amd/librtzig.so || exit 2; echo "== using $LIB" ;;
    *) echo "unknown step: $step"; exit 2 ;;
  esac
done
exit 0
