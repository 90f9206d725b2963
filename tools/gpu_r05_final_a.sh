#!/bin/bash
# Round-5 evidence, part A: smoke, the GPU suite (one process, per-test limits), the default bench
# line, then the instrumented counts and the rocprofv3 trace + PMC passes (tools/profile.sh).
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
T=${TAG:-r05}
timeout -k 10 150 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gputest_$T.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$T.json; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROFILE" ] && exit 0
timeout -k 10 200 python3 -u tools/kprofile.py --spp 100 --variants bvh --out gpurun_out/kprof_$T.json > gpurun_out/kprof_$T.log 2>&1
rc=$?; echo "kprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=$T bash tools/profile.sh
