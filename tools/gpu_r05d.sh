#!/bin/bash
# Kernel change round trip: parity suite on the in-tree build, in-process A/B of $AB (config 4 frame
# and rank 0's rows of an 8-GPU job), then the instrumented counts of the in-tree build.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
T=${TAG:-r05d}
timeout -k 10 150 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/smoke_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_$T.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 100 --rounds 7 > gpurun_out/ab_$T.json 2> gpurun_out/ab_$T.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 500 --rounds 5 --row-step 8 > gpurun_out/ab_${T}_r8.json 2> gpurun_out/ab_${T}_r8.err
rc=$?; echo "ab8 rc=$rc"; cat gpurun_out/ab_${T}_r8.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/kprofile.py --spp 100 --variants bvh --out gpurun_out/kprof_$T.json > gpurun_out/kprof_$T.log 2>&1
rc=$?; echo "kprof rc=$rc"; tail -3 gpurun_out/kprof_$T.log; exit $rc
