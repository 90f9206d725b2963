#!/bin/bash
# Kernel change round trip: parity suite on the new build, then in-process A/B (config 4 frame and
# rank 0's rows of an 8-GPU job).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r05c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_r05c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 100 --rounds 7 > gpurun_out/ab_r05c.json 2> gpurun_out/ab_r05c.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_r05c.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 500 --rounds 5 --row-step 8 > gpurun_out/ab_r05c_r8.json 2> gpurun_out/ab_r05c_r8.err
rc=$?; echo "ab8 rc=$rc"; cat gpurun_out/ab_r05c_r8.json; exit $rc
