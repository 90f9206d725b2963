#!/bin/bash
# Round evidence on the GPU box: the default bench line (with the CPU baseline), the instrumented
# counts of one 100-spp frame, and the rocprofv3 trace + PMC passes of tools/profile.sh.
#   TAG=r02_x tools/gpu_bench_profile.sh      (then: python tools/pmc_summary.py <tag>)
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kprofile.py --spp 100 --variants bvh --out gpurun_out/kprof_$TAG.json > gpurun_out/kprof_$TAG.log 2>&1
rc=$?; echo "kprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/profile.sh
