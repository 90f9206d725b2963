#!/bin/bash
# GPU round trip for a kernel change: pytest -m gpu (parity) -> in-process A/B of ab/*.so builds.
#   AB="ab/base.so ab/new.so" SPP=100 tools/gpu_ab.sh
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB=${AB:-"ab/base.so ab/new.so"}
SPP=${SPP:-100}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/ab_libs.py $AB --spp $SPP --rounds ${ROUNDS:-5} > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.json; tail -5 gpurun_out/ab.err
exit $rc
