#!/bin/bash
# One GPU round trip: smoke -> pytest -m gpu -> bench.  Every GPU step has its own time limit; a
# fault / abort / segfault / timeout (exit not in {0,1}) stops the script before the next GPU step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1"}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
