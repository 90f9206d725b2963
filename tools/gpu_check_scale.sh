#!/bin/bash
# GPU round trip after a scheduling change: pytest -m gpu (parity), the default bench line, and the
# one-GPU strong-scaling rehearsal (rank 0's row set for N = 1, 2, 4, 8; tools/rank_sim.py).
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
timeout -k 10 200 python -u tools/rank_sim.py --spp 500 --reps 3 > gpurun_out/rank_sim.json 2> gpurun_out/rank_sim.err
rc=$?; echo "rank_sim rc=$rc"; cat gpurun_out/rank_sim.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/rank_sim.err; exit $rc; }
timeout -k 10 400 python -u tools/configs_bench.py --out gpurun_out/r01_configs.json > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; tail -6 gpurun_out/configs.log; [ $rc -eq 0 ] || exit $rc
