#!/bin/bash
# Round 5: operand-form issue costs, the drop-in's one-shot cost, and the GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bin/peak_rates 60 2 > gpurun_out/peak_table2.json 2> gpurun_out/peak_table2.err
rc=$?; echo "peak_rates rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/dropin_cold.py --runs 3 --configs 2,4,5 > gpurun_out/dropin_cold2.json 2> gpurun_out/dropin_cold2.err
rc=$?; echo "dropin_cold rc=$rc"; tail -3 gpurun_out/dropin_cold2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r05b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputest_r05b.log; exit $rc
