#!/bin/bash
# VALU issue-rate microbenchmark (tools/valu_rates.hip, built beforehand into tools/bin/valu_rates).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bin/valu_rates > gpurun_out/valu_rates.json 2> gpurun_out/valu_rates.err
rc=$?; echo "valu_rates rc=$rc"; cat gpurun_out/valu_rates.json; exit $rc
