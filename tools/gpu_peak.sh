#!/bin/bash
# Event-timed VALU peak rates and the full opcode table (tools/peak_rates.hip, built beforehand into
# tools/bin/peak_rates), then the drop-in's one-shot cost per config (tools/dropin_cold.py).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bin/peak_rates ${PEAK_MS:-60} 1 > gpurun_out/peak_table.json 2> gpurun_out/peak_table.err
rc=$?; echo "peak_rates rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/dropin_cold.py --runs 3 --configs 2,4,5 > gpurun_out/dropin_cold.json 2> gpurun_out/dropin_cold.err
rc=$?; echo "dropin_cold rc=$rc"; tail -3 gpurun_out/dropin_cold.err; exit $rc
