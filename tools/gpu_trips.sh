#!/bin/bash
# Rejection-trip microbenchmark (tools/trip_bench.hip, built beforehand into tools/bin/trip_bench)
# at the request mix of the instrumented frame and two bracketing mixes.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
: > gpurun_out/trip_bench.jsonl
for mix in "${MIX:-0.45 0.2}" "0.3 0.1" "0.6 0.3"; do
  timeout -k 10 120 ./tools/bin/trip_bench $mix 2000 >> gpurun_out/trip_bench.jsonl 2> gpurun_out/trip_bench.err || exit 3
done
cat gpurun_out/trip_bench.jsonl
