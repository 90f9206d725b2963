#!/bin/bash
# Round-5 evidence, part B (after tools/gpu_bench_profile.sh): the drop-in's one-shot cost in fresh
# processes, every rank's rows in bench.py's frame pipeline (deferred at N = 1/2/4/8; the
# one-buffer plain pipeline and ring mode at N = 8), and every BASELINE config.
# Every GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
T=${TAG:-r05}
# the bench line again, now reading the round's own PMC summary (profiles/pmc_traffic.json)
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_${T}_final.json 2> gpurun_out/bench_${T}_final.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${T}_final.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u tools/dropin_cold.py --runs 3 --configs 2,4,5 > gpurun_out/dropin_cold_$T.json 2> gpurun_out/dropin_cold_$T.err
rc=$?; echo "dropin rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/rank_sim.py --ns 1 2 4 8 --reps 2 --pipe-frames 8 --pipe-mode deferred > gpurun_out/ranksim_deferred_$T.json 2> gpurun_out/ranksim_deferred_$T.err
rc=$?; echo "rank_sim deferred rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/rank_sim.py --ns 1 8 --reps 2 --pipe-frames 8 --pipe-mode plain > gpurun_out/ranksim_plain_$T.json 2> gpurun_out/ranksim_plain_$T.err
rc=$?; echo "rank_sim plain rc=$rc"; [ $rc -eq 0 ] || exit $rc
RTZIG_UNIT_MODE=ring timeout -k 10 200 python3 -u tools/rank_sim.py --ns 1 8 --reps 2 --pipe-frames 8 > gpurun_out/ranksim_ring_$T.json 2> gpurun_out/ranksim_ring_$T.err
rc=$?; echo "rank_sim ring rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/configs_bench.py --out gpurun_out/configs_$T.json > gpurun_out/configs_$T.log 2>&1
rc=$?; echo "configs rc=$rc"; exit $rc
