#!/bin/bash
# PMC A/B of the seed window + the N = 8 footprint options (rank_sim in the bench pipeline).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB="ab/stk.so ab/win3.so" TAG=win bash tools/pmc_ab.sh || exit $?
for mode in deferred split; do
  timeout -k 10 300 python3 -u tools/rank_sim.py --ns 1 8 --reps 2 --pipe-frames 8 --pipe-mode $mode > gpurun_out/ranksim_$mode.json 2> gpurun_out/ranksim_$mode.err
  rc=$?; echo "rank_sim $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
RTZIG_UNIT_MODE=ring timeout -k 10 300 python3 -u tools/rank_sim.py --ns 1 8 --reps 2 --pipe-frames 8 > gpurun_out/ranksim_ring.json 2> gpurun_out/ranksim_ring.err
rc=$?; echo "rank_sim ring rc=$rc"; exit $rc
