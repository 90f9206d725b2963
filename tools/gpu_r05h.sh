#!/bin/bash
# Seed-window A/B (default build vs -DRTZIG_SEED_WINDOW=1) and the one-buffer N = 8 pipeline
# (rank_sim --pipe-mode plain: the workspace-halving option of VERDICT r04 item 5).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB="ab/cur.so ab/win.so" TAG=r05h bash tools/gpu_ab.sh || exit $?
timeout -k 10 300 python3 -u tools/rank_sim.py --ns 1 8 --reps 2 --pipe-frames 8 --pipe-mode plain > gpurun_out/ranksim_plain.json 2> gpurun_out/ranksim_plain.err
rc=$?; echo "rank_sim plain rc=$rc"; exit $rc
