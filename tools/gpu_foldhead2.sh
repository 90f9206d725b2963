#!/bin/bash
# Head-fold waves per block: 1 / 2 / 4 (ab/fh*.so) against none (ab/base.so), every rank's rows in
# bench.py's deferred pipeline (rank_sim), each library copied over the in-tree one in turn.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for v in ${VARIANTS:-base fh fh2 fh4 base fh fh2 fh4}; do
  cp ab/$v.so raytracing-with-zig_amd/librtzig.so
  timeout -k 10 200 python3 -u tools/rank_sim.py --ns 1 8 --reps 3 --pipe-frames 8 --pipe-mode deferred > gpurun_out/ranksim_$v.json 2> gpurun_out/ranksim_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "rank_sim $v rc=$rc"; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/ranksim_$v.json'));r=d['ranks']['8'];print('$v', r['pipelined_frame_ms_max_over_ranks'], r['efficiency_pipelined'], d['ranks']['1']['pipelined_frame_ms_max_over_ranks'])" | tee -a gpurun_out/foldhead_sweep.txt
done
