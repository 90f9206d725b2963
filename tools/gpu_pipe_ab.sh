#!/bin/bash
# Deferred pipeline A/B at rank 0 of 8: library (ab/base.so: follow-up fold pass after every
# deferred launch; ab/nf.so: none for the uninstrumented kernels) x row buffers (2 / 3), each
# library copied over the in-tree one in turn (tools/rank_sim.py, bench.py's N > 1 frame loop).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base nf; do
    cp ab/$v.so raytracing-with-zig_amd/librtzig.so
    for nb in 2 3; do
      timeout -k 10 200 python3 -u tools/rank_sim.py --ns 1 8 --reps 3 --pipe-frames 8 --pipe-mode deferred --row-buffers $nb > gpurun_out/ranksim_${v}_nb$nb.json 2> gpurun_out/ranksim_${v}_nb$nb.err
      rc=$?; [ $rc -eq 0 ] || { echo "rank_sim $v nb$nb rc=$rc"; exit $rc; }
      python3 -c "import json;d=json.load(open('gpurun_out/ranksim_${v}_nb$nb.json'));r=d['ranks']['8'];print('$v nb$nb', r['pipelined_frame_ms_max_over_ranks'], r['efficiency_pipelined'], r['pipelined_sample_kernel_ms_slowest_rank'], r['pipelined_reduce_ms_slowest_rank'], d['ranks']['1']['pipelined_frame_ms_max_over_ranks'])" | tee -a gpurun_out/pipe_ab.txt
    done
  done
done
