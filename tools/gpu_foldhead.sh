#!/bin/bash
# Head-fold A/B: rank 0's rows of an 8-GPU job as plain launches (ab_libs: the sample kernel alone),
# then every rank's rows in bench.py's deferred pipeline (rank_sim) with the in-tree library and
# with ab/base.so copied over it.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab_libs.py ab/base.so ab/fh.so --spp 500 --rounds 7 --row-step 8 > gpurun_out/ab_fh_r8.json 2> gpurun_out/ab_fh_r8.err
rc=$?; echo "ab8 rc=$rc"; cat gpurun_out/ab_fh_r8.json; [ $rc -eq 0 ] || exit $rc
for v in fh base fh base; do
  if [ $v = base ]; then cp ab/base.so raytracing-with-zig_amd/librtzig.so; else cp ab/fh.so raytracing-with-zig_amd/librtzig.so; fi
  timeout -k 10 200 python3 -u tools/rank_sim.py --ns 1 8 --reps 3 --pipe-frames 8 --pipe-mode deferred > gpurun_out/ranksim_$v.json 2> gpurun_out/ranksim_$v.err
  rc=$?; echo "rank_sim $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/ranksim_$v.json'));r=d['ranks']['8'];print('$v', r['pipelined_frame_ms_max_over_ranks'], r['efficiency_pipelined'], d['ranks']['1']['pipelined_frame_ms_max_over_ranks'])"
  cp gpurun_out/ranksim_$v.json gpurun_out/ranksim_${v}_$(date +%s%N).json
done
