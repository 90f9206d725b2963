#!/bin/bash
# In-process A/B (tools/ab_libs.py) of ab/*.so builds on rank 0 of 8 (config 4) and chapter 9.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB=${AB:-"ab/base.so ab/new.so"}
timeout -k 10 200 python -u tools/ab_libs.py $AB --spp 500 --row-step 8 --rounds ${ROUNDS:-5} $NOCHECK > gpurun_out/ab2_r8.json 2> gpurun_out/ab2_r8.err || exit 3
cat gpurun_out/ab2_r8.json
timeout -k 10 200 python -u tools/ab_libs.py $AB --scene ch9 --width 400 --spp 100 --rounds ${ROUNDS:-5} $NOCHECK > gpurun_out/ab2_ch9.json 2> gpurun_out/ab2_ch9.err || exit 4
cat gpurun_out/ab2_ch9.json
