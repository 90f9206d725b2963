#!/bin/bash
# In-process A/B (tools/ab_libs.py) of ab/*.so builds: config 4's whole frame at $SPP spp (ring mode)
# and rank 0's rows of an 8-GPU job at 500 spp (direct mode).  Outputs must be bit-identical.
#   AB="ab/f0.so ab/f2.so" TAG=walkform tools/gpu_ab3.sh
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB=${AB:-"ab/base.so ab/new.so"}
TAG=${TAG:-ab}
timeout -k 10 300 python -u tools/ab_libs.py $AB --spp ${SPP:-100} --rounds ${ROUNDS:-7} > gpurun_out/${TAG}_full.json 2> gpurun_out/${TAG}_full.err || exit 3
cat gpurun_out/${TAG}_full.json
timeout -k 10 300 python -u tools/ab_libs.py $AB --spp 500 --row-step 8 --rounds ${ROUNDS:-7} > gpurun_out/${TAG}_r8.json 2> gpurun_out/${TAG}_r8.err || exit 4
cat gpurun_out/${TAG}_r8.json
