#!/bin/bash
# In-process A/B of the libraries in $AB: config 4's frame at 100 spp and rank 0's rows of an
# 8-GPU job at 500 spp (tools/ab_libs.py), nothing else.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
T=${TAG:-ab}
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 100 --rounds 7 > gpurun_out/ab_$T.json 2> gpurun_out/ab_$T.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_$T.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_libs.py $AB --spp 500 --rounds 7 --row-step 8 > gpurun_out/ab_${T}_r8.json 2> gpurun_out/ab_${T}_r8.err
rc=$?; echo "ab8 rc=$rc"; cat gpurun_out/ab_${T}_r8.json; exit $rc
