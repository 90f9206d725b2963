#!/bin/bash
# In-process A/B of queue-claim builds (ab/*.so from tools/build_variant.sh with EXTRA=-DRTZIG_...)
# on chapter 9, chapter 13, the final scene, and rank 0's row set of an 8-GPU job.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
L=${AB:-"ab/base.so ab/new.so"}
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python -u tools/ab_libs.py $L "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err
  local rc=$?; echo "$n rc=$rc"; cat gpurun_out/ab_$n.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$n.err; exit $rc; }
}
run ch9 --scene ch9 --width 400 --spp 100 --rounds 25
run ch13 --scene ch13 --width 1200 --spp 500 --rounds 3
run r8 --spp 500 --rounds 7 --row-step 8
run full --spp 500 --rounds 3
