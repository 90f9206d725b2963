#!/bin/bash
# One GPU round trip for a leaf-round change: pytest -m gpu on the in-tree build, in-process A/B of
# ab/*.so builds, then the instrumented counts of each build (copied over the in-tree library of
# this scratch copy, one at a time).  Every GPU step is time-limited; the first failure ends it.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB=${AB:-"ab/f0.so ab/f1.so ab/f2.so"}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/ab_libs.py $AB --spp ${SPP:-100} --rounds ${ROUNDS:-5} > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err
[ $rc -eq 0 ] || exit $rc
for so in $AB; do
  n=$(basename $so .so)
  cp "$so" raytracing-with-zig_amd/librtzig.so
  timeout -k 10 200 python -u tools/kprofile.py --spp 100 --variants bvh --out gpurun_out/kprof_$n.json > gpurun_out/kprof_$n.log 2>&1
  rc=$?; echo "kprof $n rc=$rc"; tail -1 gpurun_out/kprof_$n.log
  [ $rc -eq 0 ] || exit $rc
done
