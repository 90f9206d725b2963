#!/bin/bash
# Verdict r03 item 1 on the GPU box: the shipped build and the -DRTZIG_BOUNDS=1 knob variants
# (ab/bounds*.so, tools/build_variant.sh) through tools/diag_modes.py — every output bit-exact with
# the shipped build, no error word set — then the self-test build, whose deliberately narrowed node
# range the check must report.  Each GPU step has its own time limit; the script stops at the first
# unexpected result.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_modes.py raytracing-with-zig_amd/librtzig.so ab/bounds.so ab/bounds_w3.so \
  ab/bounds_b256.so ab/bounds_s16.so --oracle-row > gpurun_out/diag_modes.jsonl 2> gpurun_out/diag_modes.err
rc=$?; echo "diag rc=$rc"; tail -3 gpurun_out/diag_modes.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/diag_modes.py raytracing-with-zig_amd/librtzig.so ab/bounds_self.so \
  > gpurun_out/diag_selftest.jsonl 2> gpurun_out/diag_selftest.err
rc=$?; echo "selftest rc=$rc (1 expected)"; grep -c "index out of range" gpurun_out/diag_selftest.jsonl
[ $rc -eq 1 ] || exit 5
exit 0
