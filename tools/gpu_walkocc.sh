#!/bin/bash
# Walk-only microkernel (tools/walk_occupancy.hip, built beforehand into tools/bin/walk_occ): the
# round-3 static-stride lane assignment and the round-4 path-ordered one, at 4/5/6/8 waves per SIMD.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bin/walk_occ 1200000 5 40 > gpurun_out/walk_occ.json 2> gpurun_out/walk_occ.err
rc=$?; echo "walk_occ rc=$rc"; cat gpurun_out/walk_occ.err | tail -12; exit $rc
