#!/bin/bash
# Diagnostics of the in-tree build on the GPU: in-kernel instrumentation (tools/kprofile.py) and
# PMC passes of one 100-spp frame (tools/pmc_sets.sh).  Steps are time-limited and chained.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
TAG=${TAG:-diag}
timeout -k 10 200 python -u tools/kprofile.py --spp 100 --variants bvh --out gpurun_out/kprof_$TAG.json > gpurun_out/kprof_$TAG.log 2>&1
rc=$?; echo "kprofile rc=$rc"; tail -30 gpurun_out/kprof_$TAG.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG CMD="tools/ab_variants.py --env RTZIG_KERNEL --variants bvh --spp 100 --rounds 1" \
SETS="${SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE,SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}" tools/pmc_sets.sh
