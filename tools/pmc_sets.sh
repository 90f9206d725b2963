#!/bin/bash
# Extra PMC passes (one rocprofv3 run per set, no trace domains) on a short kprofile-sized run.
#   SETS are space-separated groups joined by ','.  Output: gpurun_out/pmc_<tag>/<first>/...
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-bvh}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
CMD=${CMD:-"tools/ab_variants.py --env RTZIG_KERNEL --variants bvh --spp 100 --rounds 1"}
IFS=',' read -ra SETS <<< "${SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES GRBM_GUI_ACTIVE,SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SALU,SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F32}"
for set in "${SETS[@]}"; do
  name=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/$name" -o pmc --output-format csv -- python3 $CMD > "$OUT/$name.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $name rc=$rc"; tail -3 "$OUT/$name.log"; [ $rc -eq 1 ] || exit $rc; continue; fi
  echo "pmc $name ok"
done
