#!/bin/bash
# rocprofv3 evidence for the dominant kernel (run on the GPU box via gpurun):
#   1. kernel trace + stats of the bench command;
#   2. PMC passes, one rocprofv3 run per counter set (no trace domains): FETCH_SIZE, WRITE_SIZE and
#      the SQ sets of the VALU-issue / wave-cycle / LDS analysis (tools/pmc_summary.py).
# Each GPU step has its own time limit; the script stops at a timeout / abort / kill / segfault.
#   TAG=r02_x tools/profile.sh      then: python tools/pmc_summary.py r02_x
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH=${BENCH:-"bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin"}
PMC_BENCH=${PMC_BENCH:-"bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fast --no-dropin"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || exit $?
echo "trace ok"
SETS=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_THREAD_CYCLES_VALU"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_F64"
)
for set in "${SETS[@]}"; do
  name=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $set -d "$OUT/pmc_$name" -o pmc --output-format csv -- python3 $PMC_BENCH > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.err"
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pmc $name rc=$rc"; tail -3 "$OUT/pmc_$name.err"
    case $rc in 124|134|137|139) exit $rc;; esac
    continue
  fi
  echo "pmc $name ok"
done
