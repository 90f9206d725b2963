#!/bin/bash
# rocprofv3 evidence for the dominant kernel (run on the GPU box via gpurun):
#   1. kernel trace + stats of the bench command;
#   2. PMC passes (separate runs, no trace domains): SQ/GRBM counters, then FETCH_SIZE, WRITE_SIZE.
# Each GPU step has its own time limit; the script stops at the first failing step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH=${BENCH:-"bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
PMC_BENCH=${PMC_BENCH:-"bench.py --steps 1 --warmup 0 --no-cpu-baseline"}
set -o pipefail
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || exit $?
echo "trace ok"
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"; do
  name=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/pmc_$name" -o pmc --output-format csv -- python3 $PMC_BENCH > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.err" 
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $name failed rc=$rc"; tail -5 "$OUT/pmc_$name.err"; [ $rc -eq 1 ] || exit $rc; continue; fi
  echo "pmc $name ok"
done
