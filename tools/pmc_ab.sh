#!/bin/bash
# PMC counters of an in-process A/B (tools/ab_libs.py, one round: each build's sample kernel runs
# twice, in the order the builds are given), one rocprofv3 pass per counter set.  Summarise with
#   python tools/pmc_ab.py gpurun_out/pmcab_<tag> <n_builds>
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
T=${TAG:-ab}
OUT=gpurun_out/pmcab_$T
mkdir -p "$OUT"
ARGS=${ARGS:-"--spp 100 --rounds 1"}
SETS=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM"
  "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 tools/ab_libs.py $AB $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?
  echo "pmc set $i rc=$rc"
  case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/p$i.err";; esac
done
