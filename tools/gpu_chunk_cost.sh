#!/bin/bash
# Frame time of config 4 by sample-chunk plan: workspace limit (RTZIG_WORKSPACE_MB) x chunk
# pipeline on / off (RTZIG_PIPELINE).  Each run has its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/chunk_cost
for cfg in ${CFGS:-"20000 1" "4096 1" "4096 0" "8192 0" "8192 1"}; do
  set -- $cfg
  RTZIG_WORKSPACE_MB=$1 RTZIG_PIPELINE=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fast --no-dropin --steps 5 \
    > gpurun_out/chunk_cost/mb$1_p$2.json 2> gpurun_out/chunk_cost/mb$1_p$2.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/chunk_cost/mb$1_p$2.json'));r=d['roofline'];print('$1 MB pipeline=$2', d['ms_per_step'], r['launches_per_frame'], r['kernel_ms_per_frame'], r['reduce_kernel_ms_per_frame'])"
done
