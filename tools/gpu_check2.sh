#!/bin/bash
# GPU round trip: pytest -m gpu -> bench (N=1) -> 2-rank gloo rehearsal of the distributed bench
# (both ranks share the one GPU).  Each step is time-limited; the first failure ends the script.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus ${NPROC:-2} --steps 2 --warmup 1 --dist-backend gloo > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
rc=$?; echo "gloo2 rc=$rc"; cat gpurun_out/bench_gloo2.json; [ $rc -eq 0 ] || tail -5 gpurun_out/bench_gloo2.err
exit $rc
