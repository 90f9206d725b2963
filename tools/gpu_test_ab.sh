cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_libs.py ab/base.so ab/new.so --spp 500 --row-step 8 --rounds 7 > gpurun_out/ab_r8.json 2> gpurun_out/ab_r8.err || exit 3
cat gpurun_out/ab_r8.json
timeout -k 10 200 python -u tools/ab_libs.py ab/base.so ab/new.so --scene ch9 --width 400 --aspect 1.7777777777777777 --spp 100 --rounds 9 > gpurun_out/ab_ch9.json 2> gpurun_out/ab_ch9.err || exit 4
cat gpurun_out/ab_ch9.json
timeout -k 10 200 python -u tools/ab_libs.py ab/base.so ab/new.so --spp 100 --rounds 5 > gpurun_out/ab_full.json 2> gpurun_out/ab_full.err || exit 5
cat gpurun_out/ab_full.json
