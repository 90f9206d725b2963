cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
L="ab/c256.so ab/c64k8m4k.so ab/c128k8m4k.so ab/c192k8m4k.so ab/c256k8m4k.so ab/c128k6m4k.so ab/c128k8.so"
timeout -k 10 200 python -u tools/ab_libs.py $L --spp 500 --rounds 9 --row-step 8 > gpurun_out/ab_r8.json 2> gpurun_out/ab_r8.err
rc=$?; echo "r8 rc=$rc"; cat gpurun_out/ab_r8.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_r8.err; exit $rc; }
timeout -k 10 250 python -u tools/ab_libs.py $L --spp 500 --rounds 5 > gpurun_out/ab_full.json 2> gpurun_out/ab_full.err
rc=$?; echo "full rc=$rc"; cat gpurun_out/ab_full.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_full.err; exit $rc; }
