cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
AB="ab/base.so ab/w4.so"
timeout -k 10 200 python -u tools/ab_libs.py $AB --spp 100 --rounds 5 > gpurun_out/w4_full.json 2> gpurun_out/w4_full.err || exit 3
timeout -k 10 300 python -u tools/ab_libs.py $AB --scene big --n-spheres 4000 --spp 100 --rounds 5 > gpurun_out/w4_big.json 2> gpurun_out/w4_big.err || exit 4
timeout -k 10 300 python -u tools/ab_libs.py $AB --scene big --n-spheres 4000 --spp 500 --row-step 8 --rounds 5 > gpurun_out/w4_big_r8.json 2> gpurun_out/w4_big_r8.err || exit 5
cat gpurun_out/w4_full.json gpurun_out/w4_big.json gpurun_out/w4_big_r8.json
