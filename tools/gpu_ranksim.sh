cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for v in ${VARIANTS:-g0 g1}; do
  cp ab/$v.so raytracing-with-zig_amd/librtzig.so
  timeout -k 10 200 python -u tools/rank_sim.py --spp 500 --reps 3 > gpurun_out/rank_$v.json 2> gpurun_out/rank_$v.err
  rc=$?; echo "$v rc=$rc"; cat gpurun_out/rank_$v.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/rank_$v.err; exit $rc; }
done
