# A/B of k_dp_perturb: the grid-stride form (main) vs the tile form
# (SA_DP_TILE = 1, 2, 4 Philox blocks per lane, one pass per workgroup);
# the DP parity tests run once against each tile variant first
set -o pipefail
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/dp_tile_ab.txt gpurun_out/r05/dp_tile_tests.log
for v in tile1 tile2 tile4; do
  SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_$v.so timeout -k 10 200 python -u -m pytest -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_dp.py >> gpurun_out/r05/dp_tile_tests.log 2>&1 || exit 1
done
for v in main tile1 tile2 tile4 main tile1 tile2 tile4; do
  if [ $v = main ]; then export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa.so; else export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_$v.so; fi
  echo "== $v" >> gpurun_out/r05/dp_tile_ab.txt
  timeout -k 10 100 python tools/dp_bench.py --passes 2 >> gpurun_out/r05/dp_tile_ab.txt 2>&1 || exit 1
done
