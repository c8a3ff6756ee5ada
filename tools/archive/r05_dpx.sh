# A/B of the streaming kernels' workgroup -> tile mapping (sa_tiles.h): the
# dispatcher's round-robin over the 8 XCDs (main, SA_XCD_TILES=0) vs
# XCD-contiguous runs of tiles (the _xcd build: make VARIANT=_xcd
# EXTRA=-DSA_XCD_TILES=1); DP perturb (tools/dp_bench.py) and the server
# kernels (tools/server_bench.py).  The GPU parity tests of those kernels run
# against the variant first.  (profiles/r05/xcd_tiles_ab.txt was recorded
# when main was the contiguous build and the variant _noxcd.)
set -o pipefail
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/xcd_tiles_ab.txt
SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_xcd.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dp.py \
  tests/test_gpu_parity.py tests/test_gpu_aggregator.py > gpurun_out/r05/xcd_tiles_tests.log 2>&1 || exit 1
for v in main xcd main xcd main xcd; do
  if [ $v = main ]; then export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa.so; else export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_$v.so; fi
  echo "== $v" >> gpurun_out/r05/xcd_tiles_ab.txt
  timeout -k 10 100 python tools/dp_bench.py --passes 2 >> gpurun_out/r05/xcd_tiles_ab.txt 2>&1 || exit 1
  timeout -k 10 100 python tools/server_bench.py >> gpurun_out/r05/xcd_tiles_ab.txt 2>&1 || exit 1
done
