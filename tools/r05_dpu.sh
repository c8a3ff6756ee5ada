# A/B of k_dp_perturb forms: blocks in flight per lane (SA_DP_UNROLL 1 / 2 / 4),
# with and without the scheduling barrier after the loads
set -o pipefail
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/dp_unroll_ab.txt
for v in main nosb u1 u4 main nosb u1 u4; do
  if [ $v = main ]; then export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa.so; else export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_$v.so; fi
  echo "== $v" >> gpurun_out/r05/dp_unroll_ab.txt
  timeout -k 10 100 python tools/dp_bench.py --passes 2 >> gpurun_out/r05/dp_unroll_ab.txt 2>&1 || exit 1
done
