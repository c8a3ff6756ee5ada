# A/B of k_dp_perturb forms: non-temporal vs plain 16-B accesses, blocks in
# flight per lane, grid multiple of the occupancy
set -o pipefail
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/dp_forms_ab.txt
for v in main plain1 plain2 g2 plaing4 main plain1 plain2 g2 plaing4; do
  if [ $v = main ]; then export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa.so; else export SFL_SA_LIB=$PWD/sfl_amd/lib/libsfl_sa_$v.so; fi
  echo "== $v" >> gpurun_out/r05/dp_forms_ab.txt
  timeout -k 10 100 python tools/dp_bench.py --passes 2 >> gpurun_out/r05/dp_forms_ab.txt 2>&1 || exit 1
done
