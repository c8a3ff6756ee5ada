# Tuning: where the non-draw time goes -- kernel time of the SA_ABLATE
# variants (results wrong, timing only) against the default build.
set -e
mkdir -p gpurun_out/abl
rm -f gpurun_out/abl/kb.jsonl
for v in "" _abl2 _abl8 _abl32 _abl128 ""; do
  SFL_SA_LIB=sfl_amd/lib/libsfl_sa${v}.so timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 --shapes 8:1,8:8 >> gpurun_out/abl/kb.jsonl 2>/dev/null
done
