#!/bin/bash
# Interleaved kernel timing of library variants: tools/debug/ab_variants.sh OUT "v1 v2 ..." [shapes] [passes]
# (variant "" = the product build sfl_amd/lib/libsfl_sa.so; others sfl_amd/lib/libsfl_sa<v>.so)
set -e
out=$1; vars=$2; shapes=${3:-8:1,8:2,8:4,8:8}; passes=${4:-3}
mkdir -p gpurun_out/$out
rm -f gpurun_out/$out/kb.jsonl
for p in $(seq $passes); do
  for v in $vars; do
    [ "$v" = "base" ] && v=""
    SFL_SA_LIB=sfl_amd/lib/libsfl_sa${v}.so timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 --shapes $shapes >> gpurun_out/$out/kb.jsonl
  done
done
echo AB_OK
