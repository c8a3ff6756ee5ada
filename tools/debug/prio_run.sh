# Tuning: kernel time of the issue-priority rotation variants vs the default
# library, and the wave timeline with rotation on.
set -e
mkdir -p gpurun_out/prio
rm -f gpurun_out/prio/kb.jsonl
for v in "" _p12 _p13 _p14 _p15 _p16 "" _p13 _p14; do
  lib=sfl_amd/lib/libsfl_sa${v}.so
  SFL_SA_LIB=$lib timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 --shapes 8:1,8:2,8:4,8:8 >> gpurun_out/prio/kb.jsonl
done
SFL_SA_LIB=sfl_amd/lib/libsfl_sa_tsp14.so timeout -k 10 120 python -u tools/wave_timeline.py --launches 2 > gpurun_out/prio/tl_p14.jsonl
