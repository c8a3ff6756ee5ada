# Tuning: kernel time of the issue-priority rotation window variants vs the
# default library (SA_PRIO=14), interleaved.
set -e
mkdir -p gpurun_out/prio
rm -f gpurun_out/prio/kb.jsonl
for v in "" _p0 _p12 _p13 _p15 "" _p0 _p13; do
  SFL_SA_LIB=sfl_amd/lib/libsfl_sa${v}.so timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 --shapes 8:1,8:2,8:8 >> gpurun_out/prio/kb.jsonl 2>/dev/null
done
