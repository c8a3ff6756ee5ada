#!/bin/bash
# Lazy input registration A/B on the GPU box, after the pipeline tests:
# tools/party_bench.py with fresh inputs every round (registration inside
# every call) -- whole arrays on entry (SFL_HOSTPIPE_LAZY_REGISTER=0),
# chunk by chunk (SFL_HOSTPIPE_LAZY_GROWTH=1), geometric (growth 2) -- at
# 8 x 100M (drop-in and in-process) and config 5 (32 x 256M, in-process),
# interleaved.
set -e
mkdir -p gpurun_out/lazy
export SFL_HOSTPIPE_TRACE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_party_pipeline.py \
  > gpurun_out/lazy/pipeline_tests.log 2>&1
tail -1 gpurun_out/lazy/pipeline_tests.log
for rep in 1 2; do
  for V in "0 2" "1 1" "1 2"; do
    set -- $V
    tag=lazy$1_growth$2_rep$rep
    SFL_HOSTPIPE_LAZY_REGISTER=$1 SFL_HOSTPIPE_LAZY_GROWTH=$2 timeout -k 10 240 python tools/party_bench.py \
      --fresh-inputs --reps 3 > gpurun_out/lazy/8x100M_$tag.jsonl 2> gpurun_out/lazy/8x100M_$tag.trace
    SFL_HOSTPIPE_LAZY_REGISTER=$1 SFL_HOSTPIPE_LAZY_GROWTH=$2 timeout -k 10 300 python tools/party_bench.py \
      --clients 32 --elems 256000000 --reps 2 --in-process-only --fresh-inputs \
      > gpurun_out/lazy/config5_$tag.jsonl 2> gpurun_out/lazy/config5_$tag.trace
  done
done
