#!/bin/bash
# Chunks of registered copies issued ahead (SFL_HOSTPIPE_LOOKAHEAD 1 vs 2):
# config 5 in process with fresh inputs (lazy registration on the caller's
# thread between issues), interleaved twice.
set -e
mkdir -p gpurun_out/lookahead
for rep in 1 2; do
  for K in 1 2; do
    SFL_HOSTPIPE_LOOKAHEAD=$K SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py --clients 32 \
      --elems 256000000 --reps 2 --in-process-only --fresh-inputs \
      > gpurun_out/lookahead/config5_k${K}_rep$rep.jsonl 2> gpurun_out/lookahead/config5_k${K}_rep$rep.trace
  done
done
