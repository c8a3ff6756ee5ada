#!/bin/bash
# Chunks per pipelined server / in-process call (SFL_HOSTPIPE_CHUNKS 8 vs 16)
# at 8 x 100M, reused inputs, interleaved three times on one box.
set -e
mkdir -p gpurun_out/chunks
for rep in 1 2 3; do
  for K in 8 16; do
    SFL_HOSTPIPE_CHUNKS=$K timeout -k 10 200 python tools/party_bench.py --reps 5 \
      > gpurun_out/chunks/k${K}_rep$rep.jsonl 2> gpurun_out/chunks/k${K}_rep$rep.err
  done
done
