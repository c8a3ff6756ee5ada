#!/bin/bash
# Fresh inputs every round: the caller's arrays registered lazily
# (SFL_HOSTPIPE_REGISTER=1, the default) vs staged through pinned slots by
# the feeder (0): 8 x 100M drop-in and in-process, config 5 in process;
# interleaved twice.
set -e
mkdir -p gpurun_out/regfeed
for rep in 1 2; do
  for R in 1 0; do
    SFL_HOSTPIPE_REGISTER=$R SFL_HOSTPIPE_TRACE=1 timeout -k 10 240 python tools/party_bench.py --fresh-inputs \
      --reps 3 > gpurun_out/regfeed/8x100M_reg${R}_rep$rep.jsonl 2> gpurun_out/regfeed/8x100M_reg${R}_rep$rep.trace
    SFL_HOSTPIPE_REGISTER=$R SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py --clients 32 \
      --elems 256000000 --reps 2 --in-process-only --fresh-inputs \
      > gpurun_out/regfeed/config5_reg${R}_rep$rep.jsonl 2> gpurun_out/regfeed/config5_reg${R}_rep$rep.trace
  done
done
