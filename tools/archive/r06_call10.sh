#!/bin/bash
# round 6, GPU call 10: the staged (no pageable DMA) pipelined paths --
# the party tests three times over (stop at the first failure), then the
# timing with the result pool on and off
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c10
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_party_pipeline.py > $O/t_$i.txt 2>&1
  echo "pass $i: $(tail -n 1 $O/t_$i.txt)"
done
SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py --ab > $O/party_bench.jsonl 2> $O/party_bench_trace.err
cut -c1-1200 $O/party_bench.jsonl
SFL_HOSTPIPE_POOL_BYTES=0 SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py \
  > $O/party_bench_nopool.jsonl 2> $O/party_bench_nopool.err
cut -c1-900 $O/party_bench_nopool.jsonl
grep hostpipe $O/party_bench_nopool.err | tail -n 3
echo CALL10_OK
