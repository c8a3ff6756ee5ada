#!/bin/bash
# round 6, GPU call 6: pipelined results into numpy memory (pageable D2H)
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c6
mkdir -p $O
SFL_HOSTPIPE_TRACE=1 timeout -k 10 400 python tools/party_bench.py --ab > $O/party_bench.jsonl 2> $O/party_bench_trace.err
cut -c1-1500 $O/party_bench.jsonl
grep hostpipe $O/party_bench_trace.err | tail -n 4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_party_pipeline.py > $O/tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/tests.txt
echo CALL6_OK
