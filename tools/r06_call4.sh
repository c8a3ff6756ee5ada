#!/bin/bash
# round 6, GPU call 4: the pipelined drop-in with a private result mapping
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_party_pipeline.py > $O/tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/tests.txt
SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py --ab > $O/party_bench.jsonl 2> $O/party_bench_trace.err
cut -c1-900 $O/party_bench.jsonl
grep hostpipe $O/party_bench_trace.err | tail -n 6
echo CALL4_OK
