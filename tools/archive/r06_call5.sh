#!/bin/bash
# round 6, GPU call 5: the pipelined drop-in's result handling, three ways
# (pageable D2H into pool-faulted pages / per-chunk registration / whole
# registration after faulting), then the pipelined tests
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c5
mkdir -p $O
for mode in 0 1 whole; do
  SFL_HOSTPIPE_REGISTER_OUT=$mode SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py \
    > $O/party_bench_$mode.jsonl 2> $O/party_bench_trace_$mode.err
  echo "mode $mode: $(cut -c1-420 $O/party_bench_$mode.jsonl)"
  grep hostpipe $O/party_bench_trace_$mode.err | tail -n 2
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_party_pipeline.py > $O/tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/tests.txt
echo CALL5_OK
