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
timeout -k 10 200 python bench.py --clients 4 --elems 10000000 --steps 200 --warmup 20 --cpu-baseline-seconds 0 \
  --extra > $O/config2.jsonl 2> $O/config2.err
python3 -c "import json; l=json.loads(open('$O/config2.jsonl').read().splitlines()[-1]); print(json.dumps(l['extra']))"
echo CALL4_OK
