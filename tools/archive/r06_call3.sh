#!/bin/bash
# round 6, GPU call 3: the RCCL record with NCCL_DEBUG raised to INFO, the
# chunk-wise faulted result of the pipelined drop-in (tests + timing)
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_party_pipeline.py > $O/tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bench_rehearsal.py \
  -k "every_design and rccl" > $O/rehearsal_tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/rehearsal_tests.txt
mkdir -p $PWD/$O/rccl_logs
SFL_BENCH_RCCL_LOG_DIR=$PWD/$O/rccl_logs timeout -k 10 150 python bench.py --gpus 2 --rehearse-one-gpu \
  --rehearse-comm rccl --elems 1000003 --steps 3 --warmup 1 --variants none --host-resident-steps 0 \
  --cpu-baseline-seconds 0 > $O/reh_w2.jsonl 2> $O/reh_w2.err
python3 -c "import json; l=json.loads(open('$O/reh_w2.jsonl').read().splitlines()[-1]); print(json.dumps(l.get('rccl')))"
SFL_HOSTPIPE_TRACE=1 timeout -k 10 300 python tools/party_bench.py --ab > $O/party_bench.jsonl 2> $O/party_bench_trace.err
cut -c1-900 $O/party_bench.jsonl
grep hostpipe $O/party_bench_trace.err | tail -n 6
echo CALL3_OK
