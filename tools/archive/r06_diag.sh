#!/bin/bash
# round 6: why the rehearsal's RCCL log came back empty; phase times of the
# pipelined drop-in
set -e
export TMPDIR=/tmp
O=gpurun_out/diag
mkdir -p $O $PWD/gpurun_out/rccl_logs
(env | grep -i nccl || true) > $O/env.txt
SFL_BENCH_RCCL_LOG_DIR=$PWD/gpurun_out/rccl_logs timeout -k 10 150 python bench.py --gpus 2 --rehearse-one-gpu \
  --rehearse-comm rccl --elems 1000003 --steps 3 --warmup 1 --variants none --host-resident-steps 0 \
  --cpu-baseline-seconds 0 > $O/reh.jsonl 2> $O/reh.err || echo "rehearsal rc=$?"
ls -laR gpurun_out/rccl_logs > $O/logs_ls.txt
python3 -c "import json; l=json.loads(open('$O/reh.jsonl').read().splitlines()[-1]); print(json.dumps(l.get('rccl')))"
SFL_HOSTPIPE_TRACE=1 timeout -k 10 200 python tools/party_bench.py --reps 3 > $O/party_bench.jsonl 2> $O/party_bench_trace.err
cut -c1-600 $O/party_bench.jsonl
grep hostpipe $O/party_bench_trace.err | tail -n 12
echo DIAG_OK
