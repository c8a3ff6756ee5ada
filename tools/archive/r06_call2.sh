#!/bin/bash
# round 6, GPU call 2: the new GPU tests (pipelined drop-in, one-call vs
# general path, RCCL record of the one-GPU rehearsal), the drop-in's large
# payload timing, configs 2 and 5 on the current library (+ rocprof)
set -e
export TMPDIR=/tmp
O=gpurun_out/r06c2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_party_pipeline.py tests/test_gpu_host_entry_errors.py \
  "tests/test_gpu_aggregator.py::test_general_one_call_matches_general_path" > $O/tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/tests.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bench_rehearsal.py \
  -k "every_design and rccl" > $O/rehearsal_tests.txt 2>&1 || [ $? -eq 1 ]
tail -n 3 $O/rehearsal_tests.txt
timeout -k 10 300 python tools/party_bench.py --ab > $O/party_bench.jsonl 2> $O/party_bench.err
cut -c1-400 $O/party_bench.jsonl
timeout -k 10 200 python bench.py --clients 4 --elems 10000000 --steps 200 --warmup 20 --cpu-baseline-seconds 0 \
  --extra > $O/config2.jsonl 2> $O/config2.err
cut -c1-300 $O/config2.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_config2 -o run -- \
  python3 bench.py --clients 4 --elems 10000000 --steps 200 --warmup 20 --cpu-baseline-seconds 0 \
  > $O/config2_prof.jsonl 2> $O/config2_prof.err
timeout -k 10 500 python bench.py --clients 32 --elems 256000000 --steps 20 --warmup 5 --cpu-baseline-seconds 0 \
  --extra > $O/config5.jsonl 2> $O/config5.err
cut -c1-300 $O/config5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_config5 -o run -- \
  python3 bench.py --clients 32 --elems 256000000 --steps 20 --warmup 5 --cpu-baseline-seconds 0 \
  > $O/config5_prof.jsonl 2> $O/config5_prof.err
echo CALL2_OK
