#!/bin/bash
# Does a rehearsal still run slower when the test runner holds a GPU context
# of its own (W + 1 processes on the one GPU)?  The W = 8 rehearsal tests,
# first as the suite orders them (runner without a context), then after a
# GPU test module in the same runner with the reordering off
# (SFL_TEST_NO_REORDER=1).  Durations of both in gpurun_out/ctx/.
set -e
mkdir -p gpurun_out/ctx
SEL='test_bench_n_ranks_every_design and 8 or test_full_size_check_n8'
timeout -k 10 420 python -u -m pytest -v --timeout 200 --timeout-method thread --durations=0 \
  tests/test_gpu_bench_rehearsal.py -k "$SEL" > gpurun_out/ctx/ordered.log 2>&1
tail -1 gpurun_out/ctx/ordered.log
SFL_TEST_NO_REORDER=1 timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  --durations=0 tests/test_gpu_party_pipeline.py tests/test_gpu_bench_rehearsal.py \
  -k "test_large_payload_rounds_bit_exact or $SEL" > gpurun_out/ctx/with_context.log 2>&1
tail -1 gpurun_out/ctx/with_context.log
