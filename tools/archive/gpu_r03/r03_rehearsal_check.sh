# The W-rank one-GPU bench rehearsal (test_gpu_bench_rehearsal.py) twice,
# with per-test timing, to see whether its world-8 case is stable.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rehearsal
timeout -k 10 400 python -u -m pytest -v --durations=0 --timeout 200 --timeout-method thread tests/test_gpu_bench_rehearsal.py > gpurun_out/rehearsal/run1.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -v --durations=0 --timeout 200 --timeout-method thread tests/test_gpu_bench_rehearsal.py > gpurun_out/rehearsal/run2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|s call" gpurun_out/rehearsal/run*.log
exit $rc
