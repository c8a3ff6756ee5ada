set -e
mkdir -p gpurun_out/noreorder
SFL_TEST_NO_REORDER=1 timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread --durations=25 -m gpu tests/ > gpurun_out/noreorder/gpu_suite.log 2>&1
tail -1 gpurun_out/noreorder/gpu_suite.log
