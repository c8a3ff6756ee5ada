set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 tools/microbench/stream_rate > gpurun_out/stream_rate.jsonl 2>&1 || { tail gpurun_out/stream_rate.jsonl; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_integration_stub.py tests/test_gpu_rejection.py tests/test_gpu_aggregator.py tests/test_compat_secretflow.py tests/test_gpu_loopback.py > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
cat gpurun_out/stream_rate.jsonl
