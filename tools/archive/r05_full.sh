# round 5: the whole GPU suite, then the round profile (tools/gpu_profile.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests \
  > gpurun_out/r05/gpu_suite.log 2>&1 || { tail -30 gpurun_out/r05/gpu_suite.log; exit 1; }
tail -3 gpurun_out/r05/gpu_suite.log
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_driver_form.jsonl 2> gpurun_out/r05/bench_driver_form.err || exit 1
bash tools/gpu_profile.sh
