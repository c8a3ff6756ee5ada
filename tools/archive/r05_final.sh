# round 5, final: smoke, the driver's bench command, the round profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke.log 2>&1 || exit 1
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_driver_form.jsonl 2> gpurun_out/r05/bench_driver_form.err || exit 1
bash tools/gpu_profile.sh
