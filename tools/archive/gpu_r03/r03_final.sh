set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_r03.txt; exit 1; }
tail -2 gpurun_out/gpu_tests_r03.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
bash tools/gpu_profile.sh > gpurun_out/profile_run.log 2>&1 || { tail -20 gpurun_out/profile_run.log; exit 1; }
tail -3 gpurun_out/profile_run.log | cut -c1-300
