set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_r03.txt; exit 1; }
tail -2 gpurun_out/gpu_tests_r03.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 600 python tools/loopback_bench.py --clients 32 --elems 256000000 --parties-per-process 4 --rounds 3 --dump-after 500 > gpurun_out/lb_c5.json 2> gpurun_out/lb_c5.err || { grep -v amdgpu.ids gpurun_out/lb_c5.err | tail -30; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lb_c5.json')); print('c5', d['period_s'], d['grad_elems_per_s']/1e9, d['server'])"
timeout -k 10 300 python tools/loopback_bench.py --clients 2 --elems 1000000 --rounds 20 > gpurun_out/lb_c1.json 2> gpurun_out/lb_c1.err || { grep -v amdgpu.ids gpurun_out/lb_c1.err | tail -30; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lb_c1.json')); print('c1', d['period_s'], d['grad_elems_per_s']/1e9)"
