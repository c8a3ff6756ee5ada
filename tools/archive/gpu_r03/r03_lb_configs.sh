set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -40 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
timeout -k 10 600 python tools/loopback_bench.py --clients 32 --elems 256000000 --parties-per-process 4 --rounds 2 --dump-after 500 > gpurun_out/lb_c5.json 2> gpurun_out/lb_c5.err || { grep -v amdgpu.ids gpurun_out/lb_c5.err | tail -30; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lb_c5.json')); print('c5', d['period_s'], d['grad_elems_per_s']/1e9, d['server'])"
timeout -k 10 300 python tools/loopback_bench.py --clients 2 --elems 1000000 --rounds 20 > gpurun_out/lb_c1.json 2> gpurun_out/lb_c1.err || { grep -v amdgpu.ids gpurun_out/lb_c1.err | tail -30; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lb_c1.json')); print('c1', d['period_s'], d['grad_elems_per_s']/1e9)"
timeout -k 10 300 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 6 > gpurun_out/lb_c3.json 2> gpurun_out/lb_c3.err || { grep -v amdgpu.ids gpurun_out/lb_c3.err | tail -30; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/lb_c3.json')); print('8x100M', d['period_s'], d['grad_elems_per_s']/1e9)"
