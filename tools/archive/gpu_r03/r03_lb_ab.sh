set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -40 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
timeout -k 10 900 python tools/loopback_bench.py --clients 32 --elems 256000000 --parties-per-process 4 --rounds 2 --ab 1 --dump-after 800 > gpurun_out/lb_c5_ab.jsonl 2> gpurun_out/lb_c5_ab.err || { grep -v amdgpu.ids gpurun_out/lb_c5_ab.err | tail -30; exit 1; }
python -c "
import json
for l in open('gpurun_out/lb_c5_ab.jsonl'):
    d=json.loads(l); print('c5', d['send'], d['wait'], d['client_rx'], round(d['period_s'],3), round(d['grad_elems_per_s']/1e9,2))"
timeout -k 10 600 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 5 --ab 2 > gpurun_out/lb_c3_ab.jsonl 2> gpurun_out/lb_c3_ab.err || { grep -v amdgpu.ids gpurun_out/lb_c3_ab.err | tail -30; exit 1; }
python -c "
import json
for l in open('gpurun_out/lb_c3_ab.jsonl'):
    d=json.loads(l); print('8x100M', d['ab_pass'], d['send'], d['wait'], d['client_rx'], round(d['period_s'],3), round(d['grad_elems_per_s']/1e9,2))"
