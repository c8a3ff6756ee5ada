set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -40 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
timeout -k 10 600 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 5 --ab 2 --dump-after 500 > gpurun_out/loopback_ab.jsonl 2> gpurun_out/loopback_ab.err || { grep -v amdgpu.ids gpurun_out/loopback_ab.err | tail -30; exit 1; }
python -c "
import json
for l in open('gpurun_out/loopback_ab.jsonl'):
    d=json.loads(l); print(d['ab_pass'], d['send'], d['wait'], round(d['period_s'],3), round(d['grad_elems_per_s']/1e9,2))
"
