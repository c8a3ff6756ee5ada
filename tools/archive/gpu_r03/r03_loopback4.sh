set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/socket_floor_r03.jsonl
for o in "--overlap" "--overlap --sendfile" "--overlap --sendfile --sendfile-side clients" "--overlap --sendfile --sendfile-side server" "" "--sendfile"; do
  timeout -k 5 120 python tools/socket_floor.py --clients 8 --elems 100000000 --rounds 4 --timeout 60 $o >> gpurun_out/socket_floor_r03.jsonl 2>> gpurun_out/socket_floor_r03.err || echo "FAILED: $o" >> gpurun_out/socket_floor_r03.jsonl
done
cut -c100-420 gpurun_out/socket_floor_r03.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -40 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
timeout -k 10 200 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 6 --dump-after 120 > gpurun_out/loopback_sendfile.json 2> gpurun_out/loopback_sendfile.err || { grep -v amdgpu.ids gpurun_out/loopback_sendfile.err | tail -30; exit 1; }
cut -c1-600 gpurun_out/loopback_sendfile.json
