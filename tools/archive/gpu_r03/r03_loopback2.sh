set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -40 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
timeout -k 10 400 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 6 > gpurun_out/loopback_sendfile.json 2> gpurun_out/loopback_sendfile.err || { tail gpurun_out/loopback_sendfile.err; exit 1; }
cut -c1-700 gpurun_out/loopback_sendfile.json
timeout -k 10 600 python tools/loopback_bench.py --clients 32 --elems 256000000 --parties-per-process 4 --rounds 3 > gpurun_out/loopback_c5_sendfile.json 2> gpurun_out/loopback_c5_sendfile.err || { tail gpurun_out/loopback_c5_sendfile.err; exit 1; }
cut -c1-700 gpurun_out/loopback_c5_sendfile.json
