set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/t_loop.log 2>&1 || { tail -30 gpurun_out/t_loop.log; exit 1; }
tail -1 gpurun_out/t_loop.log
nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"
for o in "" "--overlap" "--overlap --sendfile" "--sendfile"; do
  timeout -k 10 200 python tools/socket_floor.py --clients 8 --elems 100000000 --rounds 4 $o >> gpurun_out/socket_floor.jsonl || exit 1
done
cat gpurun_out/socket_floor.jsonl | cut -c 1-400
timeout -k 10 400 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 5 > gpurun_out/loopback_stages.json 2> gpurun_out/loopback_stages.err || { tail gpurun_out/loopback_stages.err; exit 1; }
cat gpurun_out/loopback_stages.json
