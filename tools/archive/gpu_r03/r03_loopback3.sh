set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python tools/loopback_bench.py --clients 8 --elems 100000000 --rounds 2 --dump-after 60 > gpurun_out/loopback_dbg.json 2> gpurun_out/loopback_dbg.err
echo rc=$?
grep -v amdgpu.ids gpurun_out/loopback_dbg.err | head -150
