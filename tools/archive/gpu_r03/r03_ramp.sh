# How much the driver's short bench (--steps 20 --warmup 5) sits in the
# first launches' ramp: the same box, short runs with 5 / 30 warm-up steps
# and a long run, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ramp
rm -f gpurun_out/ramp/*.jsonl
for w in 5 30 5 30; do
  timeout -k 10 200 python bench.py --steps 20 --warmup $w --cpu-baseline-seconds 0 >> gpurun_out/ramp/w$w.jsonl 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --steps 2000 --warmup 20 --cpu-baseline-seconds 0 >> gpurun_out/ramp/long.jsonl 2>/dev/null || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_bench_rehearsal.py > gpurun_out/ramp/pytest.log 2>&1 || { tail -30 gpurun_out/ramp/pytest.log; exit 1; }
tail -1 gpurun_out/ramp/pytest.log
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ramp/*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f, d["warmup"], d["steps"], round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms_per_step"], 4))
PY
