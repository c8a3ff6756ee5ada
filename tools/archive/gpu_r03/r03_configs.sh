set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --clients 4 --elems 10000000 --cpu-baseline-seconds 3 > gpurun_out/c2.jsonl 2> gpurun_out/c2.err || { tail gpurun_out/c2.err; exit 1; }
cut -c1-300 gpurun_out/c2.jsonl
timeout -k 10 300 python bench.py --clients 32 --elems 256000000 --steps 30 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/c5.jsonl 2> gpurun_out/c5.err || { tail gpurun_out/c5.err; exit 1; }
cut -c1-300 gpurun_out/c5.jsonl
timeout -k 10 300 python tools/config1_bench.py > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail gpurun_out/c1.err; exit 1; }
cut -c1-400 gpurun_out/c1.json
timeout -k 10 400 python tools/fl_round_bench.py > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
cut -c1-600 gpurun_out/c4.json
