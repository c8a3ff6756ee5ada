# Per-rank kernel shapes (C = 8 over W = 1, 2, 4, 8) and the L = 8 size
# sweep with the default library -> gpurun_out/shapes/.
set -e
mkdir -p gpurun_out/shapes
timeout -k 10 120 python -u tools/kernel_bench.py --rounds 7 > gpurun_out/shapes/kernel_bench_shapes.json
rm -f gpurun_out/shapes/size_sweep.jsonl
for n in 262144 12500000 25000000 50000000 100000000 200000000 400000000; do
  timeout -k 10 120 python -u tools/kernel_bench.py --shapes 8:1 --elems $n --rounds 5 >> gpurun_out/shapes/size_sweep.jsonl
done
