#!/bin/bash
# sample GPU clock / power while the bench runs (read-only queries)
timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --steps 4000 > gpurun_out/bclk.jsonl 2>&1 &
pid=$!
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  sleep 1
  (rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|Power|Temperature|fclk|mclk" ) >> gpurun_out/clk.txt || true
  echo "--- $i" >> gpurun_out/clk.txt
done
wait $pid
