#!/bin/bash
# Round refresh of the secondary BASELINE configs (not the headline line):
# config 2 (4 clients x 10M), config 5 device-resident on one GPU
# (32 clients x 256M), the config-4 FL round, the host-resident loopback
# round (8 x 100M), and a wave timeline of the 8-client launch.
set -e
out=gpurun_out/secondary
mkdir -p $out
timeout -k 10 300 python bench.py --clients 4 --elems 10000000 --cpu-baseline-seconds 0 > $out/bench_config2_4x10M.jsonl 2> $out/c2.err
timeout -k 10 400 python bench.py --clients 32 --elems 256000000 --steps 5 --warmup 2 --cpu-baseline-seconds 0 > $out/config5_device_1gpu.jsonl 2> $out/c5.err
timeout -k 10 300 python tools/fl_round_bench.py > $out/fl_round_config4.json 2> $out/fl.err
timeout -k 10 400 python tools/loopback_bench.py > $out/loopback_8x100M.json 2> $out/lb.err
SFL_SA_LIB=sfl_amd/lib/libsfl_sa_ts.so timeout -k 10 200 python tools/wave_timeline.py --launches 3 > $out/wave_timeline.jsonl 2> $out/ts.err
echo SECONDARY_OK
