#!/bin/bash
# Copy tools/gpu_profile.sh's outputs from gpurun_out/ into profiles/<round>/.
set -e
P=profiles/${1:?round, e.g. r03}
mkdir -p $P
tail -1 gpurun_out/bench.jsonl > $P/bench_n1.jsonl
tail -1 gpurun_out/bench_prof.jsonl > $P/bench_n1_under_rocprof.jsonl
tail -1 gpurun_out/bench_driver_form.jsonl > $P/bench_n1_driver_form.jsonl
tail -1 gpurun_out/bench_driver_form_prof.jsonl > $P/bench_n1_driver_form_under_rocprof.jsonl
cp gpurun_out/prof_driver_form/run_kernel_stats.csv $P/bench_n1_driver_form_kernel_stats.csv
cp gpurun_out/prof_driver_form/run_kernel_trace.csv $P/bench_n1_driver_form_kernel_trace.csv
tail -1 gpurun_out/bench_extra.jsonl > $P/bench_n1_extra.jsonl
tail -1 gpurun_out/bench_dist_world1.jsonl > $P/bench_dist_world1_all_designs.jsonl
cp gpurun_out/prof_bench/run_kernel_stats.csv $P/bench_n1_kernel_stats.csv
cp gpurun_out/prof_bench/run_kernel_trace.csv $P/bench_n1_kernel_trace.csv
cp gpurun_out/prof_server/run_kernel_stats.csv $P/server_kernel_stats.csv
cp gpurun_out/pmc_fetch/run_counter_collection.csv $P/pmc_fetch_size.csv
cp gpurun_out/pmc_write/run_counter_collection.csv $P/pmc_write_size.csv
cp gpurun_out/pmc_server_fetch/run_counter_collection.csv $P/pmc_server_fetch_size.csv
cp gpurun_out/pmc_server_write/run_counter_collection.csv $P/pmc_server_write_size.csv
cp gpurun_out/prof_dp/run_kernel_stats.csv $P/dp_kernel_stats.csv
cp gpurun_out/pmc_dp_fetch/run_counter_collection.csv $P/pmc_dp_fetch_size.csv
cp gpurun_out/pmc_dp_write/run_counter_collection.csv $P/pmc_dp_write_size.csv
grep '^{' gpurun_out/dp_bench.jsonl > $P/dp_bench.jsonl
python3 - "$P" <<'PY'
import csv, sys
P = sys.argv[1]
rows = list(csv.reader(open("gpurun_out/pmc_sq/run_counter_collection.csv")))
keep = [rows[0]] + [r for r in rows[1:] if "k_clients" in r[8]]
csv.writer(open(f"{P}/pmc_sq_census.csv", "w"), quoting=csv.QUOTE_ALL).writerows(keep)
PY
grep '^{' gpurun_out/kb_shapes.jsonl > $P/kernel_bench_shapes.json
grep '^{' gpurun_out/draw_ops.jsonl > $P/draw_ops.jsonl
grep '^{' gpurun_out/stream_rate.jsonl > $P/stream_rate.jsonl
grep '^{' gpurun_out/server_bench.jsonl > $P/server_bench.jsonl
echo saved to $P
