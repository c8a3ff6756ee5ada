# Copy the outputs of tools/gpu_profile.sh (+ draw_issue / kernel_bench runs)
# from gpurun_out/ into profiles/r01/ and print the numbers DESIGN.md quotes.
set -e
P=profiles/r01
tail -1 gpurun_out/bench.jsonl > $P/bench_n1.jsonl
tail -1 gpurun_out/bench_prof.jsonl > $P/bench_n1_under_rocprof.jsonl
cp gpurun_out/prof_bench/run_kernel_stats.csv $P/bench_n1_kernel_stats.csv
cp gpurun_out/prof_bench/run_kernel_trace.csv $P/bench_n1_kernel_trace.csv
cp gpurun_out/pmc_fetch/run_counter_collection.csv $P/pmc_fetch_size.csv
cp gpurun_out/pmc_write/run_counter_collection.csv $P/pmc_write_size.csv
[ -f gpurun_out/draw_issue_new.txt ] && cp gpurun_out/draw_issue_new.txt $P/draw_issue_microbench.txt
[ -f gpurun_out/kb_new.jsonl ] && grep '^{' gpurun_out/kb_new.jsonl > $P/kernel_bench_shapes.json
python3 - <<'PY'
import csv, collections, json
P = "profiles/r01"
rows = list(csv.reader(open("gpurun_out/pmc_sq/run_counter_collection.csv")))
keep = [rows[0]] + [r for r in rows[1:] if "k_clients" in r[8]]
csv.writer(open(f"{P}/pmc_sq_census.csv", "w"), quoting=csv.QUOTE_ALL).writerows(keep)
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f"{P}/pmc_sq_census.csv")):
    by[(r["Kernel_Name"][:45], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in by.items():
    if "8, 0" in k[0]:
        wc = d["SQ_WAVE_CYCLES"]
        print("census L8: valu/draw %.2f salu/draw %.2f active_valu %.3f wait_any %.3f wait_inst %.3f" % (
            d["SQ_INSTS_VALU"] * 64 / 2.8e9, d["SQ_INSTS_SALU"] * 64 / 2.8e9, d["SQ_ACTIVE_INST_VALU"] / wc,
            d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc))
        break
for f in ("bench_n1.jsonl", "bench_n1_under_rocprof.jsonl"):
    d = json.loads(open(f"{P}/{f}").read()); r = d["roofline"]
    print(f, "ms %.4f  G/s %.1f  kernel %.4f  TB/s %.3f frac %.4f draws %.3fe12 valu_frac %.3f cpu %s" % (
        d["ms_per_step"], d["value"] / 1e9, r["kernel_ms"], r["achieved"] / 1e3, r["frac"],
        r["valu"]["draws_per_s"] / 1e12, r["valu"]["frac"], d["cpu_baseline"] and round(d["cpu_baseline"]["value"] / 1e6, 2)))
rows = [r for r in csv.DictReader(open(f"{P}/bench_n1_kernel_trace.csv")) if "k_clients" in r["Kernel_Name"]]
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print("trace: %d dispatches avg %.4f, last 20 avg %.4f, first %s" % (len(ds), sum(ds) / len(ds), sum(ds[-20:]) / 20,
      [round(x, 2) for x in ds[:8]]))
for l in open(f"{P}/kernel_bench_shapes.json"):
    d = json.loads(l)
    print("shapes", [(c["L"], round(c["ms_median"], 3), round(c["draws_per_s"] / 1e12, 3)) for c in d["cases"]])
PY
