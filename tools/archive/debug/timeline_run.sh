# Wave timelines of the 8-client launch without (SA_PRIO=0) and with the
# issue-priority rotation (default build), then the round profile.
set -e
mkdir -p gpurun_out/timeline
SFL_SA_LIB=sfl_amd/lib/libsfl_sa_ts0.so timeout -k 10 120 python -u tools/wave_timeline.py --launches 3 > gpurun_out/timeline/prio_off.jsonl
cp gpurun_out/wave_timeline.json gpurun_out/timeline/prio_off.json
SFL_SA_LIB=sfl_amd/lib/libsfl_sa_ts.so timeout -k 10 120 python -u tools/wave_timeline.py --launches 3 > gpurun_out/timeline/prio_on.jsonl
cp gpurun_out/wave_timeline.json gpurun_out/timeline/prio_on.json
bash tools/gpu_profile.sh > gpurun_out/profile.log 2>&1
