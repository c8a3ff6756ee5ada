#!/bin/bash
# Same-box A/B of the headline bench in the driver's exact form
# (`bench.py --gpus 1 --steps 20 --warmup 5`) across library builds:
# _ab/<tag>/ holds an older commit's tree with its own built library
# (git worktree + __graft_entry__.build(), staged by hand; _ab/ is
# git-ignored), "head" is this tree.  Runs interleaved A/B/C ROUNDS times,
# then per build one rocprofv3 kernel trace of the same form and one of a
# long form (200 timed steps: the steady state after the clock ramp), and
# one SQ census pass (VALU / SALU per launch).
# usage: tools/ab_driver_form.sh "r03 r04 head" 6
set -e
export TMPDIR=/tmp
TAGS=${1:-"r03 r04 head"}
ROUNDS=${2:-6}
OUT=$PWD/gpurun_out/ab
mkdir -p $OUT
dir_of() { if [ "$1" = head ]; then echo "$PWD"; else echo "$PWD/_ab/$1"; fi; }
for i in $(seq 1 $ROUNDS); do
  for t in $TAGS; do
    d=$(dir_of $t)
    line=$(cd $d && timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2> $OUT/bench_${t}_$i.err | tail -n 1)
    echo "{\"tag\": \"$t\", \"pass\": $i, \"line\": $line}" >> $OUT/ab_driver_form.jsonl
    echo "$t pass $i: $(echo "$line" | cut -c1-120)"
  done
done
for t in $TAGS; do
  d=$(dir_of $t)
  (cd $d && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_short_$t -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_short_$t.jsonl 2> $OUT/prof_short_$t.err)
  echo "$t rocprof short done"
  (cd $d && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_long_$t -o run -- \
    python3 bench.py --gpus 1 --steps 200 --warmup 20 --cpu-baseline-seconds 0 > $OUT/prof_long_$t.jsonl 2> $OUT/prof_long_$t.err)
  echo "$t rocprof long done"
  (cd $d && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq_$t -o run -- \
    python3 bench.py --gpus 1 --steps 10 --warmup 2 --cpu-baseline-seconds 0 > $OUT/pmc_sq_$t.jsonl 2> $OUT/pmc_sq_$t.err)
  echo "$t pmc done"
done
echo AB_OK
