#!/bin/bash
# Profile the bench's kernels on the GPU box: kernel trace + stats (CSV), then PMC passes (one
# rocprofv3 run per counter group; never combined with trace domains).  Output: gpurun_out/prof_<tag>/
# usage: tools/profile.sh <tag> [bench args...]      (CMD="python3 tools/bench_configs.py c3" profiles that instead)
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH=${CMD:-"python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-host $*"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1 || exit $?
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc$i -o run -- $BENCH > $OUT/pmc$i.log 2>&1 || exit $?
done
