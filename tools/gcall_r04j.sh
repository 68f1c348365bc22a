#!/bin/bash
# round 4: per-string service with two polls in flight (A/B, HHUFF_SVC_PIPE) against the head, interleaved
mkdir -p gpurun_out /tmp/svp
export TMPDIR=/tmp
T=${T:-r04j}
cp build/ab/libhhuff_svp.so /tmp/svp/libhhuff.so
for r in 1 2; do
  timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_head_$r.jsonl 2>&1 || exit 8
  LD_LIBRARY_PATH=/tmp/svp timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_svp_$r.jsonl 2>&1 || exit 9
done
