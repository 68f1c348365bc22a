#!/bin/bash
# round 4: GPU suite at the head (split decode of long strings, tagged per-string output chunks); A/B:
# chunk sizes, 64-B stream flush segments, per-string with tagged output chunks against the previous service
mkdir -p gpurun_out /tmp/ps_base /tmp/ps_tag
export TMPDIR=/tmp
T=${T:-r04p}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -u tools/split_bench.py split nosplit > gpurun_out/${T}_split.log 2>&1 || exit 6
timeout -k 10 300 python3 -u -c "import json, torch, bench; from h2o_amd import codec; print(json.dumps(bench.per_string_latency(codec, 500)))" > gpurun_out/${T}_ps_long.json 2>&1 || exit 5
cp build/ab/libhhuff_base5.so /tmp/ps_base/libhhuff.so && cp build/ab/libhhuff_tag.so /tmp/ps_tag/libhhuff.so || exit 9
for r in 1 2; do
  LD_LIBRARY_PATH=/tmp/ps_base timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_base_$r.jsonl 2>&1 || exit 8
  LD_LIBRARY_PATH=/tmp/ps_tag timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_tag_$r.jsonl 2>&1 || exit 8
done
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_enco c4,c2 base4 e192 e320 || exit 7
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_seg c3,c5 base5 seg64 seg32 || exit 7
