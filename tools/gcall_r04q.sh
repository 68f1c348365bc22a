#!/bin/bash
# round 4: GPU suite at the head (split decode in the service, the one-string kernel and batches); per-string
# A/B: the service's split decoder against the candidate-chain decoder; split bench; long per-string latency
mkdir -p gpurun_out /tmp/ps_a /tmp/ps_b
export TMPDIR=/tmp
T=${T:-r04q}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -u -c "import json, torch, bench; from h2o_amd import codec; print(json.dumps(bench.per_string_latency(codec, 500)))" > gpurun_out/${T}_ps_long.json 2>&1 || exit 5
cp build/ab/libhhuff_svs.so /tmp/ps_a/libhhuff.so && cp build/ab/libhhuff_svc0.so /tmp/ps_b/libhhuff.so || exit 9
for r in 1 2; do
  LD_LIBRARY_PATH=/tmp/ps_a timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_svs_$r.jsonl 2>&1 || exit 8
  LD_LIBRARY_PATH=/tmp/ps_b timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_svc0_$r.jsonl 2>&1 || exit 8
done
timeout -k 10 300 python3 -u tools/split_bench.py split nosplit > gpurun_out/${T}_split.log 2>&1 || exit 6
