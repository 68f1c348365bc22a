#!/bin/bash
# round 4: GPU suite at the head (windowed split decode, one-string kernel up to 32 KB); split bench; long
# per-string latency; per-string scaling at the head
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04r}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -u tools/split_bench.py split nosplit > gpurun_out/${T}_split.log 2>&1 || exit 6
timeout -k 10 300 python3 -u -c "import json, torch, bench; from h2o_amd import codec; print(json.dumps(bench.per_string_latency(codec, 500)))" > gpurun_out/${T}_ps_long.json 2>&1 || exit 5
timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_head.jsonl 2>&1 || exit 8
