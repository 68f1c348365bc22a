#!/bin/bash
# round 4 session 1: GPU suite at the head (incl. the bench self-spawn test), smoke, per-string threads, bench,
# c3 profile, stream-decode shape A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 || exit 4
timeout -k 10 300 ./tools/per_string_bench 1 2 4 8 16 32 64 > gpurun_out/r04a_per_string.jsonl 2>&1 || exit 8
HHUFF_SVC_WAVES=2 timeout -k 10 120 ./tools/per_string_bench 1 16 >> gpurun_out/r04a_per_string.jsonl 2>&1 || exit 9
timeout -k 10 600 python3 bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 5
CMD="python3 tools/bench_configs.py c3" timeout -k 10 600 bash tools/profile.sh r04a_c3 || exit 6
timeout -k 10 600 bash tools/gcall_ab.sh r04a_stream c3,c5 base ms t12 t16b || exit 7
