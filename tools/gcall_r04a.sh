#!/bin/bash
# round 4 session 1: GPU suite at the head (incl. the bench self-spawn test), smoke, bench, c3 profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 5
CMD="python3 tools/bench_configs.py c3" timeout -k 10 600 bash tools/profile.sh r04a_c3 || exit 6
