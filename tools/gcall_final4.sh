#!/bin/bash
# round 4, final: the head -- GPU suite, smoke, per-string threads, bench, c4 / c3 / c5 traces + PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04z}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 4
timeout -k 10 300 ./tools/per_string_bench 1 2 4 8 16 32 64 > gpurun_out/${T}_per_string.jsonl 2>&1 || exit 8
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 5
timeout -k 10 900 bash tools/profile.sh ${T}_c4 --no-extra || exit 6
CMD="python3 tools/bench_configs.py c3" timeout -k 10 600 bash tools/profile.sh ${T}_c3 || exit 6
CMD="python3 tools/bench_configs.py c5" timeout -k 10 600 bash tools/profile.sh ${T}_c5 || exit 6
