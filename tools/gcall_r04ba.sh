#!/bin/bash
# final-head verification after the long-encoder commit: full gpu suite, smoke, bench, kernel-trace stats
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04ba}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 4
timeout -k 10 300 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-host > gpurun_out/${T}_prof.log 2>&1 || exit 6
