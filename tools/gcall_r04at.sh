#!/bin/bash
# final head: GPU suite, smoke, bench; then the block-list grid cap (g32 / g128) on c5 decode and long strings
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04at}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 5
bash tools/gcall_ab.sh ${T} c5 g32 g128 g32 g128 || exit 6
timeout -k 10 400 python3 -u tools/split_bench.py g32 g128 > gpurun_out/${T}_split_ab.log 2>&1 || exit 7
