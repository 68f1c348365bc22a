#!/bin/bash
# stream decode: the prefetched window landed before the flush stores (se1) against the round-3 order (se0);
# the decode GPU tests first (product build = se1)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04ak}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "decode or parity or golden" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
bash tools/gcall_ab.sh ${T} c3,c5,c2 se1 se0 || exit 4
