#!/bin/bash
# block split decode (split_decode_block) in the block list and in one_string_kernel: the per-string, split and
# decode GPU tests, then the full bench line (per-string long-value latencies included)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04ap}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "split or launch_path or long or per_string or decode or dropin or capi" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
timeout -k 10 500 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 4
