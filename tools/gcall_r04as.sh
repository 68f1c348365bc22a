#!/bin/bash
# per-string launch path: spin on the result length (wait_one) against stream synchronisation, alternating (T=r04av: 64 KB added)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04as}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "per_string or launch_path or dropin or capi" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
for m in 0 1 0 1; do
  HHUFF_LONG_ENC=1 HHUFF_ONE_SYNC=$m timeout -k 10 200 python3 -u tools/one_wait_ab.py >> gpurun_out/${T}_one_wait_ab.jsonl 2>> gpurun_out/${T}_one_wait_ab.err || exit 4
done
