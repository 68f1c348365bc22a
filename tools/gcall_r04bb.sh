#!/bin/bash
# per-string encode of the 64-KB value: one-block encoder (HHUFF_LONG_ENC=1) against one lane (0), alternating processes
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04bb}
for m in 0 1 0 1; do
  HHUFF_LONG_ENC=$m timeout -k 10 200 python3 -u tools/one_wait_ab.py | sed "s/^{/{\"long_enc\": \"$m\", /" >> gpurun_out/${T}_long_enc_ab.jsonl 2>> gpurun_out/${T}_long_enc_ab.err || exit 4
done
