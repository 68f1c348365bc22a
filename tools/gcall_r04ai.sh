#!/bin/bash
# per-string: the hot mailbox's header-line pieces polled with the headers (inl2) against the head (base9);
# the per-string GPU tests first
mkdir -p gpurun_out /tmp/pa /tmp/pb
export TMPDIR=/tmp
T=${T:-r04ai}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "per_string or dropin or capi or host_batch" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
cp build/ab/libhhuff_inl2.so /tmp/pa/libhhuff.so && cp build/ab/libhhuff_base9.so /tmp/pb/libhhuff.so || exit 9
for v in a b a b; do
  LD_LIBRARY_PATH=/tmp/p$v timeout -k 10 200 ./tools/per_string_bench 1 4 16 >> gpurun_out/${T}_ps_$v.jsonl 2>&1 || exit 8
done
