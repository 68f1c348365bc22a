#!/bin/bash
# per-string: short strings inline in the header line (inl, inld stamps) against base7; per-string GPU tests
mkdir -p gpurun_out /tmp/pa /tmp/pb /tmp/pc
export TMPDIR=/tmp
T=${T:-r04z1}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "per_string or dropin or capi or host_batch" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
cp build/ab/libhhuff_inl.so /tmp/pa/libhhuff.so && cp build/ab/libhhuff_inld.so /tmp/pb/libhhuff.so && cp build/ab/libhhuff_base7.so /tmp/pc/libhhuff.so || exit 9
for v in b a c a c; do
  LD_LIBRARY_PATH=/tmp/p$v timeout -k 10 200 ./tools/per_string_bench 1 4 16 >> gpurun_out/${T}_ps_$v.jsonl 2>&1 || exit 8
done
