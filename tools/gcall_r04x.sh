#!/bin/bash
# per-string A/B: poll load order (base7: header then chunks; pck: chunks first; pgap: a pause between them)
mkdir -p gpurun_out /tmp/pa /tmp/pb /tmp/pc
export TMPDIR=/tmp
T=${T:-r04x}
cp build/ab/libhhuff_base7.so /tmp/pa/libhhuff.so && cp build/ab/libhhuff_pck.so /tmp/pb/libhhuff.so && cp build/ab/libhhuff_pgap.so /tmp/pc/libhhuff.so || exit 9
for r in 1 2; do
  for v in a b c; do
    LD_LIBRARY_PATH=/tmp/p$v timeout -k 10 200 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_ps_${v}_$r.jsonl 2>&1 || exit 8
  done
done
