#!/bin/bash
# per-string diagnostics: the device writes a request's input chunk lines before `done` (pclr, pclrd stamps)
mkdir -p gpurun_out /tmp/pd /tmp/pe /tmp/pg
export TMPDIR=/tmp
T=${T:-r04y2}
cp build/ab/libhhuff_pclrd.so /tmp/pd/libhhuff.so && cp build/ab/libhhuff_pclr.so /tmp/pe/libhhuff.so && cp build/ab/libhhuff_base7.so /tmp/pg/libhhuff.so || exit 9
for v in d e g e g; do
  LD_LIBRARY_PATH=/tmp/p$v timeout -k 10 200 ./tools/per_string_bench 1 4 16 >> gpurun_out/${T}_ps_$v.jsonl 2>&1 || exit 8
done
