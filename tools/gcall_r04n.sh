#!/bin/bash
# round 4: sorted-encoder chunk sizes (A/B)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04n}
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_enco c4,c2 base4 e192 e320 || exit 7
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_seg c3,c5 base5 seg64 || exit 7
