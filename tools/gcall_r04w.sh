#!/bin/bash
# A/B: the sorted encoder's second word per step stored instead of OR-ed (w4a: everywhere, wrong at string ends;
# w4b: where the word is the lane's own)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04w}
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_w4 c4,c2 base6 x_w4a w4b || exit 7
