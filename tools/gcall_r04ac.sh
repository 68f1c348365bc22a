#!/bin/bash
# A/B: proportional-lane encode / flatten with clamped unconditional offset loads (plc) and the next span
# committed before the tile's stores (pl1), against the head before them (base8)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04ac}
timeout -k 10 900 bash tools/gcall_ab.sh ${T}_pl c5,c3 base8 plc pl1 || exit 7
