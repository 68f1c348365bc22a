#!/bin/bash
# A/B: flatten with the next tile's span DMA issued before the tile's stores (fl1) against fl0 and pl1 (head)
mkdir -p gpurun_out
export TMPDIR=/tmp
export AB_FLAT=1
T=${T:-r04ae}
timeout -k 10 900 bash tools/gcall_ab.sh ${T}_flat c5 fl0 fl2 fl0 fl2 || exit 7
