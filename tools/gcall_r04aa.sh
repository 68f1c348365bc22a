#!/bin/bash
# A/B: sorted encoder with the next chunk's offsets and span waited for before the chunk's stores (early)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04aa}
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_early c4,c2 base8 early base8 early || exit 7
