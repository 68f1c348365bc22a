#!/bin/bash
# A/B: tile / chunk edge byte ranges stored in the kernels (ei1) against records + edge_fix_kernel (ei0)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04ag}
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_edge c4,c2,c3 ei0 ei1 ei0 ei1 || exit 7
AB_FLAT=1 timeout -k 10 300 bash tools/gcall_ab.sh ${T}_edge c5 ei0 ei1 || exit 7
