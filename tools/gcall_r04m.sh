#!/bin/bash
# round 4: phase profile of the sorted encoder (c4, HHUFF_PROFILE build)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04m}
timeout -k 10 300 python3 -u tools/ab.py run cfg=c4 fl eprof > gpurun_out/${T}_eprof_c4.log 2>&1 || exit 7
