#!/bin/bash
# round 4: counters available on gfx950 (for a TA / TD / TCP pass on the stream decode); c4 decode phases
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04k}
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/${T}_counters.txt 2>&1
timeout -k 10 300 python3 -u tools/ab.py run cfg=c4 lay dprof > gpurun_out/${T}_dprof_c4.log 2>&1 || exit 7
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_shape c3,c5 fl w6 w4n32 w6n24 || exit 7
