#!/bin/bash
# round 4: GPU suite at the head (repacked LUT, flatten span staging by LDS-DMA); A/B of flatten staging
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04i}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
AB_FLAT=1 timeout -k 10 600 bash tools/gcall_ab.sh ${T}_fl c5,c3 lay fl || exit 7
bash tools/gcall_r04j.sh || exit $?
bash tools/gcall_r04k.sh || exit $?
