#!/bin/bash
# round 4: GPU suite with the repacked window LUT (sym2 in bits 16..23, L12 = 0 for long codes), explicit
# price calibration and the fixed-schedule stream flush; A/B of the head, the repacked LUT, and both + stream
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04h}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_lay c4,c2 head lay st || exit 7
AB_FLAT=1 timeout -k 10 600 bash tools/gcall_ab.sh ${T}_st c3,c5 head lay st || exit 7
