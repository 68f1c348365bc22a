#!/bin/bash
# round 4: GPU suite at the head (monotone encode default), stream2 decode correctness (parity suites against its
# A/B build), A/B of stream2 shapes on c3 / c5 / c4
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04e}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
HHUFF_AB_LIB=$PWD/build/ab/libhhuff_s2w12.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_packed.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_s2w12_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_s2w12_tests.log; [ $rc -le 1 ] || exit 4
AB_FLAT=1 timeout -k 10 900 bash tools/gcall_ab.sh ${T}_s2 c3,c5 base cur s2w8 s2w12 || exit 7
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_c4 c4 base cur || exit 7
