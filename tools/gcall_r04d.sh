#!/bin/bash
# round 4: GPU suite, smoke, bench, A/B (stream decode shapes, PL encoder / flatten, monotone encode), the HTTP/3
# rules inlined (A/B build), c5 profile
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04d}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_gpu_tests.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 5
AB_FLAT=1 timeout -k 10 900 bash tools/gcall_ab.sh ${T}_mix c3,c5 base ms t12 t16b cur mono || exit 7
timeout -k 10 600 bash tools/gcall_ab.sh ${T}_c4 c4 base cur mono || exit 7
HHUFF_AB_LIB=$PWD/build/ab/libhhuff_h3inl.so timeout -k 10 600 python3 -u -m pytest tests/test_qpack.py -m gpu -q -k "requests" --timeout 300 --timeout-method thread > gpurun_out/${T}_h3inline_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_h3inline_tests.log; [ $rc -le 1 ] || exit 10
CMD="python3 tools/bench_configs.py c5" timeout -k 10 600 bash tools/profile.sh ${T}_c5 || exit 6
