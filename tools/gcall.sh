mkdir -p gpurun_out
for r in 1 2 3; do
for nc in 1 2; do
HHUFF_SVC_NC=$nc timeout -k 10 60 ./tools/per_string_bench > gpurun_out/ps_nc${nc}_$r.json 2>&1 || exit 4
done
done
timeout -k 10 300 python3 -u -m pytest tests/test_capi.py tests/test_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || exit 3
HHUFF_SVC_NC=2 timeout -k 10 300 python3 -u -m pytest tests/test_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ps_tests_nc2.log 2>&1 || exit 5
