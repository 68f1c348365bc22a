mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_responses.py tests/test_hpack_blocks.py tests/test_qpack.py tests/test_capi.py tests/test_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/resp_tests.log 2>&1 || exit 3
timeout -k 10 120 ./tools/per_string_bench > gpurun_out/ps_bench_c.json 2>&1 || exit 4
timeout -k 10 120 python3 tools/per_string_lat.py > gpurun_out/ps_bench_py.json 2>&1 || exit 5
