mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_hpenc.py tests/test_qpenc.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_req_gpu_tests.log 2>&1 || exit 3
