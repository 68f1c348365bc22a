mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_all.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/r03_bench_head.json 2> gpurun_out/r03_bench_head.err || exit 5
