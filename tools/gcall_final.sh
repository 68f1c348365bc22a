mkdir -p gpurun_out
true
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03s6_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s6_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/r03s6_bench.json 2> gpurun_out/r03s6_bench.err || exit 5
