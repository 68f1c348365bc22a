mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s2_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s2_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/r03s2_bench.json 2> gpurun_out/r03s2_bench.err || exit 5
bash tools/profile.sh r03s2c4 --no-extra || exit 6
CMD="python3 tools/bench_configs.py c3" bash tools/profile.sh r03s2c3 || exit 7
