mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab.py run cfg=c4 base srt11 srt12 > gpurun_out/ab_srt12_c4.log 2>&1 || exit 2
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03s5_gpu_tests.log 2>&1 || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s5_smoke.log 2>&1 || exit 4
timeout -k 10 600 python3 bench.py > gpurun_out/r03s5_bench.json 2> gpurun_out/r03s5_bench.err || exit 5
