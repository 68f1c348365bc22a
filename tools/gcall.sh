#!/bin/bash
# The GPU-box recipe (run through gpurun from the repo root):  T=<tag> bash tools/gcall.sh STEP...
#   tests       the whole -m gpu suite (K="<pytest -k expr>" narrows it)
#   smoke       __graft_entry__.smoke()
#   bench       python3 bench.py (BENCH_ARGS="..." appends arguments)
#   trace       kernel trace + stats of the c4 bench (rocprofv3 --kernel-trace --stats)
#   prof_c4 / prof_c3 / prof_c5   tools/profile.sh: trace + PMC passes of one config
#   ab          tools/ab.py $AB_ARGS (interleaved A/B of two builds, see tools/ab.py)
#   per_string  tools/per_string_bench 1 4 16 (caller threads)
# Every GPU step has its own time limit and the steps are chained: the first failure ends the call.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-run}
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} \
        > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3 ;;
    smoke)
      timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 4 ;;
    bench)
      timeout -k 10 600 python3 -u bench.py $BENCH_ARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 5 ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}/trace -o run -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-host > gpurun_out/${T}_trace.log 2>&1 || exit 6 ;;
    prof_c4)
      timeout -k 10 900 bash tools/profile.sh ${T}_c4 --no-extra || exit 6 ;;
    prof_c3|prof_c5)
      CMD="python3 tools/bench_configs.py ${step#prof_}" timeout -k 10 600 bash tools/profile.sh ${T}_${step#prof_} || exit 6 ;;
    ab)
      timeout -k 10 900 python3 -u tools/ab.py $AB_ARGS > gpurun_out/${T}_ab.log 2>&1 || exit 7 ;;
    per_string)
      timeout -k 10 300 ./tools/per_string_bench 1 4 16 > gpurun_out/${T}_per_string.jsonl 2>&1 || exit 8 ;;
    *) echo "gcall.sh: unknown step $step" >&2; exit 2 ;;
  esac
done
