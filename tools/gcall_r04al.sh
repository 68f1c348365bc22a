#!/bin/bash
# split decode: a whole block per very long string (blk: 16 waves, block list) against the one-wave split
# (r4head: the committed round-4 build; w4old: this source with 4-wave blocks and no block list)
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r04al}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "split or launch_path or long or per_string or decode" > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 3
timeout -k 10 400 python3 -u tools/split_bench.py blk r4head > gpurun_out/${T}_split_ab.log 2>&1 || exit 4
bash tools/gcall_ab.sh ${T} c5 blk r4head || exit 5
