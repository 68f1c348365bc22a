# per-string decode walk A/B (HHUFF_SVC_NC=1: one step per link; default: jump table), then the tests that
# drive the per-string service
mkdir -p gpurun_out
out=gpurun_out/r03_per_string_jump_ab.jsonl
: > $out
for r in 1 2 3; do
  for nc in 1 3; do
    echo "{\"run\": \"nc${nc}_$r\", \"result\": $(HHUFF_SVC_NC=$nc timeout -k 10 120 ./tools/per_string_bench)}" >> $out || exit 2
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_capi.py tests/test_dropin.py tests/test_gpu_parity.py -m gpu -q -k "per_string or capi or dropin or symbols" --timeout 300 --timeout-method thread > gpurun_out/r03_per_string_jump_tests.log 2>&1 || exit 3
