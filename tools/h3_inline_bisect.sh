# HTTP/3 rules inlined into qpack_sections_kernel (-DHHUFF_H3_INLINE): which compiler setting makes the lost
# err_desc word come back.  One pytest run per A/B build (tools/ab.py build NAME ...); writes
# gpurun_out/${T}_h3_<build>.log and one summary line per build.
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in "$@"; do
  HHUFF_AB_LIB=$PWD/build/ab/libhhuff_$b.so timeout -k 10 240 python3 -u -m pytest tests/test_qpack.py -m gpu -q \
    -k "requests_match" --timeout 120 --timeout-method thread > gpurun_out/${T}_h3_$b.log 2>&1
  rc=$?
  echo "{\"build\": \"$b\", \"rc\": $rc, \"summary\": \"$(tail -n1 gpurun_out/${T}_h3_$b.log)\"}" | tee -a gpurun_out/${T}_h3_bisect.jsonl
  [ $rc -gt 1 ] && exit $rc
done
exit 0
