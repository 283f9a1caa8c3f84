#!/bin/bash
# A/B of the Fuse per-call path (tools/build_variant.sh pd0 -DORBX_PROJ_DIRECT=0, pd1): projection parity tests per
# variant, then the Fuse row of tools/bench_rows.py three times each.
for v in pd0 pd1; do
  ORBAMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_projection.py > gpurun_out/pd_test_$v.log 2>&1; rc=$?
  echo "$v parity rc=$rc $(tail -n 1 gpurun_out/pd_test_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi  # a variant with broken parity is not timed
done
for r in 1 2 3; do for v in pd0 pd1; do
  echo "r$r $v $(ORBAMD_LIB_VARIANT=$v BENCH_ROWS_ONLY=fuse timeout -k 10 120 python tools/bench_rows.py | tail -n 1)"
done; done
