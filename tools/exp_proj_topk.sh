#!/bin/bash
# per-call SearchByProjection / Fuse rows for liborbamd variants of the scan's top-K (ORBX_PROJ_TOPK), parity first
for v in "$@"; do
  ORBAMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_projection.py > gpurun_out/topk_test_$v.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 gpurun_out/topk_test_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for r in 1 2; do
  for v in "$@"; do
    ORBAMD_LIB_VARIANT=$v BENCH_ROWS_ONLY=projection,fuse timeout -k 10 120 python tools/bench_rows.py 2>/dev/null | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('r$r', '$v', d['row'], d['gpu_host_api_ms_per_call'], d.get('gpu_cached_kf_ms_per_call', ''), d['cpu_oracle_ms_per_call'])" || exit 1
  done
done
