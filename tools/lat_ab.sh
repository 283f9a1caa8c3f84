#!/bin/bash
# per-call latency A/B of liborbamd variants (tests/cpp/build/bench_latency through LD_LIBRARY_PATH)
mkdir -p gpurun_out
for v in "$@"; do
  ORBAMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_cpp_dropin.py > gpurun_out/lat_test_$v.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 gpurun_out/lat_test_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi  # a variant with broken parity is not timed
done
for r in 1 2; do
  for v in "$@"; do
    d=/tmp/libv_$v; mkdir -p $d; cp cooperative-orb-slam_amd/lib/liborbamd_$v.so $d/liborbamd.so
    LD_LIBRARY_PATH=$d timeout -k 10 200 tests/cpp/build/bench_latency 2000 > gpurun_out/lat_${v}_${r}.jsonl 2>&1 || exit $?
    echo "r$r $v: $(python3 -c "
import json
for l in open('gpurun_out/lat_${v}_${r}.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d['row'], d['gpu_host_api_us_per_call'], end='; ')
")"
  done
done
