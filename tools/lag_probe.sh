#!/bin/bash
# Repeats the lagged-solve parity test under three device-buffer modes (poisoned allocations, no buffer cache,
# buffer cache) and keeps each run's log under gpurun_out/ (diagnostic for run-to-run variation vs stale buffers).
T="tests/test_gpu_parity.py::test_repeated_solves_lagged_coarse_inverse"
for mode in poison nocache cache; do
  for r in 1 2 3; do
    case $mode in
      poison) env="INSFM_DEVICE_POISON=1";;
      nocache) env="INSFM_DEVICE_CACHE_MB=0";;
      cache) env="INSFM_NOTHING=0";;
    esac
    env $env timeout -k 10 120 python -u -m pytest $T -q -s --timeout 100 --timeout-method thread \
      > gpurun_out/lag_${mode}_$r.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
exit 0
