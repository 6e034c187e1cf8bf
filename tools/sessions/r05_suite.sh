#!/bin/bash
# round 5: failure-path tests first, then the whole GPU suite (stop on a fault / timeout)
mkdir -p gpurun_out/r05a
timeout -k 10 300 python -u -m pytest tests/test_gpu_failure.py -v --timeout 240 --timeout-method thread \
  > gpurun_out/r05a/pytest_fail.log 2>&1
rc=$?
echo "failure tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_failure.py > gpurun_out/r05a/pytest_gpu.log 2>&1
rc2=$?
echo "suite rc=$rc2"
tail -30 gpurun_out/r05a/pytest_gpu.log
exit $(( rc | rc2 ))
