#!/bin/bash
# Drop-in host path: boundary + download tests, then the drop-in bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_download.py tests/test_gpu_boundary.py tests/test_gpu_properties.py -m gpu -q -rf --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log; ok $rc
timeout -k 10 400 python bench_dropin.py --agents 100000 > $O/dropin.log 2>&1; rc=$?
echo "dropin rc=$rc"; tail -c 900 $O/dropin.log; ok $rc
