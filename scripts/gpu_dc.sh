#!/bin/bash
# Demand-charge extension mode on the GPU: its parity tests, then the
# reference-mode bench (regression check) and the com_dc_batt bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_demand.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_res.log 2>&1 || exit $?
cut -c1-300 gpurun_out/bench_res.log | tail -1
timeout -k 10 400 python bench.py --config com_dc_batt --agents 200000 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_dc.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dc.log | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}'
if [ -n "$COM" ]; then
  timeout -k 10 400 python bench.py --config com_8m --agents 200000 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_com.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_com.log | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}'
fi
