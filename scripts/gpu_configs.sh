#!/bin/bash
# GPU tests (TESTS, default: the whole GPU suite), then a bench line per
# configuration (CONFIGS) at 200k agents and the default C3 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-ca_res_storage com_dc_batt}; do
timeout -k 10 400 python bench.py --config $cfg --agents 200000 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_$cfg.log 2>&1 || exit $?
echo $cfg; tail -1 gpurun_out/bench_$cfg.log | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}'
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_res.log 2>&1 || exit $?
echo res_1m_nem_tou; tail -1 gpurun_out/bench_res.log | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}'
