#!/bin/bash
# Round-2 GPU session A: parity tests on the vmcnt-fixed build, the DC demand
# test on the spilling two-wave two-agent variant, default bench + rocprof.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -4 $O/pytest_gpu.log; ok $rc
DGEN_LIB=dgen_amd/lib/ablate/libdgen_dc2w.so timeout -k 10 300 python -u -m pytest tests/test_gpu_demand.py -v --timeout 120 --timeout-method thread > $O/pytest_dc2w.log 2>&1; rc=$?
echo "dc2w rc=$rc"; tail -6 $O/pytest_dc2w.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench_default.log; ok $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 5 > $GRAFT_REPO_ROOT/$O/bench_rocprof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; ok $rc
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
