#!/bin/bash
# One GPU session: parity tests -> smoke -> bench.  Stops at the first crash-type
# exit (fault / abort / segfault / timeout); assertion failures do not stop it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
AGENTS=${AGENTS:-200000}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc
timeout -k 10 400 python bench.py --agents $AGENTS --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_small.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_small.log; ok $rc
if [ -n "$FULL" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?
  echo "bench full rc=$rc"; tail -3 gpurun_out/bench_full.log; ok $rc
fi
