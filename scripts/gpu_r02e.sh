#!/bin/bash
# Round-2 GPU session E: net-billing split without lockstep; two-wave DC
# builds with / without the envelope fast path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']),{k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -2 $O/pytest_gpu.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; bj $O/bench_default.log; ok $rc
for c in ca_res_storage com_dc_batt national_mixed; do
  timeout -k 10 300 python bench.py --no-cpu --config $c --agents 200000 --steps 3 --warmup 1 > $O/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; bj $O/bench_$c.log; ok $rc
done
for v in w2_noenv w2; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_demand.py -q --timeout 120 --timeout-method thread > $O/pytest_dc_$v.log 2>&1; rc=$?
  echo "dc $v rc=$rc"; tail -2 $O/pytest_dc_$v.log; ok $rc
done
