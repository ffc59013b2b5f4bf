#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),r.get('valu_busy_frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -12; ok $rc
timeout -k 10 400 python bench_dropin.py --agents 100000 > $O/dropin.log 2>&1; rc=$?
echo "dropin rc=$rc"; tail -c 700 $O/dropin.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench C3 rc=$rc"; bj $O/bench_default.log; ok $rc
