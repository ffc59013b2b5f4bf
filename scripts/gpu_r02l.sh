#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),r.get('valu_busy_frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED|Error|flips" $O/pytest_gpu.log | tail -12; ok $rc
timeout -k 10 400 python bench.py --no-cpu --config com_dc_batt --agents 200000 --steps 3 --warmup 1 > $O/bench_com_dc_batt.log 2>&1; rc=$?
echo "bench C4 rc=$rc"; bj $O/bench_com_dc_batt.log; ok $rc
