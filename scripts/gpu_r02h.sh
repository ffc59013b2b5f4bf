#!/bin/bash
# Round-2 GPU session H: full GPU tests after the spill-guard build and the
# reference-order demand generation (flips), the drop-in bench with the
# device net sum, the default bench and the C4 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or d.get('sizing_kernel_ms_per_call') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED|flips" $O/pytest_gpu.log | tail -12; ok $rc
timeout -k 10 400 python bench_dropin.py --agents 100000 > $O/dropin.log 2>&1; rc=$?
echo "dropin rc=$rc"; tail -c 900 $O/dropin.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; bj $O/bench_default.log; ok $rc
timeout -k 10 400 python bench.py --no-cpu --config com_dc_batt --agents 200000 --steps 3 --warmup 1 > $O/bench_c4dc.log 2>&1; rc=$?
echo "bench C4 dc rc=$rc"; bj $O/bench_c4dc.log; ok $rc
