#!/bin/bash
# Round-2 GPU session I: full GPU tests after the compact net-billing records,
# then the C2 / national / C3 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or d.get('sizing_kernel_ms_per_call') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED|flips" $O/pytest_gpu.log | tail -12; ok $rc
for cfg in ca_res_storage:200000 national_mixed:200000 com_dc_batt:200000; do
  c=${cfg%%:*}; a=${cfg##*:}
  timeout -k 10 400 python bench.py --no-cpu --config $c --agents $a --steps 3 --warmup 1 > $O/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; bj $O/bench_$c.log; ok $rc
done
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench C3 rc=$rc"; bj $O/bench_default.log; ok $rc
timeout -k 10 600 python bench_loop.py --agents 1000000 --years 3 > $O/loop_1m.log 2>&1; rc=$?
echo "loop 1M rc=$rc"; bj $O/loop_1m.log; ok $rc
