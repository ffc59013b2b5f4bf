#!/bin/bash
# Round-2 GPU session G: full GPU tests (metering options 0-4, vectorized
# drop-in frame path), the drop-in host-path bench, the default bench and the
# 1M national loop with the state-major order (k_state_hourly coalesced).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or d.get('sizing_kernel_ms_per_call') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|FAILED" $O/pytest_gpu.log | tail -8; ok $rc
timeout -k 10 400 python bench_dropin.py --agents 100000 > $O/dropin.log 2>&1; rc=$?
echo "dropin rc=$rc"; tail -c 900 $O/dropin.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; bj $O/bench_default.log; ok $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loop -o run -- python3 bench_loop.py --agents 1000000 --years 3 > $O/loop_1m.log 2>&1; rc=$?
echo "loop 1M rc=$rc"; tail -c 600 $O/loop_1m.log; ok $rc
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/r02g/trace_loop/run_kernel_stats.csv')))[:8]:
    print(f"{r['Name'][:50]:50s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
PY
