#!/bin/bash
# Round-2 GPU session F: full GPU tests (market kernels, table-driven year
# loop, C1, PV-only variant), benches of every config with the new roofline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or d.get('sizing_kernel_ms_per_call') or {}).items() if isinstance(v,float)})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; grep -E "passed|failed|flips|FAILED" $O/pytest_gpu.log | tail -8; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; bj $O/bench_default.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu --config de_res --agents 50000 --no-batt > $O/bench_de_res_nobatt.log 2>&1; rc=$?
echo "bench de_res nobatt rc=$rc"; bj $O/bench_de_res_nobatt.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu --config de_res --agents 50000 > $O/bench_de_res.log 2>&1; rc=$?
echo "bench de_res rc=$rc"; bj $O/bench_de_res.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu --no-batt > $O/bench_default_nobatt.log 2>&1; rc=$?
echo "bench C3 nobatt rc=$rc"; bj $O/bench_default_nobatt.log; ok $rc
timeout -k 10 400 python bench_loop.py --config de_res --agents 50000 --first-year 2022 --step 2 --years 5 > $O/loop_de_res.log 2>&1; rc=$?
echo "loop de_res rc=$rc"; tail -c 400 $O/loop_de_res.log; ok $rc
timeout -k 10 600 python bench_loop.py --agents 200000 --years 25 > $O/loop_national_200k.log 2>&1; rc=$?
echo "loop national rc=$rc"; tail -c 600 $O/loop_national_200k.log; ok $rc
