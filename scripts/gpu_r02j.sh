#!/bin/bash
# Round-2 GPU session J: the default bench as the driver runs it (CPU
# baseline included), C1 (DE residential PV-only, 2022-2030 in 2-year steps),
# and the per-config lines with the PMC VALU-busy field.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
bj() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print(round(d['value']),r.get('kernel'),r.get('frac'),r.get('valu_busy_frac'),{k:round(v,2) for k,v in (r.get('kernel_ms') or d.get('sizing_kernel_ms_per_call') or {}).items() if isinstance(v,float)}, (d.get('cpu_baseline') or {}).get('value'))"; }
timeout -k 10 400 python bench.py > $O/bench_default_full.log 2>&1; rc=$?
echo "bench default rc=$rc"; bj $O/bench_default_full.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu --config de_res --agents 50000 --no-batt > $O/bench_c1_de_res_nobatt.log 2>&1; rc=$?
echo "bench C1 no-batt rc=$rc"; bj $O/bench_c1_de_res_nobatt.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu --config de_res --agents 50000 > $O/bench_c1_de_res.log 2>&1; rc=$?
echo "bench C1 rc=$rc"; bj $O/bench_c1_de_res.log; ok $rc
timeout -k 10 400 python bench_loop.py --config de_res --agents 50000 --first-year 2022 --step 2 --years 5 --no-batt > $O/loop_c1_de_res.log 2>&1; rc=$?
echo "loop C1 rc=$rc"; bj $O/loop_c1_de_res.log; ok $rc
for cfg in ca_res_storage:200000 com_dc_batt:200000 national_mixed:200000; do
  c=${cfg%%:*}; a=${cfg##*:}
  timeout -k 10 400 python bench.py --no-cpu --config $c --agents $a --steps 3 --warmup 1 > $O/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; bj $O/bench_$c.log; ok $rc
done
