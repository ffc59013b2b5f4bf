#!/bin/bash
# Round-2 GPU session D: lockstep Brent for two-agent waves; the spilling
# two-wave DC build with lockstep; default and config benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -3 $O/pytest_gpu.log; ok $rc
DGEN_LIB=dgen_amd/lib/ablate/libdgen_dc2w_ls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_demand.py -q --timeout 120 --timeout-method thread > $O/pytest_dc2w_ls.log 2>&1; rc=$?
echo "dc2w_ls rc=$rc"; tail -3 $O/pytest_dc2w_ls.log; ok $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_default.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])"; ok $rc
for c in ca_res_storage com_dc_batt; do
  timeout -k 10 300 python bench.py --no-cpu --config $c --agents 200000 --steps 3 --warmup 1 > $O/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])"; ok $rc
done
DGEN_LIB=dgen_amd/lib/ablate/libdgen_dc2w_ls.so timeout -k 10 300 python bench.py --no-cpu --config com_dc_batt --agents 200000 --steps 3 --warmup 1 > $O/bench_com_dc_batt_2w.log 2>&1; rc=$?
echo "bench dc2w_ls rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_com_dc_batt_2w.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])"; ok $rc
DGEN_LIB=dgen_amd/lib/ablate/libdgen_ls_only.so timeout -k 10 300 python bench.py --no-cpu --config ca_res_storage --agents 200000 --steps 3 --warmup 1 > $O/bench_ca_ls_only.log 2>&1; rc=$?
echo "bench ca ls_only rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_ca_ls_only.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])"; ok $rc
