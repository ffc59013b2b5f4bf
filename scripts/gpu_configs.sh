cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_demand.py tests/test_gpu_synthetic.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in com_dc_batt ca_res_storage; do
timeout -k 10 400 python bench.py --config $cfg --agents 200000 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_$cfg.log 2>&1 || exit $?
echo $cfg; tail -1 gpurun_out/bench_$cfg.log | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}'
done
