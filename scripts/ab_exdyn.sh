set -o pipefail
O=gpurun_out/r06/s21; mkdir -p $O
TAG=r06/s21 TESTS="tests/test_gpu_exact.py" bash scripts/gpu.sh tests || exit 1
k=0
for cfg in national_mixed com_8m; do
  for v in 1 0 1 0; do
    k=$((k+1))
    DGEN_EX_DYN=$v timeout -k 10 300 python bench.py --config $cfg --agents 200000 --steps 5 --warmup 1 --no-cpu > $O/ab_${cfg}_${v}_$k.log 2>&1; rc=$?
    echo "$cfg dyn=$v rc=$rc $(grep '^{' $O/ab_${cfg}_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d["ms_per_step"], d["roofline"].get("kernel_ms"))')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
