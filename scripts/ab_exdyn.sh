# A/B of the certified re-run's scheduling (DGEN_EX_DYN, DGEN_EX_STREAM) on
# the populations that list agents; tests first (exact re-run, pipeline depth)
set -o pipefail
O=gpurun_out/${TAG:-r06/ab}; mkdir -p $O
TAG=${TAG:-r06/ab} TESTS="${AB_TESTS:-tests/test_gpu_exact.py}" bash scripts/gpu.sh tests || exit 1
k=0
for spec in ${AB_RUNS:-national_mixed:1:1 national_mixed:1:0}; do
  IFS=: read -r cfg ch st <<< "$spec"
  k=$((k+1))
  DGEN_EX_STREAM=$st timeout -k 10 300 python bench.py --config $cfg --agents ${AB_AGENTS:-200000} --chunks $ch \
    --steps 5 --warmup 1 --no-cpu > $O/ab_${cfg}_c${ch}_s${st}_$k.log 2>&1; rc=$?
  echo "$cfg chunks=$ch exstream=$st rc=$rc $(grep '^{' $O/ab_${cfg}_c${ch}_s${st}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],2), {a: round(b,2) for a,b in d["roofline"].get("kernel_ms").items()})')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
