# A/B of the in-tree library against a saved base build (AB_BASE, default abl/libdgen_base.so;
# copy the base .so there before rebuilding and delete abl/ after): the exact-path tests, then
# national / com_8m bench lines alternating the two
set -o pipefail
O=gpurun_out/r06/s25; mkdir -p $O
TAG=r06/s25 TESTS="tests/test_gpu_exact.py tests/test_gpu_synthetic.py::test_pipeline_depth_is_invisible" bash scripts/gpu.sh tests || exit 1
k=0
for v in hq base hq base; do
  for cfg in national_mixed com_8m; do
  k=$((k+1))
  if [ $v = base ]; then export DGEN_LIB=$PWD/${AB_BASE:-abl/libdgen_base.so}; else unset DGEN_LIB; fi
  timeout -k 10 300 python bench.py --config $cfg --agents 200000 --steps 5 --warmup 1 --no-cpu > $O/ab_${cfg}_${v}_$k.log 2>&1; rc=$?
  echo "$cfg $v rc=$rc $(grep '^{' $O/ab_${cfg}_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],2), {a: round(b,2) for a,b in d["roofline"].get("kernel_ms").items()})')"
  [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
