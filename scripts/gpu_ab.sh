#!/bin/bash
# A/B of bench variants on one box: GPU tests first, then one bench line per
# variant (BENCH_VARIANTS: ';'-separated bench.py argument strings).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?
  echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VARS <<< "${BENCH_VARIANTS:---no-cpu}"
k=0
for v in "${VARS[@]}"; do
  k=$((k+1))
  lib=""; args="$v"
  case "$v" in lib=*) lib="${v%% *}"; lib="${lib#lib=}"; args="${v#* }";; esac
  if [ -n "$lib" ]; then export DGEN_LIB=$PWD/dgen_amd/lib/ablate/libdgen_$lib.so; else unset DGEN_LIB; fi
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_${TAG}_$k.log 2>&1; rc=$?
  echo "== [$v] rc=$rc"
  python3 - gpurun_out/bench_${TAG}_$k.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(f"   value={d['value']:.4g} ms/step={d['ms_per_step']:.2f} kern={ {k: round(v, 2) for k, v in r['kernel_ms'].items()} } frac={r['frac']:.3f}")
PY
  [ $rc -eq 0 ] || exit $rc
done
