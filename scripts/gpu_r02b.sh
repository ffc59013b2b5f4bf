#!/bin/bash
# Round-2 GPU session B: good vs spilling two-wave demand-charge build, outputs
# and envelope buffers dumped for a bit-level comparison.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
for v in good bad; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_dbg_$v.so timeout -k 10 200 python -u scripts/dbg_dc_dump.py $O/dc_$v.npz > $O/dump_$v.log 2>&1; rc=$?
  echo "dump $v rc=$rc"; tail -2 $O/dump_$v.log; ok $rc
done
python scripts/dbg_dc_compare.py $O/dc_good.npz $O/dc_bad.npz | tee $O/compare.log
