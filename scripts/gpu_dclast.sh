#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dcdiag
for v in ${VARIANTS:-base dc_dbg}; do
DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python -u scripts/dbg_dc_last.py > gpurun_out/dcdiag/last_$v.log 2>&1; rc=$?
echo "== $v rc=$rc"; grep -v amdgpu.ids gpurun_out/dcdiag/last_$v.log | head -40
case $rc in 0) ;; *) exit $rc;; esac
done
