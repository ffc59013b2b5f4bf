#!/bin/bash
# PMC A/B of kernel variants on one workload: instruction mix and waits per
# wave for each variant (dgen_amd/lib/ablate/libdgen_<v>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/pmcab
mkdir -p $O
G1="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
G2="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
cd /tmp
for v in ${VARIANTS:-base}; do
  for g in 1 2; do
    eval grp=\$G$g
    DGEN_LIB=$R/dgen_amd/lib/ablate/libdgen_$v.so timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/${v}_$g -o run -- \
      python3 $R/bench.py --config ${CFG:-ca_res_storage} --agents ${AGENTS:-200000} --steps 1 --warmup 1 --no-cpu > $O/${v}_$g.log 2>&1; rc=$?
    echo "$v g$g rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
python3 - <<'PY'
import csv, glob, os, collections
O=os.environ.get('GRAFT_REPO_ROOT','/root/repo')+'/gpurun_out/pmcab'
res=collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O+'/*/**/*counter_collection.csv', recursive=True):
    v=os.path.relpath(f,O).split('/')[0].rsplit('_',1)[0]
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name']
        for kn in ('k_size_w','k_batt_finance_w'):
            if kn in k:
                res[(v,kn)][r['Counter_Name']]+=float(r['Counter_Value'])
for (v,kn),c in sorted(res.items()):
    w=c.get('SQ_WAVES',1) or 1
    print(v,kn,{k: round(x/w) for k,x in sorted(c.items()) if k!='SQ_WAVES'}, 'waves',w)
PY
