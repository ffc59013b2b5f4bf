#!/bin/bash
# One parameterised GPU-session driver (run through gpurun from the repo root).
#
#   scripts/gpu.sh STEP [STEP ...]        steps run in order, output under $O
#
# Steps
#   tests      pytest -m gpu (TESTS: paths / -k expression, default the suite)
#   smoke      __graft_entry__.smoke()
#   bench      one bench line per BENCH ("config:agents[:extra,args]" ..., the
#              extra bench.py arguments comma-separated; default the driver's
#              own no-flag run)
#   ab         one bench line per ';'-separated VARIANTS entry
#              ("[lib=<name>] <bench.py args>"; lib= picks ablate/libdgen_<name>.so,
#              built by scripts/make_ablations.py)
#   trace      rocprofv3 --kernel-trace --stats of each PROF workload
#   pmc        one PMC pass per counter group of each PROF workload, summarised
#              into $O/pmc_<workload>.json by scripts/pmc_summary.py
#   loop       bench_loop.py (LOOP_ARGS) and its kernel trace
#   rehearse   2-rank gloo rehearsal of the N > 1 bench.py and bench_loop.py flows
#   dropin     bench_dropin.py (DROPIN_ARGS)
#   diag       scripts/diag_pop.py per DIAG entry ("config:n[:replan_hours]")
#
# Every GPU step runs under its own timeout; a crash-type exit (fault, abort,
# segfault, time limit) ends the session, an assertion failure in the tests
# ends it too unless KEEP_GOING=1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=${O:-gpurun_out/${TAG:-run}}
mkdir -p "$O"
O=$(cd "$O" && pwd)
stop() {
  case "$1" in
    0) return 0;;
    1) [ -n "$KEEP_GOING" ] && return 0; echo "STOP: exit 1"; exit 1;;
    *) echo "STOP: exit $1"; exit "$1";;
  esac
}
line() { grep '^{' "$1" | tail -1 | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); r = d.get('roofline', {})
    km = {k: round(v, 2) for k, v in r.get('kernel_ms', {}).items() if isinstance(v, float)}
    print(f\"   value={d['value']:.4g} {d['unit']} ms/step={d['ms_per_step']:.2f} kern={km} \"
          f\"bound={r.get('bound')} frac={r.get('frac')}\")" 2>/dev/null || tail -2 "$1"; }

PROF=${PROF:-res_1m_nem_tou:1000000 ca_res_storage:200000 com_dc_batt:200000}
GROUPS_=("FETCH_SIZE" "WRITE_SIZE"
         "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
         "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY")

for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu ${PYTEST_X--x} -v -rP --timeout 300 \
      --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
    echo "pytest gpu rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3; stop $rc;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
    echo "smoke rc=$rc"; tail -2 $O/smoke.log; stop $rc;;
  bench)
    for b in ${BENCH:-default}; do
      if [ "$b" = default ]; then args=""; name=default
      else IFS=: read -r cfg ag extra <<< "$b"; extra=${extra//,/ }
           args="--config $cfg --agents $ag ${extra:---steps 5 --warmup 1 --no-cpu}"
           name=${cfg}_$ag${BENCH_SUFFIX:-}; [ -n "$extra" ] && name=${name}_$(echo "$extra" | tr -dc 'a-z0-9' | cut -c1-24); fi
      timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $args > $O/bench_$name.log 2> $O/bench_$name.err; rc=$?
      echo "bench $name rc=$rc"; line $O/bench_$name.log; stop $rc
    done;;
  ab)
    IFS=';' read -ra VARS <<< "${VARIANTS:---no-cpu}"
    k=0
    for v in "${VARS[@]}"; do
      k=$((k+1)); lib=""; args="$v"
      case "$v" in lib=*) lib="${v%% *}"; lib="${lib#lib=}"; args="${v#* }";; esac
      if [ -n "$lib" ]; then export DGEN_LIB=$R/ablate/libdgen_$lib.so; else unset DGEN_LIB; fi
      case "$lib" in phase*|dcb_*) export DGEN_PHASE_PROF=1;; *) unset DGEN_PHASE_PROF;; esac
      timeout -k 10 400 python bench.py $args > $O/ab_$k.log 2>&1; rc=$?
      echo "== [$v] rc=$rc"; line $O/ab_$k.log; stop $rc
    done
    unset DGEN_LIB DGEN_PHASE_PROF;;
  trace)
    for wa in $PROF; do
      W=${wa%%:*}; A=${wa##*:}
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- \
        python3 $R/bench.py --config $W --agents $A --steps 5 --warmup 1 --no-cpu > $O/trace_$W.log 2>&1); rc=$?
      echo "trace $W rc=$rc"; line $O/trace_$W.log; stop $rc
    done;;
  pmc)
    for wa in $PROF; do
      W=${wa%%:*}; A=${wa##*:}
      for grp in "${GROUPS_[@]}"; do
        name=$(echo $grp | cut -d' ' -f1)
        (cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${W}_$name -o run -- \
          python3 $R/bench.py --config $W --agents $A --steps 2 --warmup 1 --no-cpu > $O/pmc_${W}_$name.log 2>&1); rc=$?
        echo "pmc $W $name rc=$rc"; stop $rc
      done
      python3 $R/scripts/pmc_summary.py "$O/pmc_${W}_*" $A $O/pmc_$W.json > $O/pmc_$W.txt 2>&1
      head -4 $O/pmc_$W.txt
    done;;
  loop)
    timeout -k 10 ${LOOP_TIMEOUT:-900} python -u bench_loop.py ${LOOP_ARGS:-} > $O/bench_loop.log 2>&1; rc=$?
    echo "loop rc=$rc"; tail -2 $O/bench_loop.log | cut -c1-600; stop $rc
    if [ -n "$LOOP_TRACE" ]; then
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loop -o run -- \
        python3 $R/bench_loop.py ${LOOP_TRACE_ARGS:-${LOOP_ARGS:-}} > $O/trace_loop.log 2>&1); rc=$?
      echo "trace loop rc=$rc"; stop $rc
    fi;;
  rehearse)
    DGEN_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 ${REH_BENCH_ARGS:---agents 200000 --steps 5 --warmup 1} \
      > $O/bench_n2_gloo.log 2>&1; rc=$?
    echo "bench n2 gloo rc=$rc"; line $O/bench_n2_gloo.log; stop $rc
    DGEN_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29534 bench_loop.py ${REH_LOOP_ARGS:---agents 200000 --years 3} \
      > $O/bench_loop_n2_gloo.log 2>&1; rc=$?
    echo "bench_loop n2 gloo rc=$rc"; tail -2 $O/bench_loop_n2_gloo.log | cut -c1-600; stop $rc;;
  diag)
    for d in ${DIAG:-com_8m:160}; do
      IFS=: read -r cfg n rh <<< "$d"
      timeout -k 10 300 python -u scripts/diag_pop.py $cfg $n ${rh:-24} > $O/diag_${cfg}_${n}_${rh:-24}.log 2>&1; rc=$?
      echo "diag $d rc=$rc"; head -12 $O/diag_${cfg}_${n}_${rh:-24}.log; stop $rc
    done;;
  dropin)
    timeout -k 10 600 python -u bench_dropin.py ${DROPIN_ARGS:-} > $O/bench_dropin.log 2>&1; rc=$?
    echo "dropin rc=$rc"; tail -4 $O/bench_dropin.log | cut -c1-600; stop $rc;;
  *) echo "unknown step $step"; exit 2;;
  esac
done
