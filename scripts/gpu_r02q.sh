#!/bin/bash
# N > 1 rehearsal on one GPU (two ranks, gloo) + the default bench as the driver runs it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
[ -n "$SKIP_N2" ] || DGEN_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --agents 200000 --steps 5 --warmup 1 > $O/bench_n2_gloo.log 2>&1; rc=$?
echo "n2 rehearsal rc=$rc"; grep '^{' $O/bench_n2_gloo.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
t0=$(date +%s.%N)
timeout -k 10 600 python bench.py > $O/bench_default.log 2> $O/bench_default.err; rc=$?
t1=$(date +%s.%N)
echo "default bench rc=$rc wall=$(python3 -c "print(round($t1-$t0,1))") s"; grep '^{' $O/bench_default.log | cut -c1-400
exit $rc
