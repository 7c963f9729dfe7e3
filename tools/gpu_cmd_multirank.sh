# N-rank rehearsal of bench.py on a one-GPU box: 2 ranks on device 0 over gloo
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_BENCH_DEVICE=0 IPT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 4 > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err
echo rc=$?
