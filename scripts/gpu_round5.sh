# Round-5 closing measurement: scripts/gpu_round_bench.sh (bench lines, rocprofv3 kernel-trace summaries, PMC traffic
# and SQ counters), then the N > 1 path rehearsed on one GPU (two ranks on cuda:0 over gloo, per-rank figures and
# per-rank PCIe-inclusive rates).   gpurun -- 'TAG=r05i bash scripts/gpu_round5.sh' -> gpurun_out/$TAG/
set -e
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round_bench.sh
OUT=gpurun_out/${TAG:-round}
RAPIDO_BENCH_SAME_DEVICE=1 RAPIDO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 \
    > $OUT/bench_2rank_same_device.json 2> $OUT/bench_2rank.err
