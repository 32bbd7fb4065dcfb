# Where a one-window-per-launch record-layer stream spends its time (rocprofv3 kernel, memory-copy and HIP runtime
# traces of scripts/_build/rl_stream; no counters).   gpurun -- 'bash scripts/rl_trace.sh' -> gpurun_out/${TAG:-rltrace}/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rltrace}
mkdir -p $OUT
timeout -k 10 60 scripts/_build/rl_stream 64 4 16 dma_in 1 > $OUT/plain_1.json 2>&1
timeout -k 10 60 scripts/_build/rl_stream 64 4 16 dma_in 8 one > $OUT/plain_8one.json 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --stats -d $OUT/trace1 -o run --output-format csv -- scripts/_build/rl_stream 64 4 16 dma_in 1 > $OUT/trace1.log 2>&1
