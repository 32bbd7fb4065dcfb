# The record layer's coalescing of a connection's queued windows (record_layer.c, include/ptls_mi355x.h section 5):
# scripts/_build/rl_stream, one window per submit, with and without coalescing, at depths 4 to 32, against the
# hand-batched 8 windows per launch.   gpurun -- 'bash scripts/rl_coalesce.sh' -> gpurun_out/${TAG:-rlco}/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-rlco}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "16 4 1" "0 4 1" "16 8 1" "16 16 1" "16 32 1" "0 4 8 one"; do
    set -- $cfg
    co=$1; shift
    RL_COALESCE=$co timeout -k 10 60 scripts/_build/rl_stream 64 $1 16 dma_in $2 $3 > $OUT/co${co}_d$1_m$2$3_r$rep.json
  done
done
