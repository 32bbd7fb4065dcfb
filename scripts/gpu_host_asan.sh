# The record layer's host code under AddressSanitizer + UBSan on the GPU (diagnostic): scripts/_build/asan/rl_stream
# (built here by scripts/build_host_asan.sh; sanitizers on host code only) streams windows through every transport,
# both key sizes, one window per launch and coalesced, several connections per launch and one.  Any heap or stack
# error in the host C (staging, queue, coalescing, registration table, slot arrays) stops it with a report.
#   gpurun -- 'TAG=r05zq bash scripts/gpu_host_asan.sh'  -> gpurun_out/$TAG/asan_*.log
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-asan}
mkdir -p $OUT
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1
RL=scripts/_build/asan/rl_stream
i=0
for args in "64 4 16 dma_in 8" "64 4 32 dma_in 8 one" "64 4 16 direct 4" "64 4 16 dma 4" "64 4 16 zero_copy 2" \
            "64 4 16 copy 1" "64 16 16 dma_in 1" "64 32 32 direct 1" "48 4 32 zero_copy 8 one" "32 2 16 copy 16"; do
  i=$((i + 1))
  timeout -k 10 120 $RL $args > $OUT/asan_$i.json 2> $OUT/asan_$i.log
  echo "case $i ($args): $(head -c 160 $OUT/asan_$i.json)"
done
echo "all cases clean"
