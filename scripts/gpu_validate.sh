# Full GPU check of the tree: every -m gpu test, smoke(), then the round-end measurement
# (scripts/gpu_round_bench.sh: bench lines, rocprofv3 kernel-trace summary, PMC passes).
#   gpurun --timeout 1200 -- 'TAG=r01c bash scripts/gpu_validate.sh'
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-validate}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
if [ -z "$SKIP_BENCH" ]; then
  bash scripts/gpu_round_bench.sh
  cat $OUT/bench_1400.json
fi
