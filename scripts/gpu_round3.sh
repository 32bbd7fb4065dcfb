# round-3 full GPU pass: every GPU test, the smoke, then scripts/gpu_round_bench.sh (bench lines, rocprofv3 traces, PMC)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03i}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
TAG=${TAG:-r03i} bash scripts/gpu_round_bench.sh
