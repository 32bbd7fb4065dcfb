# Round 6: the fused multi-key range pass (mi355x_mk_bounds_all) -- multi-key tests, guard pages, the fuzz gate, then
# the layout probe (one key / 64 sessions against the single-key kernels, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06x}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multikey.py tests/test_gpu_read_bounds.py tests/test_gpu_fuzz_campaign.py tests/test_gpu_record_layer.py -k "multikey or multi_session or many_sessions or fuzz_campaign" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/mk_layout_probe.py --rounds 8 > $OUT/probe.txt 2>&1 || { tail -5 $OUT/probe.txt; exit 1; }
cat $OUT/probe.txt
