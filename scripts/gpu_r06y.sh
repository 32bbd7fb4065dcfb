# Round 6: the multi-key prep kernels per batch layout (kernel trace of scripts/mk_layout_probe.py), then the tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/mk_layout_probe.py --rounds 4 > $OUT/probe.txt 2>&1 || { tail -5 $OUT/probe.txt; exit 1; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multikey.py tests/test_gpu_read_bounds.py tests/test_gpu_fuzz_campaign.py tests/test_gpu_record_layer.py tests/test_gpu_record_layer_async.py -k "multikey or multi_session or many_sessions or fuzz_campaign or sessions" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
