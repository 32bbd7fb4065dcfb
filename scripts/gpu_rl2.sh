set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r03f}
mkdir -p $OUT
for t in direct dma copy; do timeout -k 10 60 scripts/_build/rl_stream 64 4 16 $t > $OUT/rl_$t.json 2>&1; done
for m in 4 8; do timeout -k 10 60 scripts/_build/rl_stream 64 4 16 direct $m > $OUT/rl_direct_m$m.json 2>&1; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_record_layer_async.py tests/test_gpu_record_layer.py tests/test_gpu_traffic_key.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
