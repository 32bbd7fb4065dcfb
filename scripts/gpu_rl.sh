set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_record_layer_async.py tests/test_gpu_record_layer.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03b/tests.log 2>&1
timeout -k 10 300 python -u -c "
import bench, rapido_amd as ra, torch, json
torch.cuda.init()
print(json.dumps(bench.record_layer_stream(ra, 16)))
" > gpurun_out/r03b/stream.json 2> gpurun_out/r03b/stream.err
