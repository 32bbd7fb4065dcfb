# round-3 checks: traffic-key harness, golden fixtures on every family, the record-layer stream trace
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r03e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_traffic_key.py tests/test_gpu_golden.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
export TMPDIR=/tmp
timeout -k 10 100 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- scripts/_build/rl_stream 32 4 16 direct > $OUT/trace.log 2>&1
for q in 4 8 16; do GPU_MAX_HW_QUEUES=$q timeout -k 10 60 scripts/_build/rl_stream 64 4 16 direct > $OUT/rl_q$q.json 2>&1; done
timeout -k 10 300 python -u scripts/probe_gf2.py run > $OUT/probe_gf2.log 2>&1
