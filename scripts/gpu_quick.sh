# quick GPU check: parity tests, then a short bench per lanes-per-record setting
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > $OUT/tests.log 2>&1
for k in ${LANES:-1 2 4}; do
  timeout -k 10 240 python bench.py --steps 6 --warmup 2 --lanes $k --no-cpu-baseline --no-e2e >> $OUT/b1400.jsonl 2>>$OUT/err.log
  timeout -k 10 240 python bench.py --workload 16k-aes128 --steps 4 --warmup 1 --lanes $k --no-cpu-baseline --no-e2e >> $OUT/b16k.jsonl 2>>$OUT/err.log
done
