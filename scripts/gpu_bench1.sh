set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2 4 8; do
  timeout -k 10 240 python bench.py --steps 6 --warmup 2 --lanes $k --no-cpu-baseline --no-e2e >> gpurun_out/lanes_1400.jsonl 2>>gpurun_out/lanes.err
  timeout -k 10 240 python bench.py --workload 16k-aes128 --steps 4 --warmup 1 --lanes $k --no-cpu-baseline --no-e2e >> gpurun_out/lanes_16k.jsonl 2>>gpurun_out/lanes.err
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --e2e > gpurun_out/bench1.json 2> gpurun_out/bench1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof1.log 2>&1
