# Which limiter holds the gfx clock under the batch kernels: amd-smi's throttle/violation status, temperatures,
# power and clocks, sampled while bench.py runs the north-star workload (and, for contrast, the compute-only probe).
#   gpurun -- 'bash scripts/throttle_probe.sh'  ->  gpurun_out/${TAG:-throttle}/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-throttle}
mkdir -p $OUT
timeout -k 5 30 amd-smi metric --help > $OUT/metric_help.txt 2>&1 || true
timeout -k 5 20 amd-smi metric --json > $OUT/idle_all.json 2>&1 || true
timeout -k 10 150 python bench.py --workload 16k-aes128 --steps 3000 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/bench_16k-aes128.json 2> $OUT/bench.err &
pid=$!
sleep 10
for i in 1 2 3; do
  timeout -k 5 30 amd-smi metric --json > $OUT/load_all_$i.json 2>&1 || true
  sleep 1
done
wait $pid
PROBE_MODES=2 PROBE_KEYS=16 PROBE_UNITS_PER_WAVE=480 PROBE_REPS=800 timeout -k 10 150 python scripts/probe_gf2.py run > $OUT/probe.log 2>&1 &
pid=$!
sleep 12
for i in 1 2; do
  timeout -k 5 30 amd-smi metric --json > $OUT/probe_all_$i.json 2>&1 || true
  sleep 1
done
wait $pid
