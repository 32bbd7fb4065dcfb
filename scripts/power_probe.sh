# Power and clocks the MI355X holds under the batch kernels (DVFS): amd-smi samples while a long bench runs.
#   gpurun -- 'bash scripts/power_probe.sh'
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-power}
mkdir -p $OUT
timeout -k 5 20 amd-smi metric -p -c --json > $OUT/idle.json 2>&1 || true
for ws in 16k-aes128:3000 1400:8000 16k:2500; do
  w=${ws%%:*}; steps=${ws##*:}
  timeout -k 10 150 python bench.py --workload $w --steps $steps --warmup 2 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/bench_$w.json 2> $OUT/bench_$w.err &
  pid=$!
  sleep 10
  for i in 1 2 3 4 5 6 7 8; do
    timeout -k 5 20 amd-smi metric -p -c --json > $OUT/load_${w}_$i.json 2>&1 || true
    sleep 1
  done
  wait $pid
done
