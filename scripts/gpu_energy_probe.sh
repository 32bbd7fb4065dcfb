# Energy per HBM byte of the walk's access pattern (scripts/energy_probe.hip): socket power and gfx clock (amd-smi,
# 1-s samples after the clock settles) while each (K, filler) configuration streams for ~14 s.
#   CONFIGS="4:0 64:0 ..." TAG=... bash scripts/gpu_energy_probe.sh      -> gpurun_out/$TAG/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-energy}
mkdir -p $OUT
timeout -k 5 20 amd-smi metric -p -c --json > $OUT/idle.json 2>&1 || true
for c in ${CONFIGS:-4:0 8:0 64:0 4:300 8:300 64:300}; do
  k=${c%%:*}; f=${c##*:}
  timeout -k 10 60 scripts/_bin/energy_probe $k $f ${SECONDS_PER:-14} > $OUT/probe_${k}_${f}.json 2> $OUT/probe_${k}_${f}.err &
  pid=$!
  sleep 6
  for i in 1 2 3 4 5; do timeout -k 5 20 amd-smi metric -p -c --json > $OUT/smi_${k}_${f}_$i.json 2>&1 || true; sleep 1; done
  wait $pid
done
