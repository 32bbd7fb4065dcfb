# The MFMA-GHASH probe's resources per mode: PMC per 64 blocks (LDS busy, VALU and LDS
# instructions, MFMA busy, wave cycles, GRBM clock) and socket power / clock from amd-smi during a long run.
#   gpurun -- 'bash scripts/gpu_probe_gf2_pmc.sh'   ->  gpurun_out/${TAG:-gf2pmc}/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gf2pmc}
mkdir -p $OUT
for m in 0 1 3 2; do
  PROBE_MODES=$m PROBE_KEYS=16 PROBE_REPS=2 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_$m -o run --output-format csv -- python scripts/probe_gf2.py run > $OUT/pmc_$m.log 2>&1
done
timeout -k 5 20 amd-smi metric -p -c --json > $OUT/idle.json 2>&1 || true
for m in 0 1 3 2; do
  PROBE_MODES=$m PROBE_KEYS=16 PROBE_UNITS_PER_WAVE=480 PROBE_REPS=${REPS:-800} timeout -k 10 150 python scripts/probe_gf2.py run > $OUT/long_$m.log 2>&1 &
  pid=$!
  sleep 12
  for i in 1 2 3 4 5 6; do
    timeout -k 5 20 amd-smi metric -p -c --json > $OUT/power_${m}_$i.json 2>&1 || true
    sleep 1
  done
  wait $pid
done
