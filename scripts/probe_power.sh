# Power and clock under the compute-only probe (scripts/probe_bs.hip), AES-256, T-table only vs 8 T-table + 8
# bitsliced waves: the part of scripts/aes256_study.sh that needs a ~35 s run to sample.  -> gpurun_out/${TAG:-aes256p}/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-aes256p}
mkdir -p $OUT
timeout -k 5 20 amd-smi metric -p -c --json > $OUT/idle.json 2>&1 || true
for ntt in 16 8; do
  PROBE_KEYS=32 PROBE_NTT=$ntt PROBE_REPS=1400 PROBE_UNITS_MULT=64 timeout -k 10 150 python scripts/probe_bs.py run > $OUT/probe_power_$ntt.log 2>&1 &
  pid=$!
  sleep 15
  for i in 1 2 3 4 5; do timeout -k 5 20 amd-smi metric -p -c --json > $OUT/probe_${ntt}_$i.json 2>&1 || true; sleep 1; done
  wait $pid
done
