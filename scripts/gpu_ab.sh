# Interleaved A/B of engine variants (scripts/ablate.py VARIANTS) on one box.
#   ABLATE_VARIANTS=a,b gpurun -- 'TAG=x bash scripts/gpu_ab.sh'   (WORKLOADS="1400 16k-aes128 16k" by default)
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for w in ${WORKLOADS:-1400 16k-aes128 16k}; do
  timeout -k 10 240 python -u scripts/ablate.py run --workload $w --rounds ${ROUNDS:-6} >> $OUT/ablate.txt 2>&1
done
grep -v '^{' $OUT/ablate.txt | grep -v amdgpu.ids
