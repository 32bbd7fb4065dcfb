# scripts/pmc_write_ab.sh -- write-traffic A/B of the K = 4 store variants (GPU box, via gpurun):
#   interleaved throughput (scripts/ablate.py) and one rocprofv3 WRITE_SIZE pass per variant library
#   (scripts/pmc_lengths.py through PTLS_MI355X_LIB).  Build the variants first:
#   ABLATE_VARIANTS=base,pair,ntload python scripts/ablate.py build
set -e
mkdir -p gpurun_out/r02q
R=$GRAFT_REPO_ROOT
for w in 1400 16k-aes128; do ABLATE_VARIANTS=base,pair,ntload timeout -k 10 200 python -u $R/scripts/ablate.py run --workload $w --rounds 7 >> $R/gpurun_out/r02q/ab.txt 2>&1; done
cd /tmp && export TMPDIR=/tmp
export PMC_LENGTHS=1400,16384 PMC_LANES=4 PMC_BYTES=1073741824
for v in base pair ntload; do
PTLS_MI355X_LIB=$R/rapido_amd/_lib/variants/$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/r02q/w_$v -o run --output-format csv -- python3 $R/scripts/pmc_lengths.py > $R/gpurun_out/r02q/w_$v.txt 2>&1
done
