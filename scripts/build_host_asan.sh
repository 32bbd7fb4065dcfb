# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the engine library and of the record-layer stream
# driver (diagnostic; sanitizers on HOST code only: the device code is compiled as in the product, the host halves of
# gcm_engine.hip get -fsanitize through -Xarch_host, the C files directly).  Built here, run on the GPU box by
# scripts/gpu_host_asan.sh.  Outputs: scripts/_build/asan/{libptls_mi355x.so,rl_stream}
set -e
cd "$(dirname "$0")/.."
OUT=scripts/_build/asan
mkdir -p $OUT
SAN="-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
CFLAGS="-std=gnu99 -O1 -g -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $SAN"
for f in aead_slot tls_records record_layer; do
  gcc $CFLAGS -c rapido_amd/csrc/$f.c -o $OUT/$f.o
done
BID=$(python3 -c "import sys; sys.path.insert(0, '.'); from rapido_amd import build; print(build.source_build_id())")
printf 'const char *ptls_mi355x_build_id(void) { return "%s"; }\n' "$BID" > $OUT/build_id.c
gcc $CFLAGS -c $OUT/build_id.c -o $OUT/build_id.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -g -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -c rapido_amd/csrc/gcm_engine.hip -o $OUT/gcm_engine.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libptls_mi355x.so $OUT/gcm_engine.o $OUT/build_id.o \
  $OUT/aead_slot.o $OUT/tls_records.o $OUT/record_layer.o
gcc -std=gnu99 -O1 -g -rdynamic $SAN -o $OUT/rl_stream scripts/rl_stream.c -L$OUT -lptls_mi355x \
  -Wl,-rpath,'$ORIGIN' -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
echo "built $OUT (build id $BID)"
