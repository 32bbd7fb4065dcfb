#!/bin/bash
# round 6: the new GPU tests, then the whole GPU suite, then the single-key kernels against round 5's (interleaved A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r06b}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_fault_handling.py \
    tests/test_gpu_multikey.py tests/test_gpu_record_layer.py > "$out/new_tests.log" 2>&1 || { tail -30 "$out/new_tests.log"; exit 1; }
tail -3 "$out/new_tests.log"
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
for w in 1400 16k-aes128 16k; do
    ABLATE_VARIANTS=base,head timeout -k 10 300 python scripts/ablate.py run --workload $w --rounds 6 >> "$out/ablate.txt" 2>&1 || exit 1
done
cat "$out/ablate.txt" | grep -v '^{'
