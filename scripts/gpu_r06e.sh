#!/bin/bash
# round 6: the multi-key tests, the layout probe (with the one-key multi-key kernels), and its kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
out=$R/gpurun_out/${TAG:-r06e}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_multikey.py \
    > "$out/mk_tests.log" 2>&1 || { tail -30 "$out/mk_tests.log"; exit 1; }
tail -2 "$out/mk_tests.log"
timeout -k 10 300 python scripts/mk_layout_probe.py --rounds 8 > "$out/probe.txt" 2>&1 || { tail -20 "$out/probe.txt"; exit 1; }
grep -v '^{' "$out/probe.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 "$R/scripts/mk_layout_probe.py" --rounds 2 > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
