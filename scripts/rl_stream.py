"""Runs bench.record_layer_stream alone (the host-to-host record-layer side figure), for profiling:
    rocprofv3 --kernel-trace -d gpurun_out/x -o run --output-format csv -- python scripts/rl_stream.py [nwin] [depth] [transport]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 64
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 4
print(json.dumps(bench.record_layer_stream(16, nwin=nwin, depth=depth, transport=sys.argv[3] if len(sys.argv) > 3 else "direct")))
