"""Floor of a synchronous GPU call on this box: one tiny kernel launch + hipStreamSynchronize, timed from the host
(the part of every slot / record-layer call that no kernel change removes).

    python scripts/launch_floor.py
"""
import json
import statistics
import time

import torch


def main():
    x = torch.zeros(16, device="cuda:0")
    s = torch.cuda.current_stream()
    for _ in range(200):
        x.add_(1)
        s.synchronize()
    launch_sync, sync_only = [], []
    for _ in range(2000):
        t0 = time.perf_counter()
        x.add_(1)
        s.synchronize()
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        launch_sync.append((t1 - t0) * 1e6)
        sync_only.append((t2 - t1) * 1e6)
    print(json.dumps({"what": "tiny elementwise kernel (16 floats) + stream synchronize, host-timed, median of 2000, us",
                      "launch_and_sync_us": round(statistics.median(launch_sync), 2),
                      "idle_sync_us": round(statistics.median(sync_only), 2)}))


if __name__ == "__main__":
    main()
