"""PCIe copy rates of the GPU box (pinned host <-> HBM), for DESIGN.md's PCIe-inclusive figure:
H2D alone, D2H alone, and both at once on two streams."""
import time

import torch


def main():
    dev = torch.device("cuda:0")
    nbytes = 1 << 30
    h_a = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_b = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn, reps=4):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_a, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_b.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    t1, t2, t3 = timed(h2d), timed(d2h), timed(both)
    gb = nbytes / 1e9
    print(f"H2D {gb / t1:.1f} GB/s, D2H {gb / t2:.1f} GB/s, both at once {gb / t3:.1f} GB/s each way "
          f"({2 * gb / t3:.1f} GB/s total)")


if __name__ == "__main__":
    main()
