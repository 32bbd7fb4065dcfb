"""Host <-> device copies for the GPU tests, through pinned (page-locked) host memory.

The engine never hands pageable memory to HIP: its slot calls stage through pinned memory, and the record layer works
on registered ranges or pinned staging.  The tests used to move their inputs and results with torch's `.cuda()` /
`.cpu()` on numpy arrays: pageable copies, which the HIP runtime performs by locking the user's pages for the DMA (or
staging them).  In round 6 the fault journal caught a GPU memory fault at a heap address during exactly such a copy,
with no engine work in flight since the last two successful device checks.  The tests now copy
through pinned buffers, as the engine itself does, so a GPU test exercises the engine rather than the runtime's
pageable-copy path.
"""
import numpy as np


def _host(a) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return a if a.flags.writeable else a.copy()  # torch.from_numpy warns on read-only arrays


def to_gpu(a, device="cuda"):
    """A device tensor holding a copy of the numpy array `a` (its dtype and shape), moved H2D from pinned memory."""
    import torch
    t = torch.from_numpy(_host(a))
    pinned = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    pinned.copy_(t)
    d = torch.empty(t.shape, dtype=t.dtype, device=device)
    d.copy_(pinned)  # synchronous: the pinned block may be reused once this returns
    return d


def to_cpu(t) -> np.ndarray:
    """A numpy copy of the device tensor `t`, moved D2H into pinned memory."""
    import torch
    pinned = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    pinned.copy_(t)  # synchronous
    return pinned.numpy().copy()
