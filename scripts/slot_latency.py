"""Latency of the synchronous AEAD slot (ptls_aead_encrypt / ptls_aead_decrypt through the exported
ptls_aead_algorithm_t, as picotls' record layer calls it) and of the streaming record-layer sequence,
per record size.  Host buffers in, host buffers out (one GPU round trip per call): zero-copy (the kernel
reads and writes the pinned staging buffer over PCIe) or DMA copies in and out."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (one HIP runtime for torch and the engine)

    import rapido_amd as ra
    ra.require_gpu()
    key, iv = bytes(range(16)), bytes(range(12))
    enc = ra.aead_new_direct("aes128gcm", True, key, iv)
    dec = ra.aead_new_direct("aes128gcm", False, key, iv)
    res = {}
    # window kernels zero-copy (the default), window kernels with DMA copies, batch kernels with DMA copies
    # window-zerocopy-seg64: the same with the 64-position segments (32-position ones are the default for a
    # single record, ptls_mi355x_set_seg32_records)
    for mode, limit, zc in (("window-zerocopy", 1 << 30, 1 << 30), ("window-zerocopy-seg64", 1 << 30, 1 << 30),
                            ("window-copy", 1 << 30, 0), ("batch-copy", 0, 0)):
        ra.set_aead_window_records(limit)
        ra.set_slot_zero_copy_bytes(zc)
        ra.set_seg32_records(0 if mode.endswith("seg64") else ra.SEG32_AUTO)
        for L in (64, 1400, 4096, 16384):
            pt = bytes(i & 0xFF for i in range(L))
            aad = bytes([0x17, 3, 3, (L + 16) >> 8, (L + 16) & 0xFF])
            for _ in range(20):
                ct = enc.encrypt(pt, 1, aad)
                assert dec.decrypt(ct, 1, aad) == pt
            reps = 200
            t0 = time.perf_counter()
            for i in range(reps):
                ct = enc.encrypt(pt, i, aad)
            t1 = time.perf_counter()
            for i in range(reps):
                dec.decrypt(ct, reps - 1, aad)
            t2 = time.perf_counter()
            res[f"{mode}/{L}"] = {"encrypt_us": round((t1 - t0) / reps * 1e6, 1),
                                  "decrypt_us": round((t2 - t1) / reps * 1e6, 1)}
            print(mode, L, res[f"{mode}/{L}"], flush=True)
    ra.set_aead_window_records(2048)
    ra.set_slot_zero_copy_bytes(1 << 20)
    ra.set_seg32_records(ra.SEG32_AUTO)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
