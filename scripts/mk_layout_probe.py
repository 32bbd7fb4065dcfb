"""Multi-key batches: what a launch over 64 sessions costs against one session, by how the sessions' records lie in the
batch ("Multi-key batches").  1 M x 1400 B AES-128 records, seal and open, HIP events around each
call (the by-key sort and the key-range prep run inside the call), interleaved rounds on one box:

  single      one key, the single-key batch kernels (the reference point)
  mk1         one key through the multi-key kernels (their own cost, with nothing to switch)
  contiguous  64 sessions, each session's records one contiguous run
  windows     64 sessions, runs of 16 records (a rapido send window) of a random session each
  random      64 sessions, every record of a random session

    python scripts/mk_layout_probe.py [--rounds 6] [--keys 64]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--keys", type=int, default=64)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=1400)
    a = ap.parse_args()
    import numpy as np
    import torch

    import rapido_amd as ra
    from rapido_amd import records
    n, L, nk = a.n, a.length, a.keys
    lengths = np.full(n, L, dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=256)
    recs["seq"] = np.arange(n, dtype=np.uint64)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)
    dev = torch.device("cuda:0")
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev)
    d_ct, d_pt = torch.zeros_like(d_src), torch.zeros_like(d_src)
    d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
    d_aad = torch.from_numpy(aad).to(dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    rng = np.random.default_rng(5)
    engines = [ra.Engine(bytes((b + 7 * k) & 0xFF for b in range(16))) for k in range(nk)]
    ivs = [bytes((b + k) & 0xFF for b in range(12)) for k in range(nk)]
    mk = ra.MultiKey(engines, ivs)
    mk1 = ra.MultiKey(engines[:1], ivs[:1])
    layouts = {
        "mk1": np.zeros(n, dtype=np.int32),
        "contiguous": (np.arange(n) * nk // n).astype(np.int32),
        "windows": np.repeat(rng.integers(0, nk, (n + 15) // 16), 16)[:n].astype(np.int32),
        "random": rng.integers(0, nk, n).astype(np.int32),
    }
    d_k = {k: torch.from_numpy(v).to(dev) for k, v in layouts.items()}
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def run(name):
        ev[0].record()
        if name == "single":
            engines[0].seal_batch(ivs[0], d_recs.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr(), s)
        else:
            (mk1 if name == "mk1" else mk).seal_batch(d_recs.data_ptr(), d_k[name].data_ptr(), n, d_src.data_ptr(),
                                                       d_ct.data_ptr(), d_aad.data_ptr(), s)
        ev[1].record()
        if name == "single":
            engines[0].open_batch(ivs[0], d_recs.data_ptr(), n, d_ct.data_ptr(), d_pt.data_ptr(), d_aad.data_ptr(),
                                  d_st.data_ptr(), s)
        else:
            (mk1 if name == "mk1" else mk).open_batch(d_recs.data_ptr(), d_k[name].data_ptr(), n, d_ct.data_ptr(),
                                                       d_pt.data_ptr(), d_aad.data_ptr(), d_st.data_ptr(), s)
        ev[2].record()
        torch.cuda.synchronize()
        st = d_st.cpu().numpy()
        assert (st == L).all(), name
        return ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])

    names = ["single", "mk1", "contiguous", "windows", "random"]
    res = {k: {"seal": [], "open": []} for k in names}
    for r in range(a.rounds + 1):
        for name in names:
            se, op = run(name)
            if r:
                res[name]["seal"].append(se)
                res[name]["open"].append(op)
    gib = n * L / 2 ** 30
    out = {"n": n, "length": L, "keys": nk, "rounds": a.rounds}
    ref = None
    for name in names:
        se, op = statistics.median(res[name]["seal"]), statistics.median(res[name]["open"])
        both = 2 * gib / ((se + op) / 1e3)
        ref = ref or both
        out[name] = {"seal_ms": round(se, 4), "open_ms": round(op, 4), "seal_gibps": round(gib / (se / 1e3), 1),
                     "open_gibps": round(gib / (op / 1e3), 1), "seal_open_gibps": round(both, 1),
                     "vs_single": round(both / ref, 4)}
        print(f"{name:11s} seal {se:7.3f} ms  open {op:7.3f} ms  seal+open {both:8.1f} GiB/s  x{both / ref:.3f}",
              flush=True)
    print(json.dumps(out))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
