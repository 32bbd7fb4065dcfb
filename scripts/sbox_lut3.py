"""Maps the Boyar-Peralta S-box circuit (scripts/sbox_circuit.py) onto 3-input LUTs (v_bitop3_b32):
k = 3 cut enumeration + area-flow cover selection, then an exhaustive check of the mapped network.
Prints the LUT count and, with --emit, the C++ body of sbox_bs (rapido_amd/csrc/gcm_sbox.h; two-input gates there are VOP2 ops).

Truth-table convention: leaf 0 is the most significant bit of the table index (bitop3's src0).
"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sbox_circuit import fips_sbox, gates  # noqa: E402

INPUTS = [f"U{i}" for i in range(8)]


def parse():
    nodes = {}
    for lhs, rhs in gates():
        neg = rhs.startswith("~(")
        body = rhs[2:-1] if neg else rhs
        a, op, b = body.split()
        nodes[lhs] = (op, a, b, neg)
    return nodes


def evaluate_node(nodes, name, env):
    if name in env:
        return env[name]
    op, a, b, neg = nodes[name]
    x, y = evaluate_node(nodes, a, env), evaluate_node(nodes, b, env)
    v = (x ^ y) if op == "^" else (x & y)
    if neg:
        v ^= 1
    env[name] = v
    return v


def mapped():
    nodes = parse()
    order = list(nodes)
    outputs = [f"S{i}" for i in range(8)]
    fanout = {n: 0 for n in INPUTS + order}
    for n in order:
        fanout[nodes[n][1]] += 1
        fanout[nodes[n][2]] += 1
    for o in outputs:
        fanout[o] += 1
    cuts = {u: [frozenset([u])] for u in INPUTS}
    for n in order:
        _, a, b, _ = nodes[n]
        cs = {frozenset([n])}
        for ca, cb in itertools.product(cuts[a], cuts[b]):
            u = ca | cb
            if len(u) <= 3:
                cs.add(u)
        cuts[n] = sorted(cs, key=lambda c: (len(c), sorted(c)))
    af, best = {u: 0.0 for u in INPUTS}, {}
    for n in order:
        cand = [c for c in cuts[n] if c != frozenset([n])]

        def score(c):
            return 1.0 + sum(af[leaf] / max(fanout[leaf], 1) for leaf in c)

        best[n] = min(cand, key=lambda c: (score(c), len(c)))
        af[n] = score(best[n])
    need, luts = list(outputs), {}
    while need:
        n = need.pop()
        if n in luts or n in INPUTS:
            continue
        luts[n] = best[n]
        need.extend(leaf for leaf in best[n] if leaf not in INPUTS)
    rank = {n: i for i, n in enumerate(INPUTS + order)}
    topo = [n for n in order if n in luts]
    tts = {}
    for n in topo:
        leaves = sorted(luts[n], key=rank.get)
        tt = 0
        for idx in range(8):
            env = {leaf: (idx >> (len(leaves) - 1 - k)) & 1 for k, leaf in enumerate(leaves)}
            tt |= evaluate_node(nodes, n, env) << idx
        tts[n] = (leaves, tt)
    return topo, tts


def check(topo, tts):
    sb = fips_sbox()
    for v in range(256):
        env = {f"U{i}": (v >> (7 - i)) & 1 for i in range(8)}
        for n in topo:
            leaves, tt = tts[n]
            idx = 0
            for leaf in leaves:
                idx = (idx << 1) | env[leaf]
            env[n] = (tt >> idx) & 1
        got = sum(env[f"S{i}"] << (7 - i) for i in range(8))
        if got != sb[v]:
            raise SystemExit(f"LUT network wrong at {v}: {got:#x} != {sb[v]:#x}")


def emit(topo, tts):
    lines = []
    for n in topo:
        leaves, tt = tts[n]
        if len(leaves) == 3:
            lines.append(f"const V {n} = lut3<0x{tt:02x}>({leaves[0]}, {leaves[1]}, {leaves[2]});")
        elif len(leaves) == 2:  # a 3-input LUT with the second leaf repeated: index = 4a + 2b + b
            t3 = 0
            for idx in range(8):
                a, b = (idx >> 2) & 1, idx & 1
                t3 |= ((tt >> (2 * a + b)) & 1) << idx
            lines.append(f"const V {n} = lut3<0x{t3:02x}>({leaves[0]}, {leaves[1]}, {leaves[1]});")
        else:
            raise SystemExit("1-leaf LUT")
    return lines


def main():
    topo, tts = mapped()
    check(topo, tts)
    print(f"LUT3 cover: {len(topo)} LUTs for the 128-gate circuit (verified on all 256 inputs)", file=sys.stderr)
    if "--emit" in sys.argv:
        print("\n".join(emit(topo, tts)))


if __name__ == "__main__":
    main()
