import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        print(f"{d['config']['workload'][:48]:48s} K={d['config']['lanes_per_record']} value={d['value']:8.1f} seal={d['seal_gibps']:8.1f} open={d['open_gibps']:8.1f} frac={d['roofline']['frac']:.3f}")
