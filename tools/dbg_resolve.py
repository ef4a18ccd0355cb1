import sys, os, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch, dmx
G = os.path.join(ROOT, "tests", "golden")
man = json.load(open(os.path.join(G, "manifest.json")))
v = next(x for x in man["vectors"] if x["name"] == "zlib_test.bmp_l1_fixed")
s = open(os.path.join(G, v["stream"]), "rb").read()
ref = open(os.path.join(G, "test.bmp"), "rb").read()
ctx = dmx.Context()
out = ctx.decompress(s)
print("path", ctx.stats().path, len(out), len(ref))
diff = [i for i in range(min(len(out), len(ref))) if out[i] != ref[i]]
print("ndiff", len(diff), "first", diff[:20])
if diff:
    i = diff[0]
    print("ref", ref[i-8:i+24].hex()); print("out", out[i-8:i+24].hex())
