"""Developer probe (not a test): first mismatches of GPU inflate vs the expected golden output."""
import hashlib
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402,F401
import dmx  # noqa: E402
G = os.path.join(ROOT, "tests", "golden")
man = json.load(open(os.path.join(G, "manifest.json")))
ctx = dmx.Context()
names = sys.argv[1:] or ["ref_L0_tiny.bmp", "ref_L1_tiny.bmp", "ref_L2_tiny.bmp"]
for v in man["vectors"]:
    if v["name"] not in names or "expect" not in v:
        continue
    s = open(os.path.join(G, v["stream"]), "rb").read()
    exp = open(os.path.join(G, v["expect"]), "rb").read()
    out = ctx.decompress(s)
    bad = [i for i in range(min(len(out), len(exp))) if out[i] != exp[i]]
    print(v["name"], len(s), len(out), len(exp), "mismatches", len(bad), bad[:8],
          [(out[i], exp[i]) for i in bad[:8]], s[:8].hex())
