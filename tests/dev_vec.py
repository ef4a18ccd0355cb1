"""Developer probe: inflate selected golden vectors on cuda:0, print sizes / hashes (DMX_RECS=1 for records)."""
import hashlib, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import dmx  # noqa: E402
G = os.path.join(ROOT, "tests", "golden")
vecs = json.load(open(os.path.join(G, "manifest.json")))["vectors"]
ctx = dmx.Context()
for v in vecs:
    if len(sys.argv) > 1 and not any(a in v["name"] for a in sys.argv[1:]):
        continue
    s = open(os.path.join(G, v["stream"]), "rb").read()
    try:
        out = ctx.decompress(s)
        ok = len(out) == v["out_len"] and hashlib.sha256(out).hexdigest() == v["out_sha256"]
        print(v["name"], len(s), len(out), v["out_len"], ok, ctx.stats().path, flush=True)
    except Exception as e:
        print(v["name"], "EXC", e, flush=True)
