"""Developer A/B check: hashes of deflate outputs over corpora x levels x segment sizes.
Run once per build (DMX_LIB=...) and diff the printed JSON: a change that must not alter
the emitted streams shows identical hashes."""
import hashlib
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import dmx  # noqa: E402
out = {}
for seg in (32768, 16384):
    ctx = dmx.Context(segment_bytes=seg)
    for kind in ("repeat", "text", "mixed", "random", "zeros", "bmp"):
        for n in (3 << 20, 1000003):
            data = dmx.corpus(kind, n)
            for lvl in (0, 1, 2, 3):
                c = ctx.compress(data, lvl)
                out[f"{seg}:{kind}:{n}:{lvl}"] = [len(c), hashlib.sha256(c).hexdigest()[:16]]
    ctx.close()
json.dump(out, open(sys.argv[1], "w"), indent=0, sort_keys=True)
print(len(out), "entries")
