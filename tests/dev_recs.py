"""Developer probe (not a test): per-candidate outcome flags of the inflate passes (DMX_RECS)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
os.environ["DMX_RECS"] = "1"
import torch  # noqa: E402
import dmx  # noqa: E402
n = (int(sys.argv[1]) if len(sys.argv) > 1 else 16) << 20
ctx = dmx.Context()
for kind in (sys.argv[2] if len(sys.argv) > 2 else "mixed,text,repeat,random,bmp").split(","):
    data = dmx.corpus(kind, n)
    s = ctx.compress(data, 2)
    print(kind, len(s), flush=True)
    assert ctx.decompress(s) == data
