"""Developer aid (not a test): one deflate (and optionally inflate) of a corpus on cuda:0, for
rocprofv3 counter passes.  argv: corpus MiB level [inflate: 0/1]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402
import dmx  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "repeat"
n = (int(sys.argv[2]) if len(sys.argv) > 2 else 256) << 20
lvl = int(sys.argv[3]) if len(sys.argv) > 3 else 2
inf = len(sys.argv) > 4 and sys.argv[4] == "1"
ctx = dmx.Context(segment_bytes=int(os.environ.get("DMX_SEG", "32768")))
host = torch.empty(n, dtype=torch.uint8).pin_memory()
dmx.corpus_into(kind, n, host.data_ptr())
d_in = host.cuda()
cap = dmx.deflate_bound(n) + 64
d_c = torch.empty(cap, dtype=torch.uint8, device="cuda")
clen = ctx.deflate_device(d_in.data_ptr(), n, lvl, d_c.data_ptr(), cap)
if inf:
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.inflate_device(d_c.data_ptr(), clen, d_o.data_ptr(), n + 64)
torch.cuda.synchronize()
print(kind, n, lvl, clen)
