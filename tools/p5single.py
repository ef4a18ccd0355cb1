"""Developer probe (not a test): path-5 outcome of one fixed-code block over N MiB of mixed data
(tests/streams.py), with DMX_FB_DEBUG's unit / chain-break lines on stderr."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("DMX_FB_DEBUG", "1")
import torch  # noqa: E402,F401
import dmx  # noqa: E402
import streams  # noqa: E402
ctx = dmx.Context()
for mib in [int(x) for x in (sys.argv[1:] or ["1", "4", "16"])]:
    data = dmx.corpus("mixed", mib << 20)
    for final in (True, False):
        # (not final: an empty final fixed block follows in the same bit stream; appended at a
        # byte boundary instead, the pad bits would read as a stored header: no final block)
        s = streams.single_fixed_block(data, final=final, close=True)
        out = ctx.decompress(s)
        print(f"single {mib} MiB final={final}: path {ctx.stats().path} ok {out == data}", flush=True)
        sys.stderr.flush()
