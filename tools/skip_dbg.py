"""Developer aid (not a test): find the first segment whose deflate stream zlib rejects."""
import os
import sys
import zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import dmx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (64 << 20) + 1
kind = sys.argv[2] if len(sys.argv) > 2 else "mixed"
off = int(sys.argv[3]) if len(sys.argv) > 3 else n
ctx = dmx.Context(device=0)
d = dmx.corpus(kind, n, offset=off)
s = ctx.compress(d, 2)
o = zlib.decompressobj(-15)
out = bytearray()
pos = 0
try:
    while pos < len(s):
        out += o.decompress(s[pos:pos + 4096])
        pos += 4096
    print("ok", len(out) == n and bytes(out) == d)
except zlib.error as e:
    seg = len(out) // 32768
    print("zlib error", e, "after", len(out), "bytes; segment", seg, "of", (n + 32767) // 32768)
    seg_bytes = d[seg * 32768:(seg + 1) * 32768]
    print("segment head", seg_bytes[:64].hex())
    good = bytes(out) == d[:len(out)]
    print("output so far equal:", good)
    first = next((i for i in range(len(out)) if out[i] != d[i]), None)
    print("first wrong byte", first)
