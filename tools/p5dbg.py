import sys, zlib
sys.path.insert(0, "deflate.hpp_amd")
import dmx
d = dmx.corpus("mixed", 3 << 20, offset=4321)
z = zlib.compressobj(3, zlib.DEFLATED, -15, 2, 0)
s = z.compress(d) + z.flush()
ctx = dmx.Context()
out = ctx.decompress(s)
print("path", ctx.stats().path, out == d, len(s))
