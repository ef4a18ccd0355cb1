"""Developer probe (not a test): the serial decoder (dev_inflate_pass 7) on one 16 MiB stream
shape; prints the first byte that differs from the input and the stream's block layout there."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import dmx  # noqa: E402
import streams  # noqa: E402
kind, shape = sys.argv[1], sys.argv[2]
mib = int(sys.argv[3]) if len(sys.argv) > 3 else 16
data = dmx.corpus(kind, mib << 20)
s = {"zlib6": lambda: streams.zlib_raw(data, 6), "zlib1": lambda: streams.zlib_raw(data, 1),
     "single": lambda: streams.single_fixed_block(data), "zfixed": lambda: streams.zfixed(data)}[shape]()
c = dmx.Context(inflate_pass=7)
d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
d_o = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
n = c.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), len(data) + 64)
out = d_o[:n].cpu().numpy().tobytes()
print("n", n, "want", len(data), flush=True)
bad = next((i for i in range(min(n, len(data))) if out[i] != data[i]), None) if out != data else None
if bad is None:
    print("identical" if out == data else "length differs")
else:
    import numpy as np
    a = np.frombuffer(out[:len(data)], dtype=np.uint8)
    b = np.frombuffer(data[:n], dtype=np.uint8)
    m = min(len(a), len(b))
    diff = np.nonzero(a[:m] != b[:m])[0]
    print("first diff", int(diff[0]), "count", len(diff), "last", int(diff[-1]))
    print("runs:", [(int(x), int(y)) for x, y in zip(diff[:-1][np.diff(diff) > 1][:10], diff[1:][np.diff(diff) > 1][:10])])
    i = int(diff[0])
    print("got ", out[i - 8:i + 24].hex())
    print("want", data[i - 8:i + 24].hex())
