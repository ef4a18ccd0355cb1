"""Developer probe (not a test): the serial decoder alone (dev_inflate_pass 7) on 16 MiB streams
of four shapes, with DMX_FB_DEBUG's per-phase cycle counts on stderr."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("DMX_FB_DEBUG", "1")
import torch  # noqa: E402
import dmx  # noqa: E402
import streams  # noqa: E402
c = dmx.Context(inflate_pass=7)
mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
for kind, shape in [("mixed", "zlib6"), ("text", "zlib1"), ("mixed", "single"), ("bmp", "zfixed")]:
    data = dmx.corpus(kind, mib << 20)
    s = {"zlib6": lambda: streams.zlib_raw(data, 6), "zlib1": lambda: streams.zlib_raw(data, 1),
         "single": lambda: streams.single_fixed_block(data), "zfixed": lambda: streams.zfixed(data)}[shape]()
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    ms = 1e30
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = c.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), len(data) + 64)
        ms = min(ms, (time.perf_counter() - t) * 1e3)
    ok = d_o[:n].cpu().numpy().tobytes() == data
    print(f"{kind} {shape}: {len(s)} B -> {n} B in {ms:.1f} ms = {len(data) / ms / 1e3:.1f} MB/s ok {ok}", flush=True)
    sys.stderr.flush()
