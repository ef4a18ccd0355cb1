"""Developer probe (not a test): inflate time of third-party (zlib) streams on cuda:0.

argv: list of kind:MiB:zlevel (default: the C3 bmp stand-in at zlib level 1).  Prints, per
stream, the inflate path libdmx took, its HIP-event time and whether the bytes match.
"""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402
import dmx  # noqa: E402

BMP_N = 25165962
specs = sys.argv[1:] or ["bmp:0:1"]
ctx = dmx.Context()
ctx.set_timing(True)
for spec in specs:
    kind, mib, zl = spec.split(":")
    n = BMP_N if kind == "bmp" and mib == "0" else int(mib) << 20
    data = dmx.corpus(kind, n)
    # zlib's default memLevel 8: the bench's and the manifest's C3 stream (6,206,388 B)
    z = zlib.compressobj(int(zl), zlib.DEFLATED, -15)
    s = z.compress(data) + z.flush()
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ref = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    best = 1e30
    for it in range(3):
        t0 = time.perf_counter()
        olen = ctx.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), n + 64)
        wall = time.perf_counter() - t0
        st = ctx.stats()
        best = min(best, st.ms_device_total)
        ok = olen == n and torch.equal(d_o[:n], ref)
        print(f"{kind} n={n} z{zl} clen={len(s)} path={st.path} segs={st.segments} "
              f"dev_ms={st.ms_device_total:.3f} main_ms={st.ms_main_kernel:.3f} wall_ms={wall * 1e3:.1f} "
              f"GBps={n / st.ms_device_total / 1e6:.2f} ok={ok}", flush=True)
