"""Developer probe (not a test): inflate time of third-party streams on cuda:0.

argv: stream specs (default: the C3 bmp stand-in at zlib level 1):
  kind:MiB:zlevel          zlib raw stream of the corpus (MiB 0 with kind bmp: the 25,165,962-B
                           large.bmp stand-in); zlib's default memLevel 8
  zfixed:kind:MiB          zlib strategy Z_FIXED (runs of fixed-code blocks, no dynamic header)
  single:kind:MiB          one fixed-code block over the whole input (tests/streams.py)
Prints, per stream, the inflate path libdmx took, its HIP-event time and whether the bytes
match; with --ref also the reference inflate's time on one host core (oracle/_ref).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import dmx  # noqa: E402
import streams  # noqa: E402

BMP_N = 25165962
args = [a for a in sys.argv[1:] if not a.startswith("--")]
with_ref = "--ref" in sys.argv
specs = args or ["bmp:0:1"]
ctx = dmx.Context()
ctx.set_timing(True)
for spec in specs:
    f = spec.split(":")
    if f[0] in ("zfixed", "single"):
        mode, kind, n = f[0], f[1], int(f[2]) << 20
        data = dmx.corpus(kind, n)
        s = streams.zfixed(data) if mode == "zfixed" else streams.single_fixed_block(data)
    else:
        kind, mib, zl = f
        n = BMP_N if kind == "bmp" and mib == "0" else int(mib) << 20
        data = dmx.corpus(kind, n)
        s = streams.zlib_raw(data, int(zl))
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ref = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    for it in range(3):
        t0 = time.perf_counter()
        olen = ctx.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), n + 64)
        wall = time.perf_counter() - t0
        st = ctx.stats()
        ok = olen == n and torch.equal(d_o[:n], ref)
        print(f"{spec} n={n} clen={len(s)} path={st.path} segs={st.segments} "
              f"dev_ms={st.ms_device_total:.3f} main_ms={st.ms_main_kernel:.3f} wall_ms={wall * 1e3:.1f} "
              f"GBps={n / st.ms_device_total / 1e6:.2f} ok={ok}", flush=True)
    if with_ref:
        from oracle_bind import Reference
        if Reference.available():
            t0 = time.perf_counter()
            Reference().decompress(s)
            print(f"{spec} reference inflate 1 core: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
