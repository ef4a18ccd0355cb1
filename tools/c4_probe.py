"""Developer probe (not a test): config C4's block size on one GPU -- 1 GiB of the mixed corpus
deflated and inflated with 64 KiB and 32 KiB segments (HIP-event times, ratio, inflate path),
under rocprofv3 for the per-kernel split.  argv: [corpus] [MiB]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402
import dmx  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
n = (int(sys.argv[2]) if len(sys.argv) > 2 else 1024) << 20
host = torch.empty(n, dtype=torch.uint8).pin_memory()
dmx.corpus_into(kind, n, host.data_ptr())
d_in = host.cuda()
cap = dmx.deflate_bound(n) + 64
d_c = torch.empty(cap, dtype=torch.uint8, device="cuda")
d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
for seg in (65536, 32768):
    ctx = dmx.Context(segment_bytes=seg)
    ctx.set_timing(True)
    td, ti = [], []
    for it in range(5):
        clen = ctx.deflate_device(d_in.data_ptr(), n, 2, d_c.data_ptr(), cap)
        td.append(ctx.stats().ms_device_total)
        olen = ctx.inflate_device(d_c.data_ptr(), clen, d_o.data_ptr(), n + 64)
        ti.append(ctx.stats().ms_device_total)
        path = ctx.stats().path
    ok = olen == n and bool(torch.equal(d_o[:n], d_in))
    td, ti = sorted(td)[2], sorted(ti)[2]
    print(f"{kind} seg={seg}: ratio {n / clen:.4f} deflate {td:.3f} ms ({n / td / 1e6:.1f} GB/s) "
          f"inflate {ti:.3f} ms ({n / ti / 1e6:.1f} GB/s) path {path} ok={ok}", flush=True)
    ctx.close()
