"""Developer probe: per-phase cycle breakdown of the deflate / inflate kernels (DMX_PHASES)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "phases.txt")
os.environ["DMX_PHASES"] = out
import torch  # noqa: E402
import dmx  # noqa: E402
ctx = dmx.Context(segment_bytes=int(os.environ.get("DMX_SEG", "32768")))
ctx.set_timing(True)
n = int(os.environ.get("DMX_MIB", "256")) << 20
for kind in os.environ.get("DMX_KINDS", "repeat,text,zeros").split(","):
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    dmx.corpus_into(kind, n, host.data_ptr())
    d_in = host.cuda()
    cap = dmx.deflate_bound(n) + 64
    d_c = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    with open(out, "a") as f:
        f.write(f"# corpus {kind}\n")
    for lvl in (int(os.environ.get("DMX_LEVEL", "2")),):
        clen = ctx.deflate_device(d_in.data_ptr(), n, lvl, d_c.data_ptr(), cap)
        kd = ctx.stats().ms_main_kernel
        olen = ctx.inflate_device(d_c.data_ptr(), clen, d_o.data_ptr(), n + 64)
        ki = ctx.stats().ms_main_kernel
        with open(out, "a") as f:
            f.write(f"# {kind} L{lvl} ratio {n/clen:.3f} deflate_kernel_ms {kd:.3f} inflate_kernel_ms {ki:.3f} ok {olen == n and torch.equal(d_o[:n], d_in)}\n")
print(open(out).read())
