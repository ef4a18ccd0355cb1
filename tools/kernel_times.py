"""Developer timing probe (not a test): per-corpus deflate/inflate kernel times on cuda:0.

argv: MiB (default 256), corpora (comma list), level.  Prints one line per corpus with the main
kernel time of each direction (HIP events), the inflate path taken and a byte-exact check.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402
import dmx  # noqa: E402

n = (int(sys.argv[1]) if len(sys.argv) > 1 else 256) << 20
kinds = (sys.argv[2] if len(sys.argv) > 2 else "repeat,text,mixed,random,bmp").split(",")
lvl = int(sys.argv[3]) if len(sys.argv) > 3 else 2
seg = int(os.environ.get("DMX_SEG", "32768"))
ctx = dmx.Context(segment_bytes=seg)
ctx.set_timing(True)
cap = dmx.deflate_bound(n) + 64
d_c = torch.empty(cap, dtype=torch.uint8, device="cuda")
d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
host = torch.empty(n, dtype=torch.uint8).pin_memory()
for kind in kinds:
    dmx.corpus_into(kind, n, host.data_ptr())
    d_in = host.cuda()
    best_d = best_i = 1e9
    for _ in range(3):
        clen = ctx.deflate_device(d_in.data_ptr(), n, lvl, d_c.data_ptr(), cap)
        best_d = min(best_d, ctx.stats().ms_main_kernel)
        d_o.zero_()
        olen = ctx.inflate_device(d_c.data_ptr(), clen, d_o.data_ptr(), n + 64)
        st = ctx.stats()
        best_i = min(best_i, st.ms_main_kernel)
    ok = olen == n and torch.equal(d_o[:n], d_in)
    print(f"{kind:7s} n={n} clen={clen} ratio={n / clen:.3f} deflate {best_d:.3f} ms "
          f"({n / best_d / 1e6:.1f} GB/s) inflate {best_i:.3f} ms ({n / best_i / 1e6:.1f} GB/s) "
          f"path={st.path} ok={ok}", flush=True)
