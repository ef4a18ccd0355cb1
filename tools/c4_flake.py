"""Developer probe (not a test): tests/test_gpu_parity.py::test_c4_eight_shards_of_1GiB_mixed_on_one_gpu's
stream built and inflated several times in one process; prints the stream's hash (deflate
determinism) and the inflate path each time."""
import hashlib
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
import torch  # noqa: E402
import dmx  # noqa: E402
import shard  # noqa: E402
ctx = dmx.Context()
n, world = 1 << 30, 8
host = torch.empty(n, dtype=torch.uint8).pin_memory()
dmx.corpus_into("mixed", n, host.data_ptr())
d_in = host.cuda()
d_out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    parts = []
    for r in range(world):
        b, e = shard.shard_range(n, r, world, 32768)
        buf = torch.empty(dmx.deflate_bound(e - b) + 64, dtype=torch.uint8, device="cuda")
        L = ctx.deflate_device(d_in.data_ptr() + b, e - b, 2, buf.data_ptr(), buf.numel(), not_final=(r < world - 1))
        parts.append(buf[:L])
    full = torch.cat(parts)
    h = hashlib.sha256(full.cpu().numpy().tobytes()).hexdigest()[:16]
    d_out.zero_()
    olen = ctx.inflate_device(full.data_ptr(), full.numel(), d_out.data_ptr(), n + 64)
    st = ctx.stats()
    print(it, "stream", full.numel(), h, "path", st.path, "ok", olen == n and torch.equal(d_out[:n], d_in), flush=True)
