"""Makes tests/golden/dmx/: streams produced by libdmx's GPU deflate (run on the MI355X box),
so the CPU tests (gloo multi-rank gather / scatter-inflate) exercise real libdmx output.

  python tests/golden/make_dmx_fixtures.py      # needs a gfx950 GPU
Each stream is checked against zlib and the oracle before it is written; manifest.json records
the corpus, byte range, level, flags and the SHA-256 of the decoded bytes."""
import hashlib
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
import dmx  # noqa: E402
from oracle_bind import Oracle  # noqa: E402

OUT = os.path.join(HERE, "dmx")
SEG = 32768


def main():
    os.makedirs(OUT, exist_ok=True)
    ctx = dmx.Context(segment_bytes=SEG)
    orc = Oracle()
    man = []
    total = (1 << 20) + 4321
    data = dmx.corpus("mixed", total)
    cut = 16 * SEG  # two shards at a segment boundary
    specs = [("mixed1M_L2.deflate", 0, total, 2, False),
             ("mixed1M_L2_shard0.deflate", 0, cut, 2, True),
             ("mixed1M_L2_shard1.deflate", cut, total, 2, False),
             ("mixed1M_L0_shard0.deflate", 0, cut, 0, True),
             ("mixed1M_L0_shard1.deflate", cut, total, 0, False)]
    for name, b, e, lvl, nf in specs:
        d_in = torch.frombuffer(bytearray(data[b:e]), dtype=torch.uint8).cuda()
        cap = dmx.deflate_bound(e - b) + 64
        d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        n = ctx.deflate_device(d_in.data_ptr(), e - b, lvl, d_out.data_ptr(), cap, not_final=nf)
        s = d_out[:n].cpu().numpy().tobytes()
        full = s + (b"\x03\x00" if nf else b"")
        assert zlib.decompressobj(-15).decompress(full) == data[b:e]
        assert orc.inflate(full) == data[b:e]
        open(os.path.join(OUT, name), "wb").write(s)
        man.append({"file": name, "corpus": "mixed", "begin": b, "end": e, "level": lvl, "not_final": nf,
                    "segment_bytes": SEG, "out_sha256": hashlib.sha256(data[b:e]).hexdigest()})
    json.dump({"corpus_total": total, "streams": man}, open(os.path.join(OUT, "manifest.json"), "w"), indent=1)
    print("wrote", len(man), "streams")


if __name__ == "__main__":
    main()
