"""Regenerated zlib fixtures: the multi-block zlib streams of tests/golden/manifest.json are not
committed (1.7 MB); a vector with a "zgen" spec is rebuilt from the corpus generator and zlib,
and its SHA-256 is checked against the manifest before use (the expected output is the
reference's, recorded by make_golden.py).  Spec keys: kind, n, offset, level, mem (memLevel),
strategy, flush_every (0: one compress call), flush ("full" or "sync")."""
import hashlib
import zlib


def zgen_stream(spec):
    import dmx
    d = dmx.corpus(spec["kind"], spec["n"], offset=spec["offset"])
    z = zlib.compressobj(spec["level"], zlib.DEFLATED, -15, spec.get("mem", 9), spec.get("strategy", 0))
    fe = spec.get("flush_every", 0)
    if not fe:
        return z.compress(d) + z.flush()
    mode = zlib.Z_FULL_FLUSH if spec.get("flush", "full") == "full" else zlib.Z_SYNC_FLUSH
    return b"".join(z.compress(d[i:i + fe]) + z.flush(mode) for i in range(0, len(d), fe)) + z.flush()


def stream_of(v, gold_dir):
    """The stream bytes of manifest vector v: a committed file when it has one, else regenerated
    and SHA-checked.  A zlib that makes other bytes (zlib-ng, another release) skips the vector
    under pytest, naming the version; the committed vectors still run."""
    import os
    if "zgen" in v and "stream" not in v:
        s = zgen_stream(v["zgen"])
        if hashlib.sha256(s).hexdigest() != v["stream_sha256"]:
            msg = (f"{v['name']}: zlib {zlib.ZLIB_RUNTIME_VERSION} produced another stream than the "
                   "1.2.11 one the reference's output was recorded on")
            try:
                import pytest
            except ImportError:
                raise RuntimeError(msg)
            pytest.skip(msg)
        return s
    with open(os.path.join(gold_dir, v["stream"]), "rb") as f:
        return f.read()
