"""GPU: Adler-32 / CRC-32 kernels and the zlib / gzip containers.

Checksums are compared with Python's zlib (the reference has none: its decompressZlib skips the
header and ignores the trailer, inflate.hpp:326-361, SURVEY A-9).  Containers are checked both
ways: our framed streams decode with zlib / gzip, and zlib's / gzip's streams decode with ours,
verified on the GPU."""
import gzip
import random
import zlib

import pytest

import dmx

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 255, 4095, 16383, 16384, 16385, 65535, 65537,
         (1 << 20) + 7, (16 << 20) + 3, (17 << 20) - 1]


@pytest.mark.parametrize("n", SIZES)
def test_checksums_host_api(ctx, n):
    d = random.Random(n).randbytes(n)
    assert ctx.adler32(d) == zlib.adler32(d)
    assert ctx.crc32(d) == zlib.crc32(d)
    # chained from a previous value, as zlib's adler32(init, ...) / crc32(init, ...)
    assert ctx.adler32(d, 0x1234ABCD % (65521 << 16)) == zlib.adler32(d, 0x1234ABCD % (65521 << 16))
    assert ctx.crc32(d, 0xDEADBEEF) == zlib.crc32(d, 0xDEADBEEF)


def test_checksums_device_misaligned_and_large(ctx):
    import torch
    n = (256 << 20) + 12345
    host = torch.empty(n + 64, dtype=torch.uint8).pin_memory()
    dmx.corpus_into("mixed", n + 64, host.data_ptr())
    d = host.cuda()
    raw = host.numpy().tobytes()
    for off in (0, 1, 3, 5, 13, 16, 31):
        for ln in (0, 1, 100, 1 << 20, n - 40):
            ref = raw[off: off + ln]
            assert ctx.adler32_device(d.data_ptr() + off, ln) == zlib.adler32(ref), (off, ln)
            assert ctx.crc32_device(d.data_ptr() + off, ln) == zlib.crc32(ref), (off, ln)


def test_checksum_of_constant_runs(ctx):
    for b in (0, 0xFF):  # worst cases for the Adler sums, zero runs for the CRC register
        d = bytes([b]) * ((5 << 20) + 11)
        assert ctx.adler32(d) == zlib.adler32(d)
        assert ctx.crc32(d) == zlib.crc32(d)


@pytest.mark.parametrize("kind", ["text", "mixed", "zeros", "random"])
@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_zlib_gzip_roundtrip_both_ways(ctx, kind, level):
    d = dmx.corpus(kind, 300007, offset=4242)
    z = ctx.compress_zlib(d, level)
    assert zlib.decompress(z) == d
    assert (z[0] * 256 + z[1]) % 31 == 0 and z[0] == 0x78
    g = ctx.compress_gzip(d, level)
    assert gzip.decompress(g) == d
    assert ctx.inflate_zlib(z) == d and ctx.inflate_gzip(g) == d
    assert ctx.inflate_zlib(zlib.compress(d, 6)) == d
    assert ctx.inflate_gzip(gzip.compress(d, 6)) == d


def test_empty_containers(ctx):
    assert zlib.decompress(ctx.compress_zlib(b"")) == b""
    assert gzip.decompress(ctx.compress_gzip(b"")) == b""
    assert ctx.inflate_zlib(zlib.compress(b"")) == b""
    assert ctx.inflate_gzip(gzip.compress(b"")) == b""


def test_gzip_optional_header_fields(ctx):
    d = dmx.corpus("text", 50000)
    body = zlib.compressobj(6, zlib.DEFLATED, -15)
    raw = body.compress(d) + body.flush()
    # FEXTRA | FNAME | FCOMMENT | FHCRC
    hdr = bytes([0x1F, 0x8B, 8, 4 | 8 | 16 | 2, 0, 0, 0, 0, 0, 3]) + b"\x03\x00abc" + b"name.txt\x00" + \
        b"a comment\x00"
    hdr += (zlib.crc32(hdr) & 0xFFFF).to_bytes(2, "little")
    g = hdr + raw + zlib.crc32(d).to_bytes(4, "little") + len(d).to_bytes(4, "little")
    assert gzip.decompress(g) == d
    assert ctx.inflate_gzip(g) == d


def test_corrupt_trailers_and_headers(ctx):
    d = dmx.corpus("text", 100000)
    z = bytearray(zlib.compress(d))
    z[-1] ^= 1
    with pytest.raises(dmx.DmxError) as e:
        ctx.inflate_zlib(bytes(z))
    assert e.value.code == dmx.DMX_ERR_CHECKSUM
    assert ctx.inflate_zlib(bytes(z), verify=False) == d  # the reference's behaviour: no check
    g = bytearray(gzip.compress(d))
    g[-5] ^= 0x80  # CRC byte
    with pytest.raises(dmx.DmxError) as e:
        ctx.inflate_gzip(bytes(g))
    assert e.value.code == dmx.DMX_ERR_CHECKSUM
    g = bytearray(gzip.compress(d))
    g[-1] ^= 1  # ISIZE
    with pytest.raises(dmx.DmxError) as e:
        ctx.inflate_gzip(bytes(g))
    assert e.value.code == dmx.DMX_ERR_CHECKSUM
    with pytest.raises(dmx.DmxError) as e:
        ctx.inflate_zlib(b"\x78\x9d" + bytes(z[2:]))  # FCHECK wrong
    assert e.value.code == dmx.DMX_ERR_DATA
    with pytest.raises(dmx.DmxError) as e:
        ctx.inflate_gzip(b"\x1f\x8c" + bytes(g[2:]))
    assert e.value.code == dmx.DMX_ERR_DATA


def test_reference_decompress_zlib_unchanged(ctx):
    """decompressZlib keeps the reference's semantics (skip 2 bytes, no trailer check)."""
    d = dmx.corpus("text", 20000)
    z = bytearray(zlib.compress(d))
    z[-1] ^= 0xFF
    assert ctx.decompress_zlib(bytes(z)) == d


# ---------------------------------------------------------------------------------------
# file-path overloads: streaming I/O (deflate.hpp:755-777, inflate.hpp:390-408)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 32768, (64 << 20) - 1, (64 << 20) + 1, (150 << 20) + 4321])
def test_file_roundtrip_streaming(ctx, oracle, tmp_path, n):
    src, comp, back = tmp_path / "in.bin", tmp_path / "c.deflate", tmp_path / "out.bin"
    d = dmx.corpus("mixed", n, offset=n)
    src.write_bytes(d)
    a, b = ctx.compress_file(str(src), str(comp), 2)
    s = comp.read_bytes()
    assert a == n and b == len(s)
    assert zlib.decompressobj(-15).decompress(s) == d  # one stream over all chunks
    if n <= (1 << 20):
        assert oracle.inflate(s) == d
    assert ctx.decompress_file(str(comp), str(back)) == n
    assert back.read_bytes() == d


def test_file_inflate_foreign_stream(ctx, tmp_path):
    d = dmx.corpus("text", (5 << 20) + 17)
    z = zlib.compressobj(6, zlib.DEFLATED, -15)
    (tmp_path / "z.deflate").write_bytes(z.compress(d) + z.flush())
    assert ctx.decompress_file(str(tmp_path / "z.deflate"), str(tmp_path / "o")) == len(d)
    assert (tmp_path / "o").read_bytes() == d


def test_file_missing_path_errors(ctx, tmp_path):
    with pytest.raises(dmx.DmxError) as e:
        ctx.compress_file(str(tmp_path / "nope"), str(tmp_path / "x"))
    assert e.value.code == dmx.DMX_ERR_ARG
