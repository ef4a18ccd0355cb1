"""Third-party stream shapes the block-parallel inflate (path 5) must split without scanned
dynamic headers.  TEST INFRASTRUCTURE: builders of input streams, never used
by the product path.

- ``zfixed``: zlib's raw stream with strategy Z_FIXED (fixed-code blocks of <= 16 K symbols,
  stored blocks where the data does not compress, no dynamic block anywhere).
- ``single_fixed_block``: ONE fixed-code block of literals over the whole input (RFC 1951 3.2.6),
  written with numpy -- the "huge single block" case.
- ``zlib_raw``: zlib's raw stream at a level / memLevel / strategy.
"""
import zlib

import numpy as np


def zlib_raw(data, level=6, mem=8, strategy=zlib.Z_DEFAULT_STRATEGY):
    z = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return z.compress(data) + z.flush()


def zfixed(data, level=6):
    return zlib_raw(data, level, 8, zlib.Z_FIXED)


def single_fixed_block(data, final=True, close=False):
    """One fixed-Huffman block holding every input byte as a literal, then end of block.
    close (with final=False): an empty final fixed block follows in the same bit stream."""
    a = np.frombuffer(bytes(data), dtype=np.uint8).astype(np.uint32)
    code = np.where(a < 144, 0x30 + a, 0x190 + a - 144)  # fixed literal codes, MSB first
    ln = np.where(a < 144, 8, 9)
    j = np.arange(9, dtype=np.uint32)
    bits = ((code[:, None] >> np.maximum(ln[:, None] - 1 - j[None, :], 0)) & 1).astype(np.uint8)
    valid = j[None, :] < ln[:, None]
    body = bits[valid]  # row-major: each symbol's bits in sending order
    head = np.array([1 if final else 0, 1, 0], dtype=np.uint8)  # BFINAL, BTYPE = 01 (LSB first)
    eob = np.zeros(7, dtype=np.uint8)  # symbol 256: seven zero bits
    tail = [head, body, eob]
    if close and not final:
        tail += [np.array([1, 1, 0], dtype=np.uint8), eob]
    allbits = np.concatenate(tail)
    return np.packbits(allbits, bitorder="little").tobytes()
