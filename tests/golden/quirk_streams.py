"""Large streams with the reference's lenient / quirky block semantics in their MIDDLE
(pin them where the fast paths run, not only on tiny vectors).

Test infrastructure: a small bit-level DEFLATE writer that emits, byte-aligned after the
previous block and ended by an empty stored block, the blocks whose decoding only the
reference's rules define:

  Q1  a stored block whose NLEN is not ~LEN          (inflate.hpp:293-303: NLEN unchecked)
  Q2  a non-final BTYPE-3 block                      (inflate.hpp:292: no case, an empty block)
  Q3  a fixed-Huffman block starting with a length-258 copy from 32768 bytes back
                                                     (a reference before the block: the
                                                      window of the stream, inflate.hpp:268)
  Q4  a dynamic block whose lit/len code-length RLE runs past HLIT (A-11: the reference
      decodes the two sequences with separate counts, inflate.hpp:216-220, so the overrun
      is dropped and the distance lengths start afresh)
  Q5  a dynamic block with a code 16 right after a code 17 (A-12: the reference's 16
      repeats the last LITERAL length, inflate.hpp:181, 198)

An RFC inflate (zlib) rejects Q4 and Q5 and warns on nothing else; the reference decodes
all five.  Two hosts for the quirk section:

  path5_stream(): zlib level 1 of 1 MiB of text (sync-flushed, so the quirk section starts
      byte-aligned), the quirk section, then zlib level 1 of the next 1 MiB with the previous
      32 KiB of output as its preset dictionary (its copies reach back across the quirk
      section), final.  Three 00 00 FF FF markers in 2 MiB and segments of ~1 MiB: not
      libdmx's layout, so the block-parallel path 5 decodes it.
  splice_into_segments(stream, at): a libdmx stream (segments behind 00 00 FF FF markers,
      made on the GPU by the test) with the quirk section inserted as one more segment at the
      first segment start at or after byte `at` (path 4's lanes decline it; Q3 then reaches
      into the previous segment).

The expected output of path5_stream() is the compiled reference's (SHA-256 in
manifest.json "quirk_path5", written by make_golden.py); the spliced stream is checked
against the oracle at test time.
"""
import heapq
import zlib

KB32 = 32768

# RFC 1951 code-length code order
PERM = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0
        self.out = bytearray()

    def put(self, v, nbits):  # LSB first
        self.acc |= (v & ((1 << nbits) - 1)) << self.n
        self.n += nbits
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def put_code(self, code, length):  # Huffman codes go MSB first
        self.put(int(format(code, "0%db" % length)[::-1], 2) if length else 0, length)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def empty_stored(self):  # 000, pad, 00 00 FF FF: ends the section byte-aligned
        self.put(0, 3)
        self.align()
        self.out += b"\x00\x00\xff\xff"

    def bytes(self):
        assert self.n == 0
        return bytes(self.out)


def canonical(lengths):
    """RFC 1951 3.2.2 canonical codes {symbol: (code, length)}."""
    maxl = max(lengths) if lengths else 0
    bl = [0] * (maxl + 2)
    for L in lengths:
        if L:
            bl[L] += 1
    code, nxt = 0, [0] * (maxl + 2)
    for b in range(1, maxl + 1):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    out = {}
    for s, L in enumerate(lengths):
        if L:
            out[s] = (nxt[L], L)
            nxt[L] += 1
    return out


def huffman_lengths(freq, maxbits):
    """Code lengths of a complete code over the symbols with freq > 0 (>= 2 of them), at most
    maxbits long (heap Huffman, then the overflow pushed back the zlib way)."""
    syms = [s for s, f in enumerate(freq) if f]
    assert len(syms) >= 2
    heap = [(freq[s], i, [s]) for i, s in enumerate(syms)]
    heapq.heapify(heap)
    depth = {s: 0 for s in syms}
    k = len(heap)
    while len(heap) > 1:
        fa, _, a = heapq.heappop(heap)
        fb, _, b = heapq.heappop(heap)
        for s in a + b:
            depth[s] += 1
        heapq.heappush(heap, (fa + fb, k, a + b))
        k += 1
    L = [0] * len(freq)
    for s in syms:
        L[s] = min(depth[s], maxbits)
    # Kraft repair: lengthen the shortest-but-one codes until the sum fits, then done (complete
    # because the fix only ever moves a leaf one level down into a freed slot)
    while sum(2.0 ** -L[s] for s in syms) > 1.0 + 1e-12:
        s = max((s for s in syms if L[s] < maxbits), key=lambda s: (L[s], -freq[s]))
        L[s] += 1
    # fill slack: shorten the most frequent codes while the sum stays <= 1
    changed = True
    while changed:
        changed = False
        for s in sorted(syms, key=lambda s: -freq[s]):
            if L[s] > 1 and sum(2.0 ** -L[x] for x in syms) + 2.0 ** -L[s] <= 1.0 + 1e-12:
                L[s] -= 1
                changed = True
    assert abs(sum(2.0 ** -L[s] for s in syms) - 1.0) < 1e-9
    return L


def write_dynamic_header(bw, ops, hlit, hdist):
    """ops: the code-length sequence as (symbol, extra value, extra bits) as the encoder means
    it (quirks included verbatim)."""
    pf = [0] * 19
    for s, _, _ in ops:
        pf[s] += 1
    pl = huffman_lengths(pf, 7) if sum(1 for x in pf if x) >= 2 else [1 if i in (0, 1) else 0 for i in range(19)]
    pc = canonical(pl)
    hclen = 19
    while hclen > 4 and pl[PERM[hclen - 1]] == 0:
        hclen -= 1
    bw.put(hlit - 257, 5)
    bw.put(hdist - 1, 5)
    bw.put(hclen - 4, 4)
    for i in range(hclen):
        bw.put(pl[PERM[i]], 3)
    for s, v, nb in ops:
        bw.put_code(*pc[s])
        if nb:
            bw.put(v, nb)


def rle_ops(lengths):
    """Plain RFC RLE of one code-length sequence (no quirks): 18/17 for zero runs, value then
    16s for other runs; no 16 after a 17/18."""
    ops, i, n = [], 0, len(lengths)
    while i < n:
        v = lengths[i]
        r = 1
        while i + r < n and lengths[i + r] == v:
            r += 1
        if v == 0 and r >= 3:
            left = r
            while left >= 11:
                k = min(138, left)
                ops.append((18, k - 11, 7))
                left -= k
            if left >= 3:
                ops.append((17, left - 3, 3))
                left = 0
            ops += [(0, 0, 0)] * left
        else:
            ops.append((v, 0, 0))
            left = r - 1
            while left >= 3:
                k = min(6, left)
                ops.append((16, k - 3, 2))
                left -= k
            ops += [(v, 0, 0)] * left
        i += r
    return ops


LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
            131, 163, 195, 227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
             2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0] + [k // 2 for k in range(2, 28)]


def put_match(bw, lc, dc, L, d):
    s = max(i for i in range(29) if LEN_BASE[i] <= L) if L != 258 else 28
    bw.put_code(*lc[257 + s])
    if LEN_EXTRA[s]:
        bw.put(L - LEN_BASE[s], LEN_EXTRA[s])
    k = max(i for i in range(30) if DIST_BASE[i] <= d)
    bw.put_code(*dc[k])
    if DIST_EXTRA[k]:
        bw.put(d - DIST_BASE[k], DIST_EXTRA[k])


def fixed_codes():
    lit = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
    return canonical(lit), canonical([5] * 30)


def literal_block(bw, data, final=False):
    """A plain dynamic block of literals (RFC RLE, no quirk): a strong block start for path 5."""
    freq = [0] * 286
    for b in data:
        freq[b] += 1
    freq[256] = 1
    L = huffman_lengths(freq, 15)
    hlit = max(257, max(s for s in range(286) if L[s]) + 1)
    lc = canonical(L)
    bw.put(1 if final else 0, 1)
    bw.put(2, 2)
    write_dynamic_header(bw, rle_ops(L[:hlit]) + rle_ops([1, 1]), hlit, 2)
    for b in data:
        bw.put_code(*lc[b])
    bw.put_code(*lc[256])


def quirk_section(text, far=True):
    """A plain dynamic block N0 (a unit start for path 5), then the five quirk blocks (Q1..Q5),
    byte-aligned start, ended by an empty stored block.  text: a few KiB of the text corpus
    (bytes a-z, space, newline) for block payloads.  far: Q3 copies from 32768 bytes back (into
    the output before the section); otherwise from inside the section (a section that is a
    segment of its own, decodable alone)."""
    bw = BitWriter()
    literal_block(bw, text[1300:1700])
    # Q1 stored, NLEN wrong
    bw.put(0, 1)
    bw.put(0, 2)
    bw.align()
    payload = text[:200]
    bw.put(len(payload), 16)
    bw.put(0x1234, 16)
    for b in payload:
        bw.put(b, 8)
    # Q2 BTYPE 3, not final: an empty block for the reference
    bw.put(0, 1)
    bw.put(3, 2)
    # Q3 fixed Huffman, first token a 258-byte copy from 32768 back, a few literals, EOB
    lc, dc = fixed_codes()
    bw.put(0, 1)
    bw.put(1, 2)
    put_match(bw, lc, dc, 258, 32768 if far else 400)
    for b in text[200:230]:
        bw.put_code(*lc[b])
    put_match(bw, lc, dc, 10, 32000 if far else 500)
    bw.put_code(*lc[256])
    # Q4 and Q5: lit/len code of 256 symbols of length 8 (every literal but '<' '=' '>', EOB,
    # lengths 3 and 4), distance code {1, 2} of length 1
    LL = [8] * 256 + [8, 8, 8] + [0] * 27
    for s in (60, 61, 62):
        LL[s] = 0
    lc8 = canonical(LL)
    dc1 = canonical([1, 1])
    body = text[230:1230]

    def block_body():
        i = 0
        while i < len(body):
            if i % 97 == 5:  # a copy every so often: length 3 or 4, distance 1 or 2
                put_match(bw, lc8, dc1, 3 + (i & 1), 1 + ((i >> 1) & 1))
                i += 1
                continue
            bw.put_code(*lc8[body[i]])
            i += 1
        bw.put_code(*lc8[256])

    # Q4: the zero run at the end of the lit/len lengths (symbols 259..285) is sent as ONE code
    # 18 of 30 zeros, 3 past HLIT = 286; the reference drops the 3, the distance lengths follow
    ops = rle_ops(LL[:259]) + [(18, 30 - 11, 7)] + rle_ops([1, 1])
    bw.put(0, 1)
    bw.put(2, 2)
    write_dynamic_header(bw, ops, 286, 2)
    block_body()
    # Q5: symbols 60..62 as a 17 (three zeros) and 63..65 as a 16 right after it: for the
    # reference the 16 repeats the last literal length (8); the rest plain
    ops = rle_ops(LL[:60]) + [(17, 0, 3), (16, 0, 2)] + rle_ops(LL[66:286]) + rle_ops([1, 1])
    bw.put(0, 1)
    bw.put(2, 2)
    write_dynamic_header(bw, ops, 286, 2)
    block_body()
    bw.empty_stored()
    return bw.bytes()


def path5_stream(text2m):
    """Marker-poor 2 MiB-class stream with the quirk section in the middle (see module doc).
    text2m: >= 2 MiB + 4 KiB of the text corpus."""
    half = 1 << 20
    a, b, q = text2m[:half], text2m[half:2 * half], text2m[2 * half:2 * half + 4096]
    z1 = zlib.compressobj(1, zlib.DEFLATED, -15)
    s1 = z1.compress(a) + z1.flush(zlib.Z_SYNC_FLUSH)
    sec = quirk_section(q, far=True)
    return s1, sec, b


def finish_path5(s1, sec, b, history):
    """history: the decoded output of s1 + sec (from the oracle or the reference); the second
    half is compressed against its last 32 KiB as a preset dictionary, so its copies reach
    back across the quirk section."""
    z2 = zlib.compressobj(1, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, history[-KB32:])
    return s1 + sec + z2.compress(b) + z2.flush()


def splice_into_segments(stream, at, sec):
    """libdmx stream with the quirk section inserted as one more segment at the first segment
    start (the byte after a 00 00 FF FF) at or after byte `at`."""
    i = stream.find(b"\x00\x00\xff\xff", max(0, at - 4))
    assert i >= 0
    cut = i + 4
    return stream[:cut] + sec + stream[cut:], cut
