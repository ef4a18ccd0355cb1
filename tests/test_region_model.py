"""CPU model of path 5's fixed-code region map (inflate_blocks.hip: k_fb_smap / k_fb_swalk).

The kernel cuts a run of fixed-code blocks into chunks of 4096 bits and, for every chunk and entry
offset e < 32 (a fixed-code token is at most 31 bits), decodes to the first token boundary at or
past the next chunk; the true token path is the orbit of the region head under that map.  This
model restates one lane of k_fb_smap (fbs_lane) and the walk in Python and checks, on streams that
have no scanned unit starts (one huge fixed block, zlib Z_FIXED runs with stored blocks), that
every node the walk visits is a token boundary of a sequential decode -- realDecompress,
/root/reference/include/inflate.hpp:277-322 with the fixed trees of :280-283 -- with the right
BFINAL bit, and that the walk ends where the stream does.  Test infrastructure only."""
import zlib

import dmx
import streams

CH = 4096
LE = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


def _reader(s):
    nb, b = 8 * len(s), bytes(s) + bytes(16)

    def peek(p, k):
        if p >= nb:
            return 0
        return (int.from_bytes(b[p >> 3: (p >> 3) + 8], "little") >> (p & 7)) & ((1 << k) - 1)
    return peek, nb


def _rev(v, n):
    return int(format(v, "0%db" % n)[::-1], 2)


def _fixed_token(peek, p):
    """(kind, next bit) of the fixed-code token at p (RFC 1951 3.2.6)."""
    x = _rev(peek(p, 9), 9)
    if (x >> 2) < 0x18:
        sym, ln = 256 + (x >> 2), 7
    elif 0x30 <= (x >> 1) <= 0xBF:
        sym, ln = (x >> 1) - 0x30, 8
    elif 0xC0 <= (x >> 1) <= 0xC7:
        sym, ln = 280 + (x >> 1) - 0xC0, 8
    else:
        sym, ln = 144 + x - 0x190, 9
    if sym < 256:
        return "lit", p + ln
    if sym == 256:
        return "eob", p + 7
    p += ln + (LE[sym - 257] if sym <= 285 else 0)
    ds = _rev(peek(p, 5), 5)
    return "match", p + 5 + (DE[ds] if ds < 30 else 0)


def _lane(peek, nb, p, head, E, T):
    """fbs_lane: the results for entry BFINAL f = 0 and f = 1 ('END', 'LINK', 'FAIL' or a node)."""
    target = p - (p - E) % CH + CH
    eob_seen, hdr, fcur, hdr_read = False, head, 0, False
    while True:
        if hdr:
            if p >= T or p + 3 > nb:
                res = "LINK" if p == T < nb else "FAIL"
                break
            h = peek(p, 3)
            bf, bt = h & 1, h >> 1
            if bt == 2:
                res = "FAIL"
                break
            p += 3
            hdr_read = True
            if bt == 1:
                fcur, hdr = bf, False
                continue
            if bt == 0:
                p = (p + 7) & ~7
                if p + 32 > nb:
                    res = "FAIL"
                    break
                p += 32 + 8 * peek(p, 16)
                if p > nb:
                    res = "FAIL"
                    break
            if bf:
                res = "END"
                break
            continue
        if p >= T:
            res = "FAIL"
            break
        if p >= target:
            cc, off = divmod(p - E, CH)
            if off < 32:
                res = (cc, off)
                break
            target = E + (cc + 1) * CH
        kind, p = _fixed_token(peek, p)
        if kind == "eob":
            if not hdr_read:
                eob_seen = True
            elif fcur:
                res = "END"
                break
            hdr = True
        if p > nb:
            res = "FAIL"
            break
    if isinstance(res, tuple):
        return (res[0], fcur if hdr_read else 0, res[1]), ("END" if eob_seen else (res[0], 1, res[1]))
    return res, ("END" if eob_seen else res)


def _walk(s):
    peek, nb = _reader(s)
    memo = {}

    def nxt(node):
        if node not in memo:
            c, _, e = node
            r0, r1 = _lane(peek, nb, c * CH + e, c == 0, 0, nb)
            memo[(c, 0, e)], memo[(c, 1, e)] = r0, r1
        return memo[node]
    node, path = (0, 0, 0), []
    while True:
        v = nxt(node)
        if not isinstance(v, tuple):
            return path, v
        path.append(v)
        node = v


def _boundaries(s):
    """Token boundaries (bit, BFINAL of the block) of a sequential decode; the end bit."""
    peek, _ = _reader(s)
    p, out = 0, set()
    while True:
        bf, bt = peek(p, 1), peek(p + 1, 2)
        p += 3
        if bt == 0:
            p = (p + 7) & ~7
            p += 32 + 8 * peek(p, 16)
        elif bt == 1:
            while True:
                out.add((p, bf))
                kind, p = _fixed_token(peek, p)
                if kind == "eob":
                    break
        else:
            raise AssertionError("a dynamic block in a fixed-code stream")
        if bf:
            return out, p


def _check(s):
    bounds, _ = _boundaries(s)
    path, term = _walk(s)
    assert term == "END"
    assert len(path) >= 8 * len(s) // CH - 2  # one node per chunk (no stored data to skip)...
    for c, f, e in path:
        assert (c * CH + e, f) in bounds


def test_region_map_single_fixed_block():
    _check(streams.single_fixed_block(dmx.corpus("mixed", 96 << 10)))


def test_region_map_open_block_then_final():
    _check(streams.single_fixed_block(dmx.corpus("text", 64 << 10), final=False, close=True))


def test_region_map_zfixed_with_stored_blocks():
    data = dmx.corpus("mixed", 300 << 10)
    s = streams.zfixed(data)
    assert zlib.decompress(s, -15) == data
    bounds, _ = _boundaries(s)
    path, term = _walk(s)
    assert term == "END"
    for c, f, e in path:
        assert (c * CH + e, f) in bounds
