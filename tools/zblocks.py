"""Developer aid (not a test): list the blocks of a raw DEFLATE stream (bit offset, BTYPE,
BFINAL, output bytes), by a plain Python decode.  Used to see where path 5's unit chain breaks."""
import sys


class Bits:
    def __init__(self, b):
        self.b = bytes(b) + bytes(8)
        self.p = 0

    def get(self, n):
        i = self.p >> 3
        x = (int.from_bytes(self.b[i:i + 5], "little") >> (self.p & 7)) & ((1 << n) - 1)
        self.p += n
        return x


def canon(lens):
    codes, code, bl = {}, 0, [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lens):
        if l:
            codes[(l, nxt[l])] = s
            nxt[l] += 1
    return codes


def sym(br, codes):
    c = 0
    for l in range(1, 16):
        c = (c << 1) | br.get(1)
        if (l, c) in codes:
            return codes[(l, c)]
    raise ValueError("bad code")


LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
      4097, 6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
PERM = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def blocks(s):
    br = Bits(s)
    out = 0
    while True:
        start = br.p
        fin = br.get(1)
        bt = br.get(2)
        info = ""
        n0 = out
        if bt == 0:
            br.p = (br.p + 7) & ~7
            ln = br.get(16)
            br.get(16)
            br.p += 8 * ln
            out += ln
        else:
            if bt == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                hlit, hdist, hclen = br.get(5) + 257, br.get(5) + 1, br.get(4) + 4
                pl = [0] * 19
                for i in range(hclen):
                    pl[PERM[i]] = br.get(3)
                pc = canon(pl)
                lens = []
                while len(lens) < hlit + hdist:
                    x = sym(br, pc)
                    if x < 16:
                        lens.append(x)
                    elif x == 16:
                        lens += [lens[-1]] * (3 + br.get(2))
                    elif x == 17:
                        lens += [0] * (3 + br.get(3))
                    else:
                        lens += [0] * (11 + br.get(7))
                ll, dl = lens[:hlit], lens[hlit:]
                info = f"hlit={hlit} hdist={hdist} hclen={hclen} lastpl={pl[PERM[hclen - 1]]}"
            lc, dc = canon(ll), canon(dl)
            while True:
                x = sym(br, lc)
                if x < 256:
                    out += 1
                elif x == 256:
                    break
                else:
                    L = LB[x - 257] + br.get(LE[x - 257])
                    dsym = sym(br, dc)
                    br.get(DE[dsym])
                    out += L
        yield start, bt, fin, out - n0, info
        if fin:
            return


if __name__ == "__main__":
    data = open(sys.argv[1], "rb").read()
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
    for st, bt, fin, n, info in blocks(data):
        if lo <= st <= hi:
            print(st, bt, fin, n, info)
