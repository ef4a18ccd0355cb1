"""Developer probe (run on the GPU box): exercises deflate/inflate end to end and prints a
compact report.  Not collected by pytest (no test_ prefix)."""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deflate.hpp_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dmx  # noqa: E402
from oracle_bind import Oracle, CheckerError  # noqa: E402

o = Oracle()
c = dmx.Context()
GOLD = os.path.join(ROOT, "tests", "golden")


def raw(d, lvl=6, strat=0):
    z = zlib.compressobj(lvl, zlib.DEFLATED, -15, 9, strat)
    return z.compress(d) + z.flush()


cases = [("empty", b""), ("one", b"A"), ("abc", b"abcabcabcabcabc" * 3)]
for f in ("tiny.bmp", "test.bmp"):
    p = os.path.join(GOLD, f)
    if os.path.exists(p):
        cases.append((f, open(p, "rb").read()))
for k in ("zeros", "repeat", "text", "random", "mixed", "bmp"):
    cases.append((k + "1M", dmx.corpus(k, 1 << 20)))
cases.append(("text100k+7", dmx.corpus("text", 100007)))
fails = 0
for name, d in cases:
    for lvl in (0, 1, 2, 3):
        t0 = time.time()
        try:
            s = c.compress(d, lvl)
        except Exception as e:
            print(f"FAIL deflate {name} L{lvl}: {e}")
            fails += 1
            continue
        t1 = time.time()
        try:
            ref = o.inflate(s)
        except CheckerError as e:
            ref = e
        okz = None
        try:
            okz = zlib.decompressobj(-15).decompress(s) == d
        except Exception:
            okz = False
        try:
            g = c.decompress(s)
        except Exception as e:
            g = e
        t2 = time.time()
        st = c.stats()
        good = isinstance(ref, bytes) and ref == d and g == d and okz
        if not good:
            fails += 1
        print(f"{'ok  ' if good else 'FAIL'} {name:12s} L{lvl} n={len(d):8d} c={len(s):8d} "
              f"ratio={len(d)/max(1,len(s)):8.2f} oracle={'ok' if ref == d else ('ERR' if not isinstance(ref, bytes) else 'MISMATCH')} "
              f"zlib={okz} gpu_inflate={'ok' if g == d else repr(g)[:60]} path={st.path} "
              f"t_d={t1-t0:.3f}s t_i={t2-t1:.3f}s")
# foreign (zlib) streams -> serial path
for name, d in cases[:6]:
    for lvl, strat in ((1, 0), (6, 0), (9, 1), (6, 2), (6, 3)):
        s = raw(d, lvl, strat)
        try:
            g = c.decompress(s)
        except Exception as e:
            g = e
        good = g == d
        fails += 0 if good else 1
        print(f"{'ok  ' if good else 'FAIL'} zlib {name:10s} lvl={lvl} strat={strat} c={len(s)} path={c.stats().path} "
              f"{'' if good else repr(g)[:80]}")
for nm, h in [("B", "0d83050100000040b6f27f040237"), ("A", "0d83050100000040b6f27f84c40d"),
              ("C", "0d89250100000080b6c2ff1140100027")]:
    try:
        g = c.decompress(bytes.fromhex(h))
    except Exception as e:
        g = e
    print("crafted", nm, repr(g))
print("FAILS", fails)
