"""CPU-baseline worker for bench.py (TEST INFRASTRUCTURE: drives the reference checker only).

One process of the `nproc`-process reference baseline (SURVEY.md 8(d) "Timing method (CPU
reference)" (b)): it generates its disjoint slice [offset, offset + n) of the corpus, prints
"ready", waits for a line on stdin (the parent's start signal, so every worker's timed region
overlaps), then runs the reference deflate::compress(level) + inflate::decompress
(oracle/_ref/libdeflate_ref.so) and prints one JSON line with its own timings.  No torch, no GPU.

  python tests/cpu_ref_worker.py <kind> <offset> <n> <level>
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
CORPUS = {"zeros": 0, "repeat": 1, "random": 2, "text": 3, "mixed": 4, "bmp": 5}


def corpus(kind, offset, n):
    """dmx_corpus_generate (host-only code of libdmx; no HIP call is made)."""
    lib = ctypes.CDLL(os.path.join(ROOT, "deflate.hpp_amd", "lib", "libdmx.so"))
    lib.dmx_corpus_generate.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p]
    buf = ctypes.create_string_buffer(max(1, n))
    if lib.dmx_corpus_generate(CORPUS[kind], offset, n, buf) != 0:
        raise RuntimeError("corpus generation failed")
    return buf.raw[:n]


def main():
    kind, offset, n, level = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    from oracle_bind import Reference
    data = corpus(kind, offset, n)
    ref = Reference() if Reference.available() else None
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    if ref is not None:
        comp = ref.compress(data, level)
        t1 = time.perf_counter()
        try:
            ref.decompress(comp)
        except Exception:
            pass
        t2 = time.perf_counter()
        res = {"deflate_s": t1 - t0, "inflate_s": t2 - t1, "comp": len(comp), "kind": "reference"}
    else:
        res = {"error": "oracle/_ref absent"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
