"""ctypes bindings for the test-side checkers under oracle/ (TEST INFRASTRUCTURE ONLY).

- ``Oracle``: oracle/liboracle.so, the plain-C restatement of the reference inflate.
- ``Reference``: oracle/_ref/libdeflate_ref.so, the real reference headers compiled in place
  (present when the reference was available at build time; optional on the GPU box).
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libdeflate_ref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)


class CheckerError(Exception):
    def __init__(self, code):
        super().__init__(f"checker returned error {code}")
        self.code = code


def _buf(data):
    data = bytes(data)
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0"), len(data)


class Oracle:
    RFC = 1
    PIECE = 2

    def __init__(self, path=ORACLE_SO):
        self.lib = ctypes.CDLL(path)
        self.lib.oracle_inflate.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint32,
                                            ctypes.POINTER(_u8p), ctypes.POINTER(ctypes.c_size_t)]
        self.lib.oracle_inflate.restype = ctypes.c_int
        self.lib.oracle_inflate2.argtypes = self.lib.oracle_inflate.argtypes + [ctypes.POINTER(ctypes.c_size_t)]
        self.lib.oracle_inflate2.restype = ctypes.c_int
        self.lib.oracle_free.argtypes = [ctypes.c_void_p]

    def inflate(self, data, rfc=False, piece=False):
        b, n = _buf(data)
        out = _u8p()
        ln = ctypes.c_size_t()
        fl = (self.RFC if rfc else 0) | (self.PIECE if piece else 0)
        rc = self.lib.oracle_inflate(b, n, fl, ctypes.byref(out), ctypes.byref(ln))
        if rc != 0:
            raise CheckerError(rc)
        try:
            return ctypes.string_at(out, ln.value)
        finally:
            self.lib.oracle_free(out)


    def inflate_consumed(self, data, piece=False):
        """(decoded bytes, input bytes consumed up to the end of the final block)."""
        b, n = _buf(data)
        out = _u8p()
        ln = ctypes.c_size_t()
        used = ctypes.c_size_t()
        rc = self.lib.oracle_inflate2(b, n, self.PIECE if piece else 0, ctypes.byref(out), ctypes.byref(ln),
                                      ctypes.byref(used))
        if rc != 0:
            raise CheckerError(rc)
        try:
            return ctypes.string_at(out, ln.value), used.value
        finally:
            self.lib.oracle_free(out)


class Reference:
    def __init__(self, path=REF_SO):
        self.lib = ctypes.CDLL(path)
        L = self.lib
        L.ref_compress.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_u8p),
                                   ctypes.POINTER(ctypes.c_size_t)]
        L.ref_decompress.argtypes = [_u8p, ctypes.c_size_t, ctypes.POINTER(_u8p),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.ref_decompress_zlib.argtypes = L.ref_decompress.argtypes
        L.ref_decompress_cap.argtypes = [_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.ref_free.argtypes = [ctypes.c_void_p]

    @staticmethod
    def available():
        return os.path.exists(REF_SO)

    def _call(self, fn, data, *extra):
        b, n = _buf(data)
        out = _u8p()
        ln = ctypes.c_size_t()
        rc = fn(b, n, *extra, ctypes.byref(out), ctypes.byref(ln))
        if rc != 0:
            raise CheckerError(rc)
        try:
            return ctypes.string_at(out, ln.value)
        finally:
            self.lib.ref_free(out)

    def compress(self, data, level):
        return self._call(self.lib.ref_compress, data, level)

    def decompress(self, data):
        return self._call(self.lib.ref_decompress, data)

    def decompress_zlib(self, data):
        return self._call(self.lib.ref_decompress_zlib, data)

    def decompress_cap(self, data, cap):
        b, n = _buf(data)
        out = (ctypes.c_uint8 * max(1, cap))()
        w = ctypes.c_size_t()
        rc = self.lib.ref_decompress_cap(b, n, out, cap, ctypes.byref(w))
        if rc != 0:
            raise CheckerError(rc)
        return bytes(out)[: w.value]
