"""Python binding of libdmx's C-ABI (include/dmx.h) via ctypes.

Mirrors the reference's public API names (deflate::compress / inflate::decompress /
inflate::decompressZlib, /root/reference/include/deflate.hpp:755-815, inflate.hpp:326-408)
so tests read like the reference's own; errors raise ``DmxError`` (a ``RuntimeError``, as the
reference throws ``std::runtime_error``).  The HIP library is mandatory: there is no CPU
fallback, an import without ``lib/libdmx.so`` fails loudly.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DMX_LIB: developer override (A/B runs of two builds); the default is the in-tree build
LIB_PATH = os.environ.get("DMX_LIB") or os.path.join(HERE, "lib", "libdmx.so")

DMX_OK = 0
DMX_ERR_ARG = -1
DMX_ERR_NOMEM = -2
DMX_ERR_DEVICE = -3
DMX_ERR_DATA = -4
DMX_ERR_OVERREAD = -5
DMX_ERR_CAPACITY = -6
DMX_ERR_CHECKSUM = -8
DMX_CFG_RFC_STRICT = 1
DMX_CFG_FB_SERIAL = 2
DMX_VERIFY = 1
DMX_DEFLATE_NOT_FINAL = 1

CORPUS = {"zeros": 0, "repeat": 1, "random": 2, "text": 3, "mixed": 4, "bmp": 5}

# every symbol include/dmx.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "dmx_config_default", "dmx_create", "dmx_destroy", "dmx_default_ctx", "dmx_deflate_bound",
    "dmx_deflate", "dmx_inflate", "dmx_inflate_alloc", "dmx_free", "dmx_strerror",
    "dmx_deflate_device", "dmx_inflate_device", "dmx_set_timing", "dmx_last_stats",
    "dmx_corpus_generate", "dmx_adler32_device", "dmx_crc32_device", "dmx_adler32", "dmx_crc32",
    "dmx_framed_bound", "dmx_deflate_zlib", "dmx_deflate_gzip", "dmx_inflate_zlib", "dmx_inflate_gzip",
    "dmx_deflate_file", "dmx_inflate_file", "dmx_segment_starts_device", "dmx_inflate_piece_device",
    "dmx_segment_check_device", "dmx_set_default_config", "dmx_deflate_device_async",
    "dmx_inflate_device_async",
]


class DmxError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


class Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("segment_bytes", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("n_gpus", ctypes.c_uint32), ("dev_inflate_pass", ctypes.c_uint32),
                ("dev_heavy_bytes", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("ms_main_kernel", ctypes.c_double), ("ms_device_total", ctypes.c_double),
                ("segments", ctypes.c_uint64), ("in_bytes", ctypes.c_uint64),
                ("out_bytes", ctypes.c_uint64), ("path", ctypes.c_uint32), ("shards", ctypes.c_uint32)]


_lib = None


def lib():
    """Load libdmx.so (raises OSError when the HIP library has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # share torch's HIP runtime (same SONAME libamdhip64.so.7) instead of loading a second
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} missing: build it with `make -C deflate.hpp_amd` "
                      "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    sz = ctypes.c_size_t
    vp = ctypes.c_void_p
    u8p = ctypes.POINTER(ctypes.c_uint8)
    L.dmx_config_default.argtypes = [ctypes.POINTER(Config)]
    L.dmx_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(Config)]
    L.dmx_destroy.argtypes = [vp]
    L.dmx_default_ctx.restype = vp
    L.dmx_deflate_bound.argtypes = [sz]
    L.dmx_deflate_bound.restype = sz
    L.dmx_deflate.argtypes = [vp, vp, sz, ctypes.c_int, vp, sz, ctypes.POINTER(sz)]
    L.dmx_inflate.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.dmx_inflate_alloc.argtypes = [vp, vp, sz, ctypes.POINTER(u8p), ctypes.POINTER(sz)]
    L.dmx_free.argtypes = [vp]
    L.dmx_strerror.argtypes = [ctypes.c_int]
    L.dmx_strerror.restype = ctypes.c_char_p
    L.dmx_deflate_device.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_uint32, vp, sz, ctypes.POINTER(sz), vp]
    L.dmx_deflate_device_async.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_uint32, vp, sz, vp, vp]
    L.dmx_set_default_config.argtypes = [ctypes.POINTER(Config)]
    L.dmx_inflate_device.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(sz), vp]
    L.dmx_inflate_device_async.argtypes = [vp, vp, sz, vp, sz, vp, ctypes.c_uint32, vp]
    L.dmx_set_timing.argtypes = [vp, ctypes.c_int]
    L.dmx_last_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    L.dmx_corpus_generate.argtypes = [ctypes.c_int, ctypes.c_uint64, sz, vp]
    u32p = ctypes.POINTER(ctypes.c_uint32)
    for f in ("dmx_adler32_device", "dmx_crc32_device"):
        getattr(L, f).argtypes = [vp, vp, sz, ctypes.c_uint32, u32p, vp]
    for f in ("dmx_adler32", "dmx_crc32"):
        getattr(L, f).argtypes = [vp, vp, sz, ctypes.c_uint32, u32p]
    L.dmx_deflate_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(sz),
                                   ctypes.POINTER(sz)]
    L.dmx_inflate_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(sz)]
    L.dmx_segment_starts_device.argtypes = [vp, vp, sz, ctypes.POINTER(ctypes.c_uint64), sz, ctypes.POINTER(sz), vp]
    L.dmx_inflate_piece_device.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(sz), vp]
    L.dmx_segment_check_device.argtypes = [vp, vp, sz, ctypes.POINTER(ctypes.c_uint64), sz,
                                           ctypes.POINTER(ctypes.c_uint64), vp]
    L.dmx_framed_bound.argtypes = [sz]
    L.dmx_framed_bound.restype = sz
    for f in ("dmx_deflate_zlib", "dmx_deflate_gzip"):
        getattr(L, f).argtypes = [vp, vp, sz, ctypes.c_int, vp, sz, ctypes.POINTER(sz)]
    for f in ("dmx_inflate_zlib", "dmx_inflate_gzip"):
        getattr(L, f).argtypes = [vp, vp, sz, ctypes.c_uint32, ctypes.POINTER(u8p), ctypes.POINTER(sz)]
    _lib = L
    return L


def strerror(code):
    try:
        return lib().dmx_strerror(code).decode()
    except OSError:
        return f"error {code}"


def _check(rc, what):
    if rc != DMX_OK:
        raise DmxError(rc, what)


def deflate_bound(n):
    return lib().dmx_deflate_bound(n)


def corpus(kind, n, offset=0):
    """Synthetic corpus bytes [offset, offset+n)."""
    buf = ctypes.create_string_buffer(max(1, n))
    _check(lib().dmx_corpus_generate(CORPUS[kind], offset, n, buf), "corpus")
    return buf.raw[:n]


def corpus_into(kind, n, ptr, offset=0):
    _check(lib().dmx_corpus_generate(CORPUS[kind], offset, n, ctypes.c_void_p(ptr)), "corpus")


class Context:
    """A libdmx context bound to one HIP device (dmx_create / dmx_destroy)."""

    def __init__(self, device=-1, segment_bytes=32768, rfc_strict=False, n_gpus=1, **dev):
        """dev: developer A/B controls -- inflate_pass=k forces pass k of the segmented inflate
        plan, heavy_bytes=b sets the lane decoder's heavy-candidate threshold, fb_serial=True
        makes the block-parallel path decode every unit with one wavefront."""
        cfg = Config()
        lib().dmx_config_default(ctypes.byref(cfg))
        cfg.device = device
        cfg.segment_bytes = segment_bytes
        cfg.flags = DMX_CFG_RFC_STRICT if rfc_strict else 0
        cfg.n_gpus = n_gpus
        if dev.get("fb_serial"):
            cfg.flags |= DMX_CFG_FB_SERIAL
        if dev.get("inflate_pass") is not None:
            cfg.dev_inflate_pass = int(dev["inflate_pass"]) + 1
        cfg.dev_heavy_bytes = int(dev.get("heavy_bytes") or 0)
        h = ctypes.c_void_p()
        _check(lib().dmx_create(ctypes.byref(h), ctypes.byref(cfg)), "dmx_create")
        self.h = h

    def close(self):
        if self.h:
            lib().dmx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host-buffer API: the reference's signatures -------------------------------------
    def compress(self, data, level=2):
        """deflate::compress(char*, size_t, int) -> raw DEFLATE bytes."""
        data = bytes(data)
        cap = deflate_bound(len(data))
        out = ctypes.create_string_buffer(max(1, cap))
        n = ctypes.c_size_t()
        _check(lib().dmx_deflate(self.h, data, len(data), level, out, cap, ctypes.byref(n)), "deflate")
        return out.raw[: n.value]

    def compress_raw_not_final(self, data, level=2):
        """One shard of a larger stream (DMX_DEFLATE_NOT_FINAL: no BFINAL, ends byte-aligned on
        an empty stored block), through the device API."""
        import torch
        data = bytes(data)
        d_in = torch.frombuffer(bytearray(data or b"\0"), dtype=torch.uint8).cuda()
        cap = deflate_bound(len(data)) + 64
        d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        n = self.deflate_device(d_in.data_ptr(), len(data), level, d_out.data_ptr(), cap, not_final=True)
        torch.cuda.synchronize()
        return d_out[:n].cpu().numpy().tobytes()

    def decompress(self, data, cap=None):
        """inflate::decompress(void*, size_t) -> bytes; with cap: the (void*,size_t,void*,size_t)
        overload (returns at most cap bytes)."""
        data = bytes(data)
        if cap is None:
            p = ctypes.POINTER(ctypes.c_uint8)()
            n = ctypes.c_size_t()
            _check(lib().dmx_inflate_alloc(self.h, data, len(data), ctypes.byref(p), ctypes.byref(n)), "inflate")
            try:
                return ctypes.string_at(p, n.value)
            finally:
                lib().dmx_free(p)
        out = ctypes.create_string_buffer(max(1, cap))
        w = ctypes.c_size_t()
        tot = ctypes.c_size_t()
        _check(lib().dmx_inflate(self.h, data, len(data), out, cap, ctypes.byref(w), ctypes.byref(tot)), "inflate")
        return out.raw[: w.value]

    def decompress_zlib(self, data):
        """inflate::decompressZlib(void*, size_t): skips the 2-byte zlib header (the reference's
        FDICT test never fires, inflate.hpp:355, SURVEY A-9) and ignores the Adler-32."""
        data = bytes(data)
        if len(data) < 2:
            raise DmxError(DMX_ERR_OVERREAD, "inflate_zlib")
        return self.decompress(data[2:])

    # ---- file-path overloads (streaming, deflate.hpp:755-777 / inflate.hpp:390-408) ------
    def compress_file(self, in_path, out_path, level=2):
        """deflate::compress(std::string, std::string, int); returns (input, output) sizes."""
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib().dmx_deflate_file(self.h, os.fsencode(in_path), os.fsencode(out_path), level,
                                      ctypes.byref(a), ctypes.byref(b)), "deflate_file")
        return a.value, b.value

    def decompress_file(self, in_path, out_path):
        """inflate::decompress(std::string, std::string); returns the decoded size."""
        n = ctypes.c_size_t()
        _check(lib().dmx_inflate_file(self.h, os.fsencode(in_path), os.fsencode(out_path), ctypes.byref(n)),
               "inflate_file")
        return n.value

    # ---- containers and checksums (extensions, not in the reference) -----
    def _framed(self, fn, data, level):
        data = bytes(data)
        cap = lib().dmx_framed_bound(len(data))
        out = ctypes.create_string_buffer(max(1, cap))
        n = ctypes.c_size_t()
        _check(getattr(lib(), fn)(self.h, data, len(data), level, out, cap, ctypes.byref(n)), fn)
        return out.raw[: n.value]

    def compress_zlib(self, data, level=2):
        """RFC 1950 zlib stream (Adler-32 computed on the GPU)."""
        return self._framed("dmx_deflate_zlib", data, level)

    def compress_gzip(self, data, level=2):
        """RFC 1952 gzip member (CRC-32 computed on the GPU)."""
        return self._framed("dmx_deflate_gzip", data, level)

    def _unframed(self, fn, data, verify):
        data = bytes(data)
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _check(getattr(lib(), fn)(self.h, data, len(data), DMX_VERIFY if verify else 0, ctypes.byref(p),
                                  ctypes.byref(n)), fn)
        try:
            return ctypes.string_at(p, n.value)
        finally:
            lib().dmx_free(p)

    def inflate_zlib(self, data, verify=True):
        """zlib stream -> bytes; header checked, Adler-32 verified on the GPU (DMX_ERR_CHECKSUM)."""
        return self._unframed("dmx_inflate_zlib", data, verify)

    def inflate_gzip(self, data, verify=True):
        """gzip member -> bytes; CRC-32 and ISIZE verified on the GPU."""
        return self._unframed("dmx_inflate_gzip", data, verify)

    def _ck(self, fn, data, init):
        data = bytes(data)
        v = ctypes.c_uint32()
        _check(getattr(lib(), fn)(self.h, data, len(data), init, ctypes.byref(v)), fn)
        return v.value

    def adler32(self, data, init=1):
        return self._ck("dmx_adler32", data, init)

    def crc32(self, data, init=0):
        return self._ck("dmx_crc32", data, init)

    def adler32_device(self, d, n, init=1, stream=None):
        v = ctypes.c_uint32()
        _check(lib().dmx_adler32_device(self.h, ctypes.c_void_p(d), n, init, ctypes.byref(v),
                                        ctypes.c_void_p(stream) if stream else None), "adler32_device")
        return v.value

    def crc32_device(self, d, n, init=0, stream=None):
        v = ctypes.c_uint32()
        _check(lib().dmx_crc32_device(self.h, ctypes.c_void_p(d), n, init, ctypes.byref(v),
                                      ctypes.c_void_p(stream) if stream else None), "crc32_device")
        return v.value

    # ---- device-resident API --------------------------------------------------------------
    def deflate_device(self, d_in, n, level, d_out, cap, stream=None, not_final=False):
        out_len = ctypes.c_size_t()
        rc = lib().dmx_deflate_device(self.h, ctypes.c_void_p(d_in), n, level,
                                      DMX_DEFLATE_NOT_FINAL if not_final else 0,
                                      ctypes.c_void_p(d_out), cap, ctypes.byref(out_len),
                                      ctypes.c_void_p(stream) if stream else None)
        _check(rc, "deflate_device")
        return out_len.value

    def deflate_device_async(self, d_in, n, level, d_out, cap, d_len, stream=None, not_final=False):
        """Enqueue a device deflate; the stream length lands in the 8-byte device buffer d_len."""
        rc = lib().dmx_deflate_device_async(self.h, ctypes.c_void_p(d_in), n, level,
                                            DMX_DEFLATE_NOT_FINAL if not_final else 0,
                                            ctypes.c_void_p(d_out), cap, ctypes.c_void_p(d_len),
                                            ctypes.c_void_p(stream) if stream else None)
        _check(rc, "deflate_device_async")

    def inflate_device(self, d_in, n, d_out, cap, stream=None):
        out_len = ctypes.c_size_t()
        rc = lib().dmx_inflate_device(self.h, ctypes.c_void_p(d_in), n, ctypes.c_void_p(d_out), cap,
                                      ctypes.byref(out_len), ctypes.c_void_p(stream) if stream else None)
        _check(rc, "inflate_device")
        return out_len.value

    def inflate_device_async(self, d_in, n, d_out, cap, d_result, stream=None, piece=False):
        """Enqueue the lane-path inflate of a libdmx-layout stream; d_result (16 device bytes)
        receives {decoded bytes, status}; status 1: decode it with inflate_device instead."""
        rc = lib().dmx_inflate_device_async(self.h, ctypes.c_void_p(d_in), n, ctypes.c_void_p(d_out), cap,
                                            ctypes.c_void_p(d_result), 1 if piece else 0,
                                            ctypes.c_void_p(stream) if stream else None)
        _check(rc, "inflate_device_async")

    def inflate_piece_device(self, d_in, n, d_out, cap, stream=None):
        """inflate_device for one piece of a larger stream: a reference before the piece start
        raises (DMX_ERR_DATA) instead of copying nothing (multi-GPU scatter, shard.py)."""
        out_len = ctypes.c_size_t()
        rc = lib().dmx_inflate_piece_device(self.h, ctypes.c_void_p(d_in), n, ctypes.c_void_p(d_out), cap,
                                            ctypes.byref(out_len), ctypes.c_void_p(stream) if stream else None)
        _check(rc, "inflate_piece_device")
        return out_len.value

    def segment_check_device(self, d_in, n, starts, stream=None):
        """End byte of the segment at each start (None where it does not decode in piece mode)."""
        k = len(starts)
        if not k:
            return []
        a = (ctypes.c_uint64 * k)(*starts)
        e = (ctypes.c_uint64 * k)()
        _check(lib().dmx_segment_check_device(self.h, ctypes.c_void_p(d_in), n, a, k, e,
                                              ctypes.c_void_p(stream) if stream else None), "segment_check")
        return [None if x == 0xFFFFFFFFFFFFFFFF else x for x in e]

    def segment_starts_device(self, d_in, n, stream=None):
        """Candidate segment starts (bytes after each 00 00 FF FF) of a device-resident stream."""
        cnt = ctypes.c_size_t()
        sp = ctypes.c_void_p(stream) if stream else None
        _check(lib().dmx_segment_starts_device(self.h, ctypes.c_void_p(d_in), n, None, 0, ctypes.byref(cnt), sp),
               "segment_starts")
        buf = (ctypes.c_uint64 * max(1, cnt.value))()
        _check(lib().dmx_segment_starts_device(self.h, ctypes.c_void_p(d_in), n, buf, cnt.value, ctypes.byref(cnt),
                                               sp), "segment_starts")
        return list(buf[: cnt.value])

    def set_timing(self, on=True):
        _check(lib().dmx_set_timing(self.h, 1 if on else 0), "set_timing")

    def stats(self):
        s = Stats()
        _check(lib().dmx_last_stats(self.h, ctypes.byref(s)), "stats")
        return s


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context()
    return _default


def compress(data, level=2):
    return default_context().compress(data, level)


def decompress(data, cap=None):
    return default_context().decompress(data, cap)


def decompress_zlib(data):
    return default_context().decompress_zlib(data)
