// oracle/ref_wrap.cpp -- TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// A C-linkage shim around the *unmodified* reference headers, compiled in place from
// /root/reference/include by oracle/Makefile into oracle/_ref/libdeflate_ref.so.
// It lets tests/ (golden-vector generation, parity checks) and bench.py's cpu_baseline
// leg call the real reference:
//   deflate::compress(char*, size_t, int)          /root/reference/include/deflate.hpp:779
//   inflate::decompress(void*, size_t)             /root/reference/include/inflate.hpp:363
//   inflate::decompress(void*, size_t, void*, size_t)  inflate.hpp:338
//   inflate::decompressZlib(void*, size_t)         inflate.hpp:352
// No reference source is copied: the headers are #included from where they lie.
#include <deflate.hpp>
#include <inflate.hpp>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>

namespace {
// The reference prints "Code tree is over or under subscribed!" to std::cerr every time its
// Kraft check trips (common.hpp:398-402). Silence it while the shim runs.
struct CerrMute {
    std::ostringstream sink;
    std::streambuf* old;
    CerrMute() : old(std::cerr.rdbuf(sink.rdbuf())) {}
    ~CerrMute() { std::cerr.rdbuf(old); }
};

int to_heap(const std::vector<uint8_t>& v, uint8_t** out, size_t* out_len) {
    *out_len = v.size();
    *out = static_cast<uint8_t*>(std::malloc(v.size() ? v.size() : 1));
    if (!*out) return -2;
    if (!v.empty()) std::memcpy(*out, v.data(), v.size());
    return 0;
}

// The reference dereferences in[0] even for n == 0 (A-9). Give it one readable zero byte so
// the call is defined: it then throws "Reading bits beyond the alloted buffer size!".
const uint8_t* safe_ptr(const uint8_t* in, size_t n) {
    static const uint8_t zero[8] = {0};
    return (n == 0 || in == nullptr) ? zero : in;
}
}  // namespace

extern "C" {

// 0 = ok, -1 = the reference threw std::exception, -2 = allocation failure.
int ref_compress(const uint8_t* in, size_t n, int level, uint8_t** out, size_t* out_len) {
    CerrMute mute;
    try {
        std::vector<uint8_t> r = deflate::compress((char*)safe_ptr(in, n), n, level);
        return to_heap(r, out, out_len);
    } catch (const std::exception&) {
        return -1;
    }
}

int ref_decompress(const uint8_t* in, size_t n, uint8_t** out, size_t* out_len) {
    CerrMute mute;
    try {
        std::vector<uint8_t> r = inflate::decompress((void*)safe_ptr(in, n), n);
        return to_heap(r, out, out_len);
    } catch (const std::exception&) {
        return -1;
    }
}

// Pointer overload with a capacity: returns bytes copied (<= cap) through *written.
int ref_decompress_cap(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* written) {
    CerrMute mute;
    try {
        *written = inflate::decompress((void*)safe_ptr(in, n), n, (void*)out, cap);
        return 0;
    } catch (const std::exception&) {
        return -1;
    }
}

int ref_decompress_zlib(const uint8_t* in, size_t n, uint8_t** out, size_t* out_len) {
    CerrMute mute;
    if (n < 2) return -3;  // reference would read past the buffer / segfault (A-9)
    try {
        std::vector<uint8_t> r = inflate::decompressZlib((void*)in, n);
        return to_heap(r, out, out_len);
    } catch (const std::exception&) {
        return -1;
    }
}

void ref_free(void* p) { std::free(p); }

}  // extern "C"
