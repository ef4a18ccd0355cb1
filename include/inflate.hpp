// include/inflate.hpp -- drop-in replacement for HyperBitGore/deflate.hpp's `inflate` class.
//
// Same class name and static signatures as the reference (inflate.hpp:326-408); decoding runs
// on an MI355X through libdmx's C-ABI (include/dmx.h).  Link with -ldmx.
//
// Output is bit-exact to the reference on the same input, including its lenient behaviour
// (NLEN unchecked, BTYPE 3 = empty block, a distance beyond the output copies nothing,
// trailing bytes ignored; SURVEY A-10).  Where the reference throws
// std::runtime_error("Reading bits beyond the alloted buffer size!") this throws a
// std::runtime_error too.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "dmx.h"

class inflate {
   public:
    // inflate::decompress(void*, size_t, void*, size_t)  -- reference inflate.hpp:338-350:
    // decodes the whole stream, copies at most out_size bytes, returns the count copied.
    static size_t decompress(void* in, size_t in_size, void* out, size_t out_size) {
        size_t written = 0;
        int rc = dmx_inflate(dmx_default_ctx(), static_cast<const uint8_t*>(in), in_size,
                             static_cast<uint8_t*>(out), out_size, &written, nullptr);
        if (rc != DMX_OK) throw std::runtime_error(dmx_strerror(rc));
        return written;
    }

    // inflate::decompress(void*, size_t)  -- reference inflate.hpp:363-374
    static std::vector<uint8_t> decompress(void* in, size_t in_size) {
        return run(static_cast<const uint8_t*>(in), in_size);
    }

    // inflate::decompress(std::vector<uint8_t>)  -- reference inflate.hpp:376-387 (by value)
    static std::vector<uint8_t> decompress(std::vector<uint8_t> in) { return run(in.data(), in.size()); }

    // inflate::decompress(std::string, std::string)  -- reference inflate.hpp:390-408.
    // Streaming file decode (dmx_inflate_file); returns the decoded size (the reference's
    // running total equals this for the single-Huffman-block files it handles, SURVEY A-8).
    static size_t decompress(std::string file_path, std::string new_file) {
        size_t n = 0;
        int rc = dmx_inflate_file(dmx_default_ctx(), file_path.c_str(), new_file.c_str(), &n);
        if (rc != DMX_OK) throw std::runtime_error(dmx_strerror(rc));
        return n;
    }

    // inflate::decompressZlib(void*, size_t, void*, size_t)  -- reference inflate.hpp:326-335.
    // The reference always skips 2 header bytes (its FDICT test reads bit 26 of CMF+1, which is
    // always 0: SURVEY A-9) and never checks the Adler-32.
    static size_t decompressZlib(void* in, size_t in_size, void* out, size_t out_size) {
        if (in_size < 2) throw std::runtime_error(dmx_strerror(DMX_ERR_OVERREAD));
        return decompress(static_cast<uint8_t*>(in) + 2, in_size - 2, out, out_size);
    }

    // inflate::decompressZlib(void*, size_t)  -- reference inflate.hpp:352-361
    static std::vector<uint8_t> decompressZlib(void* in, size_t in_size) {
        if (in_size < 2) throw std::runtime_error(dmx_strerror(DMX_ERR_OVERREAD));
        return run(static_cast<const uint8_t*>(in) + 2, in_size - 2);
    }

   private:
    static std::vector<uint8_t> run(const uint8_t* in, size_t n) {
        uint8_t* p = nullptr;
        size_t len = 0;
        int rc = dmx_inflate_alloc(dmx_default_ctx(), in, n, &p, &len);
        if (rc != DMX_OK) throw std::runtime_error(dmx_strerror(rc));
        std::vector<uint8_t> v(p, p + len);
        dmx_free(p);
        return v;
    }
};
