// include/deflate.hpp -- drop-in replacement for HyperBitGore/deflate.hpp's `deflate` class.
//
// Same class name and static signatures as the reference (deflate.hpp:755-815); the work runs
// on an MI355X through libdmx's C-ABI (include/dmx.h).  Link with -ldmx
// (deflate.hpp_amd/lib/libdmx.so).  Output is raw DEFLATE (RFC 1951) that the reference
// inflate::decompress round-trips exactly.
//
// Level semantics follow the reference's switch (deflate.hpp:699-717): 0 stored blocks,
// 1 Huffman only, 2 fast (greedy hash match), 3 slow (lazy match); any other value, including
// a `bool true` from the README's API, behaves like 1 -- which is what the reference does.
// Errors (no usable GPU, out of memory) throw std::runtime_error.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "dmx.h"

class deflate {
   public:
    // deflate::compress(char*, size_t, int)  -- reference deflate.hpp:779-796
    static std::vector<uint8_t> compress(char* data, size_t data_size, int compression_level) {
        return run(reinterpret_cast<const uint8_t*>(data), data_size, compression_level);
    }

    // deflate::compress(std::vector<uint8_t>&, int)  -- reference deflate.hpp:798-815
    static std::vector<uint8_t> compress(std::vector<uint8_t>& data, int compression_level) {
        return run(data.data(), data.size(), compression_level);
    }

    // deflate::compress(std::string, std::string, int)  -- reference deflate.hpp:755-777.
    // Streams the file through the GPU in 64 MiB chunks (dmx_deflate_file); returns 0 as the
    // reference does (its out_size is never updated, deflate.hpp:760, 776).
    static size_t compress(std::string file_path, std::string new_file, int compression_level) {
        int rc = dmx_deflate_file(dmx_default_ctx(), file_path.c_str(), new_file.c_str(), compression_level,
                                  nullptr, nullptr);
        if (rc != DMX_OK) throw std::runtime_error(dmx_strerror(rc));
        return 0;
    }

   private:
    static std::vector<uint8_t> run(const uint8_t* data, size_t n, int level) {
        std::vector<uint8_t> out(dmx_deflate_bound(n));
        size_t len = 0;
        int rc = dmx_deflate(dmx_default_ctx(), data, n, level, out.data(), out.size(), &len);
        if (rc != DMX_OK) throw std::runtime_error(dmx_strerror(rc));
        out.resize(len);
        return out;
    }
};
