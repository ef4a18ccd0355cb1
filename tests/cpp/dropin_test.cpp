// tests/cpp/dropin_test.cpp -- a C++ caller written against the reference's public API
// (deflate::compress / inflate::decompress / inflate::decompressZlib), compiled against the
// drop-in headers in include/ and linked to libdmx.so.  Mirrors the reference's own driver
// (test/libdeflate.cpp: round trips per level, decompressZlib on weird.dat, the file-path
// round trip, the pointer API with a capacity) but compares content, which the reference's
// driver does not.  Exit code 0 = all checks passed.
#include <deflate.hpp>
#include <inflate.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

static int fails = 0;
#define CHECK(c, msg)                                      \
    do {                                                   \
        if (!(c)) {                                        \
            std::fprintf(stderr, "[FAIL] %s\n", msg);      \
            fails++;                                       \
        } else {                                           \
            std::fprintf(stderr, "[PASS] %s\n", msg);      \
        }                                                  \
    } while (0)

static std::vector<uint8_t> slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "tests/golden";
    const std::string tmp = argc > 2 ? argv[2] : "/tmp";
    // argv[3] = N: the whole program runs with dmx_config.n_gpus = N behind the reference's API
    const int ngpus = argc > 3 ? std::atoi(argv[3]) : 1;
    if (ngpus > 1) {
        dmx_config cfg;
        dmx_config_default(&cfg);
        cfg.n_gpus = (uint32_t)ngpus;
        CHECK(dmx_set_default_config(&cfg) == DMX_OK, "dmx_set_default_config before first use");
        std::vector<uint8_t> big(6u << 20);
        for (size_t i = 0; i < big.size(); i++) big[i] = (uint8_t)((i * 2654435761u) >> 13) & 0x3F;
        std::vector<uint8_t> z = deflate::compress(big, 2);
        dmx_stats st{};
        dmx_last_stats(dmx_default_ctx(), &st);
        CHECK((int)st.shards == ngpus, "deflate::compress split over n_gpus shards");
        CHECK(inflate::decompress(z) == big, "n_gpus round trip through the reference API");
        dmx_last_stats(dmx_default_ctx(), &st);
        CHECK((int)st.shards == ngpus, "inflate::decompress split over n_gpus pieces");
        CHECK(dmx_set_default_config(&cfg) == DMX_ERR_ARG, "the default config is fixed once in use");
    }
    std::vector<uint8_t> bmp = slurp(dir + "/test.bmp");
    CHECK(bmp.size() == 21898, "test.bmp fixture present");
    for (int level = 0; level <= 3; level++) {
        std::vector<uint8_t> c1 = deflate::compress(reinterpret_cast<char*>(bmp.data()), bmp.size(), level);
        std::vector<uint8_t> c2 = deflate::compress(bmp, level);
        CHECK(c1 == c2, ("compress overloads agree, level " + std::to_string(level)).c_str());
        std::vector<uint8_t> d1 = inflate::decompress(c1.data(), c1.size());
        std::vector<uint8_t> d2 = inflate::decompress(c1);
        CHECK(d1 == bmp && d2 == bmp, ("round trip, level " + std::to_string(level)).c_str());
        std::vector<uint8_t> capbuf(1000);
        size_t w = inflate::decompress(c1.data(), c1.size(), capbuf.data(), capbuf.size());
        CHECK(w == 1000 && std::memcmp(capbuf.data(), bmp.data(), 1000) == 0, "pointer API copies <= cap");
    }
    // bool level from the README's API: true -> 1, false -> 0
    CHECK(inflate::decompress(deflate::compress(bmp, true)) == bmp, "bool level true");
    CHECK(inflate::decompress(deflate::compress(bmp, false)) == bmp, "bool level false");
    // decompressZlib on the reference's weird.dat (test/libdeflate.cpp:228-254)
    std::vector<uint8_t> weird = slurp(dir + "/weird.dat");
    std::vector<uint8_t> wz = inflate::decompressZlib(weird.data(), weird.size());
    CHECK(wz.size() == 6050, "decompressZlib(weird.dat) size 6050");
    std::vector<uint8_t> wbuf(6050);
    CHECK(inflate::decompressZlib(weird.data(), weird.size(), wbuf.data(), wbuf.size()) == 6050 && wbuf == wz,
          "decompressZlib pointer overload");
    // file-path round trip (test/libdeflate.cpp:290-296)
    deflate::compress(dir + "/test.bmp", tmp + "/dmx_test.deflate", 3);
    size_t fsz = inflate::decompress(tmp + "/dmx_test.deflate", tmp + "/dmx_test.out");
    CHECK(fsz == bmp.size() && slurp(tmp + "/dmx_test.out") == bmp, "file-path round trip");
    // truncated stream throws like the reference
    std::vector<uint8_t> c = deflate::compress(bmp, 2);
    bool threw = false;
    try {
        inflate::decompress(c.data(), c.size() / 2);
    } catch (const std::runtime_error&) {
        threw = true;
    }
    CHECK(threw, "truncated stream throws std::runtime_error");
    std::fprintf(stderr, "%s (%d failures)\n", fails ? "FAILED" : "ALL PASSED", fails);
    return fails ? 1 : 0;
}
