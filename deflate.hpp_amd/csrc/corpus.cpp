// corpus.cpp -- deterministic synthetic corpora (spec v1) used by
// bench.py and the tests as stand-ins for the reference's fixtures (large.bmp is missing
// from the reference snapshot, .MISSING_LARGE_BLOBS:1). Host-only; exported via the C-ABI
// as dmx_corpus_generate().  Every generator is prefix-stable, so any window
// [offset, offset + n) of a corpus can be produced independently.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dmx.h"

namespace {

inline uint64_t sm(uint64_t& s) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// bytestream(seed)[off, off+n): output word w is sm() after w+1 increments of the seed.
void bytestream(uint64_t seed, uint64_t off, size_t n, uint8_t* out) {
    uint64_t w = off / 8;
    unsigned skip = (unsigned)(off % 8);
    uint64_t s = seed + w * 0x9E3779B97F4A7C15ull;
    size_t i = 0;
    while (i < n) {
        uint64_t v = sm(s);
        for (unsigned b = skip; b < 8 && i < n; b++) out[i++] = (uint8_t)(v >> (8 * b));
        skip = 0;
    }
}

void gen_zeros(uint64_t, size_t n, uint8_t* out) { std::memset(out, 0, n); }

void gen_repeat(uint64_t off, size_t n, uint8_t* out) {
    uint8_t p[256];
    bytestream(0x5EED0001ull, 0, 251, p);
    uint64_t k = off % 251;
    for (size_t i = 0; i < n; i++) {
        out[i] = p[k];
        if (++k == 251) k = 0;
    }
}

void gen_random(uint64_t off, size_t n, uint8_t* out) { bytestream(0x5EED0002ull, off, n, out); }

struct TextGen {
    std::vector<std::string> vocab;
    TextGen() {
        uint64_t sv = 0x5EED0003ull;
        vocab.resize(4096);
        for (int w = 0; w < 4096; w++) {
            unsigned len = 1 + (unsigned)(sm(sv) % 10);
            std::string s;
            for (unsigned j = 0; j < len; j++) s.push_back((char)('a' + sm(sv) % 26));
            vocab[w] = s;
        }
    }
    // Stream text from position 0, copying only [off, off+n).  The word stream is sequential
    // (variable-length words), so a per-thread cursor remembers where the last call stopped:
    // ascending windows (the mixed corpus takes text slices in offset order, a bench rank
    // takes its shard) resume there instead of regenerating the prefix, and words before
    // `off` are skipped without touching bytes.
    struct Cursor {
        uint64_t st = 0x5EED0004ull, pos = 0;
    };
    void gen(uint64_t off, size_t n, uint8_t* out) const {
        thread_local Cursor cur;
        Cursor c = cur.pos <= off ? cur : Cursor{};
        const uint64_t end = off + n;
        for (;;) {  // skip whole words that end at or before off
            uint64_t s = c.st;
            const uint64_t r = sm(s);
            const unsigned k = (unsigned)(r % 13);
            const uint64_t L = vocab[(r >> 8) & ((1ull << k) - 1)].size() + 1;
            if (c.pos + L > off) break;
            c.st = s;
            c.pos += L;
        }
        cur = c;  // a word boundary at or before off
        uint64_t st = c.st, pos = c.pos;
        while (pos < end) {
            uint64_t r = sm(st);
            unsigned k = (unsigned)(r % 13);
            uint64_t rank = (r >> 8) & ((1ull << k) - 1);
            const std::string& w = vocab[rank];
            char sep = ((r >> 60) == 0) ? '\n' : ' ';
            uint64_t L = w.size() + 1;
            for (uint64_t j = 0; j < L; j++) {
                uint64_t p = pos + j;
                if (p >= off && p < end) out[p - off] = (uint8_t)(j < w.size() ? w[j] : sep);
            }
            if (pos + L <= end) { cur.st = st; cur.pos = pos + L; }
            pos += L;
        }
    }
};

void gen_text(uint64_t off, size_t n, uint8_t* out) {
    static const TextGen tg;
    tg.gen(off, n, out);
}

void gen_mixed(uint64_t off, size_t n, uint8_t* out) {
    // segment k (64 KiB) takes the same-offset slice of base corpus t(k)
    size_t i = 0;
    while (i < n) {
        uint64_t p = off + i;
        uint64_t k = p / 65536;
        uint64_t s = 0x5EED0005ull + k;
        unsigned t = (unsigned)(sm(s) % 10);
        size_t take = (size_t)std::min<uint64_t>(n - i, (k + 1) * 65536 - p);
        if (t <= 3) gen_text(p, take, out + i);
        else if (t <= 5) gen_zeros(p, take, out + i);
        else if (t <= 7) gen_repeat(p, take, out + i);
        else gen_random(p, take, out + i);
        i += take;
    }
}

void put32(uint8_t* h, int at, uint32_t v) {
    for (int b = 0; b < 4; b++) h[at + b] = (uint8_t)(v >> (8 * b));
}

void gen_bmp(uint64_t off, size_t n, uint8_t* out) {
    const uint32_t W = 4096, H = 2048;
    const uint64_t total = 138ull + 3ull * W * H;
    uint8_t hdr[138];
    std::memset(hdr, 0, sizeof hdr);
    hdr[0] = 'B';
    hdr[1] = 'M';
    put32(hdr, 2, (uint32_t)total);
    put32(hdr, 10, 138);
    put32(hdr, 14, 124);
    put32(hdr, 18, W);
    put32(hdr, 22, H);
    hdr[26] = 1;
    hdr[28] = 24;
    put32(hdr, 34, W * 3 * H);
    put32(hdr, 38, 2835);
    put32(hdr, 42, 2835);
    for (size_t i = 0; i < n; i++) {
        uint64_t p = off + i;
        if (p >= total) { out[i] = 0; continue; }
        if (p < 138) { out[i] = hdr[p]; continue; }
        uint64_t q = p - 138;
        uint64_t pix = q / 3;
        unsigned ch = (unsigned)(q % 3);
        uint32_t y = (uint32_t)(pix / W), x = (uint32_t)(pix % W);
        uint64_t s = 0x5EED0006ull + (x >> 7) + (uint64_t)(y >> 7) * 64;
        uint64_t c = sm(s);
        uint8_t v;
        if ((c & 3) != 0) {
            v = (uint8_t)(c >> (8 * (ch + 1)));
        } else {
            unsigned nz = 0;
            if (c & 4) {
                uint64_t s2 = 0x5EED0007ull + (uint64_t)y * W + x;
                nz = (unsigned)(sm(s2) & 7);
            }
            v = (uint8_t)(ch == 0 ? x + nz : ch == 1 ? y + nz : ((x + y) >> 4) + nz);
        }
        out[i] = v;
    }
}

}  // namespace

extern "C" int dmx_corpus_generate(int kind, uint64_t offset, size_t n, uint8_t* out) {
    if (!out && n) return DMX_ERR_ARG;
    switch (kind) {
        case DMX_CORPUS_ZEROS: gen_zeros(offset, n, out); break;
        case DMX_CORPUS_REPEAT: gen_repeat(offset, n, out); break;
        case DMX_CORPUS_RANDOM: gen_random(offset, n, out); break;
        case DMX_CORPUS_TEXT: gen_text(offset, n, out); break;
        case DMX_CORPUS_MIXED: gen_mixed(offset, n, out); break;
        case DMX_CORPUS_BMP: gen_bmp(offset, n, out); break;
        default: return DMX_ERR_ARG;
    }
    return DMX_OK;
}
