// corpus.cpp -- deterministic synthetic corpora (spec v1) used by
// bench.py and the tests as stand-ins for the reference's fixtures (large.bmp is missing
// from the reference snapshot, .MISSING_LARGE_BLOBS:1). Host-only; exported via the C-ABI
// as dmx_corpus_generate().  Every generator is prefix-stable, so any window
// [offset, offset + n) of a corpus can be produced independently.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include <cstdlib>

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

// Text: words drawn from a 4096-word vocabulary, each followed by ' ' or '\n'.  Word w takes
// the RNG value sm() of state seed + w * G (splitmix64 is counter-based), so only the byte
// positions are sequential: a prefix sum of word lengths.  A process-wide table keeps the byte
// position of every kBlk-th word; it grows on demand, block sums computed by several threads.
// A window [off, off + n) starts at the table entry below `off`, skips < kBlk words and writes
// its bytes; windows are independent, so large requests are cut into pieces made by threads.
struct TextGen {
    static constexpr uint64_t kSeed = 0x5EED0004ull, kG = 0x9E3779B97F4A7C15ull;
    static constexpr uint64_t kBlk = 4096;  // words per table entry (~27 KB of text)
    uint8_t len[4096];                      // word length 1..10
    uint8_t chars[4096][16];
    mutable std::mutex mu;
    mutable std::vector<uint64_t> bpos{0};  // bpos[b]: byte position of word b * kBlk
    TextGen() {
        uint64_t sv = 0x5EED0003ull;
        for (int w = 0; w < 4096; w++) {
            const unsigned L = 1 + (unsigned)(sm(sv) % 10);
            len[w] = (uint8_t)L;
            std::memset(chars[w], 0, 16);
            for (unsigned j = 0; j < L; j++) chars[w][j] = (uint8_t)('a' + sm(sv) % 26);
        }
    }
    // vocabulary rank of the word with RNG value r
    static inline uint64_t rank_of(uint64_t r) { return (r >> 8) & ((1ull << (unsigned)(r % 13)) - 1); }
    static inline uint64_t value(uint64_t w) {
        uint64_t s = kSeed + w * kG;
        return sm(s);
    }
    uint64_t block_bytes(uint64_t b) const {
        uint64_t t = 0;
        for (uint64_t w = b * kBlk; w < (b + 1) * kBlk; w++) t += len[rank_of(value(w))] + 1u;
        return t;
    }
    // the table entry (word index, byte position) at or below off; the table extended as needed
    void entry(uint64_t off, uint64_t* w, uint64_t* pos) const {
        std::lock_guard<std::mutex> g(mu);
        while (bpos.back() <= off) {
            const uint64_t b0 = bpos.size() - 1;
            const uint64_t need = (off - bpos.back()) / (kBlk * 5) + 1;  // words are >= 2 bytes
            const uint64_t nb = std::max<uint64_t>(64, std::min<uint64_t>(need, 1u << 16));
            std::vector<uint64_t> sums(nb);
            const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nt; t++)
                th.emplace_back([&, t] {
                    for (uint64_t i = t; i < nb; i += nt) sums[i] = block_bytes(b0 + i);
                });
            for (auto& x : th) x.join();
            for (uint64_t i = 0; i < nb; i++) bpos.push_back(bpos.back() + sums[i]);
        }
        const uint64_t b = (uint64_t)(std::upper_bound(bpos.begin(), bpos.end(), off) - bpos.begin()) - 1;
        *w = b * kBlk;
        *pos = bpos[b];
    }
    void gen(uint64_t off, size_t n, uint8_t* out) const {
        uint64_t w, pos;
        entry(off, &w, &pos);
        const uint64_t end = off + n;
        for (;;) {  // skip whole words that end at or before off
            const uint64_t L = len[rank_of(value(w))] + 1u;
            if (pos + L > off) break;
            pos += L;
            w++;
        }
        for (; pos < end; w++) {
            const uint64_t r = value(w);
            const uint64_t rank = rank_of(r);
            const uint8_t sep = ((r >> 60) == 0) ? '\n' : ' ';
            const uint64_t L = len[rank] + 1u;
            if (pos >= off && pos + 16 <= end) {  // whole word: one 16-byte copy, then the separator
                std::memcpy(out + (pos - off), chars[rank], 16);
                out[pos - off + L - 1] = sep;
            } else {
                for (uint64_t j = 0; j < L; j++) {
                    const uint64_t p = pos + j;
                    if (p >= off && p < end) out[p - off] = j + 1 < L ? chars[rank][j] : sep;
                }
            }
            pos += L;
        }
    }
};

const TextGen& text_gen() {
    static const TextGen tg;
    return tg;
}

void gen_text(uint64_t off, size_t n, uint8_t* out) { text_gen().gen(off, n, out); }

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

using GenFn = void (*)(uint64_t, size_t, uint8_t*);

GenFn gen_fn(int kind) {
    switch (kind) {
        case DMX_CORPUS_ZEROS: return gen_zeros;
        case DMX_CORPUS_REPEAT: return gen_repeat;
        case DMX_CORPUS_RANDOM: return gen_random;
        case DMX_CORPUS_TEXT: return gen_text;
        case DMX_CORPUS_MIXED: return gen_mixed;
        case DMX_CORPUS_BMP: return gen_bmp;
        default: return nullptr;
    }
}

}  // namespace

// Windows of at least 32 MiB are cut into pieces (multiples of 64 KiB) made by up to 16 threads
// (DMX_CORPUS_THREADS overrides); every generator is a function of the absolute offset, so the
// bytes do not depend on the split.
extern "C" int dmx_corpus_generate(int kind, uint64_t offset, size_t n, uint8_t* out) {
    if (!out && n) return DMX_ERR_ARG;
    const GenFn f = gen_fn(kind);
    if (!f) return DMX_ERR_ARG;
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("DMX_CORPUS_THREADS")) nt = std::max(1, std::atoi(e));
    if (n < (32u << 20) || nt == 1) {
        f(offset, n, out);
        return DMX_OK;
    }
    if (kind == DMX_CORPUS_TEXT || kind == DMX_CORPUS_MIXED) {  // the table first, by all threads
        uint64_t w, pos;
        text_gen().entry(offset + n, &w, &pos);
    }
    const uint64_t piece = ((n / nt + 65535) / 65536) * 65536;
    std::vector<std::thread> th;
    for (uint64_t b = 0; b < n; b += piece) {
        const size_t len = (size_t)std::min<uint64_t>(piece, n - b);
        th.emplace_back([=] { f(offset + b, len, out + b); });
    }
    for (auto& t : th) t.join();
    return DMX_OK;
}
