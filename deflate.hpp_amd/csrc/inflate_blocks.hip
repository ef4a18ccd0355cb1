// inflate_blocks.hip -- block-parallel inflate of ARBITRARY DEFLATE streams (gfx950).
//
// The segment-parallel paths (inflate_lanes.hip, inflate_kernels.hip) need byte-aligned
// independent segments behind "00 00 FF FF" markers, which zlib's, libdeflate's and the
// reference's own multi-chunk streams do not have: their blocks start at arbitrary bit offsets
// and copy from up to 32 KiB before the block.  The reference decodes such a stream with one
// block loop (realDecompress, /root/reference/include/inflate.hpp:277-322); this path splits it
// into units that decode side by side and stitches the windows together afterwards:
//
//   k_fb_scan    every bit offset of the stream is tested for a stored-block header (LEN, NLEN =
//                ~LEN at the next byte boundary, data inside the stream) and for a dynamic-block
//                header that a real encoder could have written: BTYPE 2, HLIT <= 29, HDIST <= 29, a complete
//                code-length code whose last sent length is nonzero, a code-length sequence
//                that decodes without overrun to a complete lit/len code with a nonzero
//                end-of-block length and a complete (or at most one-symbol) distance code.
//                One wavefront per 4 KiB of stream, one bit offset per lane.  Hits are block
//                starts with overwhelming probability (none false on the test corpora); a false
//                one only costs parallelism, because the chain check below discards it.
//   k_fb_decode  one wavefront per unit (unit k starts at the k-th hit; unit 0 at bit 0)
//                decodes whole blocks (stored / fixed / dynamic, the reference's lenient rules)
//                until the next unit's start or BFINAL, into a token list in HBM: literal runs,
//                (length, distance) matches, stored-data references.  A distance reaching
//                before the unit is kept as is: its bytes are not known yet.
//   host         walks the chain from bit 0 (each unit must end exactly where the next one on
//                the chain starts), sums the output sizes into offsets.
//   k_fb_replay  one wavefront per unit rebuilds its output from the tokens in a 32 Ki-entry
//                LDS ring of 16-bit values: bytes, or 0x8000 | (b - 1) for "the byte b
//                positions before the unit start" (copies propagate such markers), written to a
//                16-bit image of the output in HBM.
//   k_fb_tails   one workgroup walks the units in order with the last 32 KiB of output in LDS
//                and resolves the markers in each unit's last 32 KiB -- the only serial step,
//                32 KiB of gather work per unit.
//   k_fb_final   every other position of the image: byte, or the (already final) output byte
//                its marker names.  HBM-bound and fully parallel.
// Anything the chain check or the replay cannot vouch for (a unit that errors, over-reads, runs
// out of token space, or copies from before the stream start) sends the stream to the exact
// serial decoder instead, so results and error codes stay the reference's.
#include "inflate_common.h"


namespace dmx {

#ifndef DMX_FB_SCAN_BITS
#define DMX_FB_SCAN_BITS 16384
#endif
#ifndef DMX_FB_STEP
#define DMX_FB_STEP 2048
#endif
constexpr uint32_t FB_SCAN_BITS = DMX_FB_SCAN_BITS;  // bit offsets tested per wavefront (2 KiB of stream)
constexpr uint32_t FB_STEP = DMX_FB_STEP;            // offsets per prefilter step (32 per lane)
constexpr uint32_t FB_STAGE_WORDS = FB_SCAN_BITS / 32 + 128;  // + 4096 bits of header lookahead
constexpr uint32_t FB_HITS = 96;          // candidates kept per scan chunk (true headers -- zlib at
                                          // memLevel 1-2 writes blocks of a few hundred bytes -- and
                                          // ~17 per chunk that pass the precode test by chance)
constexpr uint32_t FB_RING = 32768;       // replay window (entries of 16 bits)
constexpr uint64_t FB_HIT_STORED = 1ull << 62;  // hit flag: a stored-block header
constexpr uint32_t FB_GROUP_MAX = 8192;   // output entries per replay group (see k_fb_replay)

// ---------------------------------------------------------------------------------------
// k_fb_scan
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fb_bits(const uint32_t* w, uint32_t p) {  // 32 bits at p
    const uint32_t i = p >> 5;
    return __builtin_amdgcn_alignbit(w[i + 1], w[i], p & 31);
}

// Full check of a candidate whose precode is complete (k_fb_check), resumable so that a lane
// can take the next candidate as soon as its own is decided.  RFC 1951 rules as zlib's inflate
// enforces them; A-11/A-12 streams are not block starts any real encoder writes, so rejecting
// them only costs parallelism.
// The code-length sequence, read through a 64-bit bit buffer refilled from the lane's staged
// column (word wi on; words past the column come from HBM).  step() decodes up to `steps`
// symbols, branch-free but for the refill; st becomes FBK_PASS (a complete lit/len code with a
// nonzero end-of-block length and a complete, or at most one-symbol, distance code) or
// FBK_FAIL.  plim: the bit count a header may take at most.
constexpr uint32_t FBK_RUN = 0, FBK_PASS = 1, FBK_FAIL = 2;
struct FbLengthCheck {
    uint64_t buf;
    uint32_t nb, wi, used, plim;
    uint32_t nlit, total, i, prev;
    uint32_t kl, kd, nd;  // Kraft sums in units of 2^-15, used distance codes
    bool eob;
    uint32_t st;
    // the precode: a 128-entry table (symbol | length << 5) in the lane's LDS column, indexed
    // by the next 7 stream bits in code order (first bit = MSB), so that each symbol's entries
    // are one contiguous range; entry c at byte 256 (c / 4) + c % 4 of the column
    __attribute__((address_space(3))) uint8_t* tab;
    // from the 19 precode lengths pl (3 bits each, by symbol) of a complete code (stage 1)
    __device__ void set_precode(uint64_t pl) {
        uint64_t cnt = 0;  // counts per length, 5-bit fields
        for (uint32_t s = 0; s < 19; s++) {
            const uint32_t l = (uint32_t)(pl >> (3 * s)) & 7;
            cnt += l ? 1ull << (5 * l) : 0ull;
        }
        uint64_t nxt = 0;  // the next code per length (8-bit fields)
        uint32_t code = 0;
        for (uint32_t l = 1; l <= 7; l++) {
            code = (code + (uint32_t)((cnt >> (5 * (l - 1))) & 31)) << 1;  // (no length-0 count)
            nxt |= (uint64_t)code << (8 * l);
        }
        for (uint32_t s = 0; s < 19; s++) {
            const uint32_t l = (uint32_t)(pl >> (3 * s)) & 7;
            if (!l) continue;
            const uint32_t c = (uint32_t)(nxt >> (8 * l)) & 0xFF;
            nxt += 1ull << (8 * l);
            const uint32_t e = s | (l << 5);
            const uint32_t c0 = c << (7 - l);  // entries [c0, c0 + 2^(7 - l))
            if (l <= 5) {
                for (uint32_t m = c0 >> 2; m < (c0 >> 2) + (1u << (5 - l)); m++)
                    *(__attribute__((address_space(3))) uint32_t*)(tab + 256 * m) = e * 0x01010101u;
            } else {
                tab[256 * (c0 >> 2) + (c0 & 3)] = (uint8_t)e;
                if (l == 6) tab[256 * (c0 >> 2) + (c0 & 3) + 1] = (uint8_t)e;
            }
        }
    }
    // the symbol and length of the code at the low bits of v
    __device__ __forceinline__ void decode(uint32_t v, uint32_t* sym, uint32_t* len) const {
        const uint32_t c7 = __builtin_bitreverse32(v) >> 25;
        const uint32_t e = tab[256 * (c7 >> 2) + (c7 & 3)];
        *sym = e & 31;
        *len = e >> 5;
    }
};

// One wavefront per FB_SCAN_BITS offsets, in two stages so that each test runs on full waves:
//   0. prefilter, 32 offsets per lane at once with 64-bit word arithmetic on the staged bits:
//      BTYPE 2, HLIT <= 29, HDIST <= 29 (~21 % of random offsets pass); byte-aligned offsets with
//      BTYPE 0 get the stored-header test (LEN / NLEN = ~LEN, data inside the stream) directly;
//   1. the survivors, queued in offset order, one per lane: a complete precode whose last sent
//      length is nonzero (~0.5 % pass).
// The chunk keeps its first FB_HITS candidates in offset order; k_fb_check then runs the full
// code-length test on all chunks' candidates at once, one per lane (round 4 ran it per chunk at
// the end of the scan: a few lanes of each wave busy for the longest test, and its per-lane
// tables limited the scan to two waves per SIMD).
// stage 1: HCLEN + 4 precode lengths (3 bits each, in the kPerm order) form a complete code
// and the last one sent is nonzero (zlib / libdeflate / libdmx send HCLEN up to the last nonzero
// length, >= 4).  x0, x1: the 64 bits from the first precode length on.
__device__ __forceinline__ bool fb_precode_ok(uint32_t h, uint32_t x0, uint32_t x1) {
    const uint32_t hclen = ((h >> 13) & 15) + 4;
    uint32_t kr = 0;
#pragma unroll
    for (uint32_t i = 0; i < 19; i++) {
        const uint32_t l = i < 10 ? (x0 >> (3 * i)) & 7 : i == 10 ? ((x0 >> 30) | (x1 << 2)) & 7 : (x1 >> (3 * i - 32)) & 7;
        kr += (i < hclen && l) ? 128u >> l : 0u;
    }
    const uint32_t bl = 3 * (hclen - 1);
    const uint32_t last = (uint32_t)((((uint64_t)x1 << 32) | x0) >> bl) & 7;
    return kr == 128 && (last != 0 || hclen == 4);
}
// the precode lengths by symbol (3 bits each)
__device__ __forceinline__ uint64_t fb_precode_lengths(uint32_t h, uint32_t x0, uint32_t x1) {
    const uint32_t hclen = ((h >> 13) & 15) + 4;
    const uint64_t x = (uint64_t)x0 | ((uint64_t)x1 << 32);
    uint64_t pl = 0;
    // kPerm as 5-bit fields in two registers (the table itself is a memory load per length)
    constexpr uint64_t kPermLo = 0x22caa324e804a30ull, kPermHi = 0x3c2e1346cull;
    for (uint32_t i = 0; i < hclen; i++) {
        const uint32_t sym = (uint32_t)((i < 12 ? kPermLo >> (5 * i) : kPermHi >> (5 * (i - 12))) & 31);
        pl |= ((x >> (3 * i)) & 7) << (3 * sym);
    }
    return pl;
}

__global__ __launch_bounds__(64) void k_fb_scan(const uint32_t* in_words, uint64_t misalign,
                                                 uint64_t n, uint32_t* counts, uint64_t* hits) {
    __shared__ uint32_t stg[FB_STAGE_WORDS + 2];
    __shared__ uint32_t q1[FB_STEP + 64];  // offsets r (bit 31: a stored-block hit)
    const uint32_t lane = threadIdx.x;
    const uint64_t c = blockIdx.x;
    // stage words of the aligned image: bit 0 of word 0 = stream bit b0 - sh
    const uint64_t b0 = c * FB_SCAN_BITS;                 // first stream bit tested
    const uint64_t abs0 = misalign * 8 + b0;              // same bit in the aligned image
    const uint64_t w0 = abs0 >> 5;
    const uint32_t sh = (uint32_t)(abs0 & 31);
    const uint64_t end_bytes = misalign + n;
    const uint64_t nwords = (end_bytes + 3) / 4;
    for (uint32_t i = lane; i < FB_STAGE_WORDS + 2; i += 64) {
        const uint64_t wi = w0 + i;
        uint32_t v = 0;
        if (wi < nwords) {
            v = in_words[wi];
            const uint64_t lim = end_bytes - 4 * wi;
            if (lim < 4) v &= (1u << (8 * lim)) - 1u;
        }
        stg[i] = v;
    }
    __syncthreads();
    const uint64_t nbits = 8 * n;
    uint32_t found = 0, n1 = 0;
    const uint64_t below = (1ull << lane) - 1ull;
    // stage 1 on q1[0, m): survivors to the chunk's candidates (in order); the rest of q1 moves down
    auto drain1 = [&](uint32_t m) {
        bool pass = false;
        uint32_t e = 0;
        if (lane < m) {
            e = q1[lane];
            if (e >> 31) {
                pass = true;
            } else {
                const uint32_t q = sh + e;
                pass = fb_precode_ok(fb_bits(stg, q), fb_bits(stg, q + 17), fb_bits(stg, q + 49));
            }
        }
        const uint64_t pm = __ballot(pass);
        const uint32_t before = __popcll(pm & below);
        if (pass && found + before < FB_HITS)
            hits[c * FB_HITS + found + before] = (b0 + (e & 0x7FFFFFFFu)) | ((e >> 31) ? FB_HIT_STORED : 0ull);
        found += __popcll(pm);
        const uint32_t rest = n1 - m;
        wave_sync();
        for (uint32_t i = lane; i < rest; i += 64) q1[i] = q1[m + i];  // (m = 64: no pass
                                                  // writes an entry that it or a later pass reads)
        wave_sync();
        n1 = rest;
    };
    for (uint32_t step = 0; step < FB_SCAN_BITS / FB_STEP && found < FB_HITS; step++) {
        const uint32_t o = step * FB_STEP + lane * 32;  // this lane's first offset (relative to b0)
        const uint32_t q = sh + o, i = q >> 5, k = q & 31;
        const uint32_t s0 = stg[i], s1 = stg[i + 1], s2 = stg[i + 2];
        const uint64_t v = (uint64_t)__builtin_amdgcn_alignbit(s1, s0, k) |
                           ((uint64_t)__builtin_amdgcn_alignbit(s2, s1, k) << 32);
        uint64_t m = ~(v >> 1) & (v >> 2);                     // BTYPE 2
        m &= ~((v >> 4) & (v >> 5) & (v >> 6) & (v >> 7));     // HLIT <= 29
        m &= ~((v >> 9) & (v >> 10) & (v >> 11) & (v >> 12));  // HDIST <= 29
        uint32_t dyn = (uint32_t)m;
        uint32_t sto = (uint32_t)(~(v >> 1) & ~(v >> 2)) & 0x01010101u;  // BTYPE 0, byte-aligned
        // offsets whose header would read past the stream end
        const uint64_t sb = b0 + o;
        const uint32_t nval = sb + 29 >= nbits ? 0u : (nbits - sb - 29 >= 32 ? 32u : (uint32_t)(nbits - sb - 29));
        const uint32_t vmask = nval >= 32 ? 0xFFFFFFFFu : ((1u << nval) - 1u);
        dyn &= vmask;
        sto &= vmask;
        // stored block at a byte boundary (where a stored block after another stored block
        // starts): LEN and NLEN = ~LEN at the next byte boundary, data inside the stream.  These
        // let runs of stored blocks (incompressible data) decode unit by unit.  A stored block
        // after a Huffman block starts at any bit; the unit before simply decodes it too (a
        // strong unit only stops on landing on a start or past its stop).  Only aligned offsets:
        // the offsets inside a header's zero padding and just before it all look like stored
        // headers, and would crowd the chunk's FB_HITS out.
        uint32_t sh_ok = 0;
        for (uint32_t t = sto; t; t &= t - 1) {
            const uint32_t bi = __builtin_ctz(t);
            const uint64_t bb = sb + bi + 8;  // stream bit of LEN
            if (bb + 32 <= nbits) {
                const uint32_t ln = fb_bits(stg, q + bi + 8);
                if (((ln ^ (ln >> 16)) & 0xFFFFu) == 0xFFFFu && bb / 8 + 4 + (ln & 0xFFFFu) <= n) sh_ok |= 1u << bi;
            }
        }
        const uint32_t all = dyn | sh_ok;
        const uint32_t cnt = __builtin_popcount(all);
        const uint32_t incl = wave_incl_scan(cnt);
        uint32_t pos = n1 + incl - cnt;
        for (uint32_t t = all; t; t &= t - 1) {
            const uint32_t bi = __builtin_ctz(t);
            q1[pos++] = (o + bi) | ((sh_ok >> bi) & 1u ? 0x80000000u : 0u);
        }
        n1 += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        wave_sync();
        while (n1 >= 64) drain1(64);
    }
    while (n1 && found < FB_HITS) drain1(n1 < 64 ? n1 : 64u);
    if (lane == 0) counts[c] = min(found, FB_HITS);
}

// stream bits from HBM (the aligned image; zero past the stream's last byte)
struct FbGlobalBits {
    const uint32_t* w;
    uint64_t nwords, end_bytes;
    __device__ uint32_t word(uint64_t i) const {
        if (i >= nwords) return 0u;
        uint32_t v = w[i];
        const uint64_t lim = end_bytes - 4 * i;
        if (lim < 4) v &= (1u << (8 * lim)) - 1u;
        return v;
    }
    __device__ uint32_t peek(uint64_t p) const {
        return __builtin_amdgcn_alignbit(word((p >> 5) + 1), word(p >> 5), (uint32_t)(p & 31));
    }
};

// The full test of the candidates k_fb_compact listed (stage 2): one per lane.  Each lane's
// first FBC_WORDS words from the candidate on are staged in LDS (a real header fits; a longer
// one reads on from HBM), and its precode table is an LDS column; both column-major, so the
// lanes of a wave read distinct banks.  A candidate that is not a dynamic-block header a real
// encoder could have written (fb_check_lengths) is marked FB_HIT_REJECT in place.
#ifndef DMX_FBC_PER_WAVE
#define DMX_FBC_PER_WAVE 64
#endif
constexpr uint32_t FBC_WORDS = 64;  // 2048 bits: the longest false candidates of a wave run ~1.2 Kbit
typedef __attribute__((address_space(3))) uint32_t FbcLdsU32;
typedef __attribute__((address_space(3))) uint8_t FbcLdsU8;
struct FbcBits {
    FbcLdsU32* col;  // staged word i at col[64 i]: aligned-image word w0 + i
    uint64_t b0;     // aligned-image bit of staged word 0
    FbGlobalBits g;
    __device__ uint32_t peek(uint64_t p) const {
        const uint64_t r = p - b0;
        if (r + 64 > 32 * FBC_WORDS) return g.peek(p);
        const uint32_t i = (uint32_t)(r >> 5);
        return __builtin_amdgcn_alignbit(col[64 * (i + 1)], col[64 * i], (uint32_t)(r & 31));
    }
};
// One lane per candidate, a wave per DMX_FBC_PER_WAVE candidates (its own range: a lane whose
// candidate is decided takes the range's next one once half the wave is idle, so a wave does
// not wait for its longest candidate -- the test runs 48 symbols on average but ~230 at a
// wave's slowest lane on C3).
struct FbcCol {
    FbcLdsU32* col;
    const uint32_t* in_words;
    uint64_t w0;
    FbGlobalBits g;
    __device__ uint32_t word(uint32_t k) const { return k < FBC_WORDS ? col[64 * k] : g.word(w0 + k); }
};
// DMX_FBK_DEFER (default): the tests that can only turn true once and stay true (a Kraft sum
// past 1, the sequence past HLIT + HDIST, the header past plim, an invalid code, a repeat with
// nothing before it) are folded into one sticky flag per symbol and decided once per call, so
// the serial symbol loop -- a true header's ~230 symbols set each wave's time -- carries fewer
// instructions; a failing candidate runs on for at most `steps` - 1 symbols.
#ifndef DMX_FBK_STEPS
#define DMX_FBK_STEPS 32  // symbols per fbk_step call (the wave refills idle lanes between calls)
#endif
#ifndef DMX_FBK_DEFER
#define DMX_FBK_DEFER 1
#endif
__device__ __forceinline__ void fbk_step_deferred(FbLengthCheck& c, const FbcCol& src, int steps) {
    if (c.st != FBK_RUN) return;
    uint32_t i = c.i, prev = c.prev, kl = c.kl, kd = c.kd, nd = c.nd, nb = c.nb, used = c.used, wi = c.wi;
    uint64_t buf = c.buf;
    bool eob = c.eob, bad = false;
    const uint32_t nlit = c.nlit, total = c.total;
    for (int k = 0; k < steps && i < total; k++) {
        if (nb < 32) {  // refill: at least 32 bits stay in the buffer (a symbol takes <= 14)
            buf |= (uint64_t)src.word(wi) << nb;
            wi++;
            nb += 32;
        }
        const uint32_t v = (uint32_t)buf;
        uint32_t sym, len;
        c.decode(v, &sym, &len);
        const uint32_t x = sym >= 16 ? 4u * (sym - 16) : 12u;  // (symbols 19+ do not occur)
        const uint32_t eb = (0x0732u >> x) & 15u;               // 16: 2, 17: 3, 18: 7 extra bits
        const uint32_t run = ((0x1B33u >> x) & 15u) + ((v >> len) & ((1u << eb) - 1u));  // 3, 3, 11; 1
        const uint32_t val = sym < 16 ? sym : sym == 16 ? prev : 0u;
        const uint32_t cons = len + eb;
        buf >>= cons;
        nb -= cons;
        used += cons;
        const uint32_t a = i < nlit ? min(i + run, nlit) - i : 0u;
        const uint32_t sh = 15 - (val ? val : 15u);
        kl += val ? a << sh : 0u;
        kd += val ? (run - a) << sh : 0u;
        nd += val ? run - a : 0u;
        eob |= val && i <= 256 && 256 < i + a;
        bad |= !len || (sym == 16 && i == 0);
        prev = val;
        i += run;
    }
    c.i = i;
    c.prev = prev;
    c.kl = kl;
    c.kd = kd;
    c.nd = nd;
    c.nb = nb;
    c.used = used;
    c.wi = wi;
    c.buf = buf;
    c.eob = eob;
    if (bad || i > total || kl > 32768 || kd > 32768 || used > c.plim) c.st = FBK_FAIL;
    else if (i == total) c.st = eob && kl == 32768 && (kd == 32768 || nd <= 1) ? FBK_PASS : FBK_FAIL;
}
__device__ __forceinline__ void fbk_step(FbLengthCheck& c, const FbcCol& src, int steps) {
    if (DMX_FBK_DEFER) {
        fbk_step_deferred(c, src, steps);
        return;
    }
    for (int k = 0; k < steps; k++) {
        if (c.st != FBK_RUN) break;
        if (c.i >= c.total) {
            c.st = c.eob && c.kl == 32768 && (c.kd == 32768 || c.nd <= 1) ? FBK_PASS : FBK_FAIL;
            break;
        }
        if (c.nb < 32) {  // refill: at least 32 bits stay in the buffer (a symbol takes <= 14)
            c.buf |= (uint64_t)src.word(c.wi) << c.nb;
            c.wi++;
            c.nb += 32;
        }
        const uint32_t v = (uint32_t)c.buf;
        uint32_t sym, len;
        c.decode(v, &sym, &len);
        const uint32_t eb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
        const uint32_t rb = sym == 16 ? 3u : sym == 17 ? 3u : sym == 18 ? 11u : 1u;
        const uint32_t run = rb + ((v >> len) & ((1u << eb) - 1u));
        const uint32_t val = sym < 16 ? sym : sym == 16 ? c.prev : 0u;
        const uint32_t cons = len + eb;
        c.buf >>= cons;
        c.nb -= cons;
        c.used += cons;
        // lengths [i, i + run): split at nlit
        const uint32_t a = c.i < c.nlit ? min(c.i + run, c.nlit) - c.i : 0u;
        const uint32_t b = run - a;
        const uint32_t sh = 15 - (val ? val : 15u);
        c.kl += val ? a << sh : 0u;
        c.kd += val ? b << sh : 0u;
        c.nd += val ? b : 0u;
        c.eob |= val && c.i <= 256 && 256 < c.i + a;
        const bool bad = !len || (sym == 16 && c.i == 0) || c.i + run > c.total || c.kl > 32768 || c.kd > 32768 ||
                         c.used > c.plim;
        c.prev = val;
        c.i += run;
        if (bad) c.st = FBK_FAIL;
    }
}
// A candidate that passes (and every stored-header hit) is also appended to keep (host memory
// mapped into the device; *nkeep counts, entries past keep_cap are dropped): the host reads the
// accepted starts -- a few hundred -- instead of the whole candidate list.
__global__ __launch_bounds__(64) void k_fb_check(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                                                  uint64_t* list, const uint64_t* pcount, unsigned long long* ph,
                                                  uint64_t* keep, uint32_t* nkeep, uint32_t keep_cap) {
    const uint64_t count = *pcount;  // (the grid is sized for the most the scan could list)
    if ((uint64_t)blockIdx.x * DMX_FBC_PER_WAVE >= count) return;
    auto accept = [&](uint64_t e) {
        if (!keep) return;
        const uint32_t k = atomicAdd(nkeep, 1u);
        if (k < keep_cap) keep[k] = e;
    };
    __shared__ uint32_t stg[FBC_WORDS * 64];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[128 * 64];
    const uint32_t lane = threadIdx.x;
    const FbGlobalBits g{in_words, (misalign + n + 3) / 4, misalign + n};
    FbcLdsU32* col = (FbcLdsU32*)(stg) + lane;
    const uint64_t below = (1ull << lane) - 1ull;
    FbLengthCheck ck;
    ck.st = FBK_FAIL;
    ck.tab = (FbcLdsU8*)(tabs) + 4 * lane;
    FbcCol src{col, in_words, 0, g};
    bool busy = false;
    uint64_t nxt = (uint64_t)blockIdx.x * DMX_FBC_PER_WAVE;
    const uint64_t end = min(count, nxt + DMX_FBC_PER_WAVE);
    uint64_t idx = 0, e = 0;
    uint64_t c_ref = 0, c_step = 0, n_out = 0, n_busy = 0, tl = ph ? clock64() : 0;
    for (;;) {
        // refill the idle lanes once half the wave is idle (or all of it)
        const uint64_t idle = __ballot(!busy);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nxt < end && (nidle >= 32 || nidle == 64)) {
            if (!busy) {
                idx = nxt + (uint64_t)__popcll(idle & below);
                if (idx < end) {
                    e = list[idx];
                    if (e & FB_HIT_STORED) {
                        accept(e);
                    } else {
                        busy = true;
                        const uint64_t q = misalign * 8 + e;
                        const uint64_t w0 = q >> 5;
                        uint32_t v[FBC_WORDS];
                        if (w0 + FBC_WORDS + 1 < g.nwords) {  // no tests: the loads issue back to back
#pragma unroll
                            for (uint32_t k = 0; k < FBC_WORDS; k++) v[k] = in_words[w0 + k];
                        } else {
#pragma unroll
                            for (uint32_t k = 0; k < FBC_WORDS; k++) v[k] = g.word(w0 + k);
                        }
#pragma unroll
                        for (uint32_t k = 0; k < FBC_WORDS; k++) col[64 * k] = v[k];
                        src.w0 = w0;
                        const FbcBits bits{col, w0 * 32, g};
                        const uint32_t h = bits.peek(q), x0 = bits.peek(q + 17), x1 = bits.peek(q + 49);
                        ck.set_precode(fb_precode_lengths(h, x0, x1));
                        // the code lengths from bit q + 17 + 3 HCLEN on; a header longer than 4096
                        // bits is none a real encoder writes
                        const uint32_t r = (uint32_t)(q - w0 * 32) + 17 + 3 * (((h >> 13) & 15) + 4);
                        ck.wi = (r >> 5) + 2;
                        ck.buf = (((uint64_t)src.word((r >> 5) + 1) << 32) | src.word(r >> 5)) >> (r & 31);
                        ck.nb = 64 - (r & 31);
                        ck.used = 0;
                        ck.plim = 4096 - (r - (uint32_t)(q - w0 * 32));
                        ck.nlit = ((h >> 3) & 31) + 257;
                        ck.total = ck.nlit + ((h >> 8) & 31) + 1;
                        ck.i = ck.prev = ck.kl = ck.kd = ck.nd = 0;
                        ck.eob = false;
                        ck.st = FBK_RUN;
                    }
                }
            }
            nxt += nidle;
        }
        if (ph) {
            const uint64_t now = clock64();
            c_ref += now - tl;
            tl = now;
        }
        const uint64_t bm = __ballot(busy);
        if (!bm) {
            if (nxt >= end) break;
            continue;
        }
        n_out++;
        n_busy += (uint64_t)__popcll(bm);
        if (busy) {
            fbk_step(ck, src, DMX_FBK_STEPS);
            if (ck.st != FBK_RUN) {
                if (ck.st == FBK_FAIL) list[idx] = e | FB_HIT_REJECT;
                else accept(e);
                busy = false;
            }
        }
        if (ph) {
            const uint64_t now = clock64();
            c_step += now - tl;
            tl = now;
        }
    }
    if (ph && lane == 0) {  // DMX_FB_DEBUG: refill and step cycles, steps, busy lanes per step
        atomicAdd(ph + 8, (unsigned long long)c_ref);
        atomicAdd(ph + 9, (unsigned long long)c_step);
        atomicAdd(ph + 10, (unsigned long long)n_out);
        atomicAdd(ph + 11, (unsigned long long)n_busy);
        atomicAdd(ph + 12, 1ull);
    }
}

// compact the per-chunk hits into one sorted list (offsets from the scan of counts)
__global__ void k_fb_compact(const uint32_t* counts, const uint64_t* offs, const uint64_t* hits,
                             uint64_t nchunks, uint64_t* list) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint32_t k = counts[c];
    for (uint32_t i = 0; i < k; i++) list[offs[c] + i] = hits[c * FB_HITS + i];
}

// ---------------------------------------------------------------------------------------
// k_fb_decode
// ---------------------------------------------------------------------------------------
// Token words (16-byte groups in HBM, one unit's list contiguous):
//   literal run   0 | cnt(7) = 1..3 | bytes(24)
//   match         1 | L(16) | d - 1(15)
//   stored        0 | 127(7) | len(24), always at an even index; the next word is the data's
//                 byte offset from the unit's first byte
//   no-op         0 (pads a stored header to an even index)
// Wave-uniform decoder state; token k of the current group of 64 is held by lane k.
struct TokSink {
    uint32_t* tk;
    uint32_t cap;    // words
    uint32_t n;      // words flushed
    uint32_t k;      // words in the lane-held group
    uint32_t reg;    // this lane's word of the group
    uint32_t pend, pendn;  // pending literal run
    uint64_t pos;    // output bytes of the unit so far
    uint64_t unit_byte0;   // unit start byte in the aligned image
    bool stream_start;
    uint32_t err;

    // fewer than two groups of room left: the unit stops at this token boundary (a soft end);
    // the chain walk resumes the block from there in a repair unit, so running out of token
    // space costs a repair, not the stream's trip to the serial decoder
    __device__ bool full() const { return n + k + 128 > cap; }
    __device__ bool flush_group() {
        if (n + 64 > cap) {
            err |= SEGF_OVERFLOW;
            return false;
        }
        tk[n + lane_id()] = reg;
        n += 64;
        k = 0;
        return true;
    }
    __device__ bool push(uint32_t w) {
        if (lane_id() == (int)k) reg = w;
        return ++k < 64 || flush_group();
    }
    __device__ bool flush_lits() {
        if (!pendn) return true;
        const uint32_t w = (pendn << 24) | pend;
        pend = 0;
        pendn = 0;
        return push(w);
    }
    __device__ bool literal(uint32_t b) {
        if (pendn == 3 && !flush_lits()) return false;
        pend |= b << (8 * pendn);
        pendn++;
        pos++;
        return true;
    }
    __device__ bool copy(uint32_t L, uint32_t dist) {
        if (L == 0 || dist == 0) return true;                 // reference: length/distance 0
        if (stream_start && dist > pos) return true;          // reference: nothing to copy
        if (!flush_lits()) return false;
        pos += L;
        return push(0x80000000u | (L << 15) | (dist - 1));
    }
    template <class BR>
    __device__ bool stored(const BR&, uint64_t b0, uint32_t len) {
        if (!flush_lits()) return false;
        if (((n + k) & 1) && !push(0)) return false;
        if (b0 - unit_byte0 > 0xFFFFFFFFull) {  // the offset word holds 32 bits: a unit spanning
            err |= SEGF_OVERFLOW;                // more than 4 GiB goes to the serial decoder
            return false;
        }
        if (!push((127u << 24) | len)) return false;
        pos += len;
        return push((uint32_t)(b0 - unit_byte0));
    }
    __device__ bool finish() {
        if (!flush_lits()) return false;
        if (k) {
            if (n + k > cap) {
                err |= SEGF_OVERFLOW;
                return false;
            }
            if (lane_id() < (int)k) tk[n + lane_id()] = reg;
            n += k;
            k = 0;
        }
        return true;
    }
};



struct FbDecodeArgs {
    const uint32_t* in_words;
    uint64_t misalign, n;
    const uint64_t* starts;
    const uint64_t* stops;   // FB_STOP_* flags
    const uint8_t* vmode;    // FB_V_*
    const uint64_t* vhdr;    // code state of FB_V_EXACT units
    uint64_t nunits;
    uint64_t u0;             // this launch decodes units u0 + blockIdx.x
    const uint64_t* tokoff;
    uint32_t* tok;
    FbUnit* units;
    uint32_t flags;
    uint32_t* stats;  // optional (DMX_FB_DEBUG): units decoded lane-parallel, serially from the
                      // start, serially after a parallel first block, weak units
    // fixed-code regions (k_fb_schunks): cbit[g] = the stream bit where the true token path
    // enters global region chunk g (~0: not entered); ucb[u] = the first global chunk of unit u's
    // super block, ~0 for a unit that is not a region unit (or nullptr: none)
    const uint64_t* cbit;
    const uint32_t* ucb;
};

// A fixed block that follows inside a unit is decoded serially only when it lies within this
// many bits of the unit's stop; farther ones end the unit at their header, and the host starts a
// unit there that decodes the run of fixed blocks lane-parallel (repair round).
constexpr uint64_t FB_SER_FIXED_MAX = 16384;

// One wavefront: realDecompress (inflate.hpp:277-322) for unit u from stream bit `from`
// (relative to stream bit 0), appending to a token list that already holds n0 words for bytes0
// output bytes; the unit's record is written at the end.  first: the block at `from` is the
// unit's first, decoded before any stop check.  mid: FB_AT_HEADER, or `from` lies inside a
// block whose code state is mid (FB_STATE_*): that block's rest is decoded first.
__device__ __attribute__((noinline)) void fb_serial(const FbDecodeArgs& A, uint64_t u, Tables& T, uint32_t* ring, uint64_t from,
                          uint32_t n0, uint64_t bytes0, bool first, uint64_t mid = FB_AT_HEADER) {
    if (lane_id() == 0) T.fixed_loaded = 0;
    wave_sync();
    const uint64_t start = A.starts[u];
    // A unit ends after the first block that lands exactly on another unit's start, or that
    // passes the next dynamic-header start (stored-header starts can be false: passing one
    // inside a block is no reason to stop, landing on one is a chain link); with a soft stop (the
    // next unit starts inside a block) at the first token boundary at or past it.
    // A unit at a stored-header start (FB_STOP_WEAK) decodes stored and fixed-code blocks
    // and ends before the first dynamic block (whose start is a scanned hit): such a start can
    // be false, and a false one then costs a bounded copy, or at most a fixed-code decode up to
    // the next dynamic-header start.  (Fixed blocks are not scanned, so a stored block followed
    // by fixed ones -- zlib's small blocks -- needs the weak unit to carry on through them.)
    const bool weak = (A.stops[u] & FB_STOP_WEAK) != 0;
    const bool soft = (A.stops[u] & FB_STOP_SOFT) != 0;
    const bool region_head = (A.stops[u] & FB_STOP_REGION) != 0;
    const uint64_t stop = A.stops[u] & FB_STOP_MASK;
    uint64_t jn = 0;  // first listed unit start above the unit's start (repair units are
    {                 // appended after the sorted list: search it)
        uint64_t hi = A.nunits;
        while (jn < hi) {
            const uint64_t mid = (jn + hi) >> 1;
            if (A.starts[mid] <= start) jn = mid + 1;
            else hi = mid;
        }
    }
    uint64_t end_at = 0;  // (end_set) aligned-image bit of the first block the unit leaves
    bool end_set = false; // undecoded: weak units, a far fixed block, a region head's run
    const uint64_t base = A.misalign * 8;  // stream bit 0 in the aligned image
    const uint64_t soft_abs = soft ? base + stop : ~0ull;
    RingIn br;
    br.init(A.in_words, A.misalign, A.n, ring);
    br.seek(base + from);
    TokSink sk;
    sk.tk = A.tok + A.tokoff[u];
    sk.cap = (uint32_t)(A.tokoff[u + 1] - A.tokoff[u]);
    sk.n = n0;
    sk.k = sk.reg = sk.pend = sk.pendn = 0;
    sk.pos = bytes0;
    sk.unit_byte0 = (base + start) >> 3;
    sk.stream_start = u == 0 && !(A.flags & DMX_IFLAG_PIECE);
    sk.err = 0;
    const bool rfc = (A.flags & DMX_CFG_RFC_STRICT) != 0;
    uint32_t err = 0;
    bool fin = false;
    uint64_t state = FB_AT_HEADER;  // the code in force while inside a block
    bool midend = false;            // stopped inside a block (soft stop)
    const uint64_t nwords = (A.misalign + A.n + 3) / 4;
    if (mid != FB_AT_HEADER) {  // the rest of a block whose code is `mid`
        state = mid;
        if (mid & FB_STATE_FIXED) {
            load_fixed(T);
            T.fixed_loaded = 1;
        } else {
            uint64_t hp = base + (mid & FB_STATE_POS) + 3;
            err = fast_header(BitInWords{nullptr, 0, 0, A.in_words, nwords, A.misalign + A.n}, &hp,
                              br.end_bits, T, rfc, true);
        }
        if (!err) err = decode_huffman(br, T, sk, soft_abs);
        if (err == SEGF_SOFT) {
            err = 0;
            midend = true;
        } else if (!err && (mid & FB_STATE_FINAL)) {
            fin = true;
        }
        first = false;
    }
    bool crossed = false;  // a block header was read after the unit's start
    for (bool f = first; !err && !fin && !midend; f = false) {
        if (!f) {
            const uint64_t pos = br.abspos() - base;
            if (pos >= stop || sk.full()) break;
            while (jn < A.nunits && A.starts[jn] < pos) jn++;
            if (jn < A.nunits && A.starts[jn] == pos) break;
        }
        const uint64_t hpos = br.abspos();
        br.ensure(3);
        const uint32_t bfinal = br.bits(1);
        const uint32_t btype = br.bits(2);
        if (br.over()) { err = SEGF_OVERREAD; break; }
        if (!f) crossed = true;
        if ((weak && btype == 2) || (f && region_head && btype != 2) ||
            (!f && btype == 1 && stop - (hpos - base) > FB_SER_FIXED_MAX)) {  // a far fixed run
            end_at = hpos;
            end_set = true;
            break;
        }
        if (btype == 0) {
            br.align();
            br.ensure(32);
            const uint32_t len = br.bits(16);
            (void)br.bits(16);  // NLEN, unchecked (inflate.hpp:293-303)
            if (br.over()) { err = SEGF_OVERREAD; break; }
            const uint64_t b0 = br.abspos() >> 3;
            if (b0 + len > br.end_bytes) { err = SEGF_OVERREAD; break; }
            if (!sk.stored(br, b0, len)) { err = sk.err; break; }
            br.seek(br.abspos() + 8ull * len);
        } else if (btype == 1) {
            if (!T.fixed_loaded) {
                load_fixed(T);
                T.fixed_loaded = 1;
            }
            state = FB_STATE_FIXED | (bfinal ? FB_STATE_FINAL : 0ull);
            err = decode_huffman(br, T, sk, soft_abs);
        } else if (btype == 2) {
            T.fixed_loaded = 0;
            state = (hpos - base) | (bfinal ? FB_STATE_FINAL : 0ull);
            uint64_t hp = br.abspos();
            err = fast_header(reader_words(br), &hp, br.end_bits, T, rfc, true);
            if (err) break;
            br.seek(hp);
            err = decode_huffman(br, T, sk, soft_abs);
        }  // BTYPE 3: an empty block (inflate.hpp:292 has no case 3)
        if (err == SEGF_SOFT) {
            err = 0;
            midend = true;
            break;
        }
        if (err) break;
        if (bfinal) {
            fin = true;
            break;
        }
    }
    if (!err && !sk.finish()) err = sk.err;
    if (lane_id() == 0) {
        FbUnit r;
        r.start = start;
        r.end = (end_set ? end_at : br.abspos()) - base;
        r.size = sk.pos;
        r.ntok = sk.n;
        r.hdr = midend ? state : FB_AT_HEADER;
        r.flags = err | (fin ? SEGF_FINAL : 0u) | (crossed ? SEGF_CROSSED : 0u);
        A.units[u] = r;
    }
}

// the serial decoder alone, one wavefront per unit (DMX_CFG_FB_SERIAL: A/B reference)
__global__ __launch_bounds__(64) void k_fb_decode(FbDecodeArgs A) {
    __shared__ Tables T;
    __shared__ uint32_t ring[FB_RW];
    const uint64_t u = A.u0 + blockIdx.x;  // (the grid is the launch's unit count)
    const uint8_t vm = A.vmode[u];
    fb_serial(A, u, T, ring, A.starts[u], 0, 0, true, vm == FB_V_EXACT ? A.vhdr[u] : FB_AT_HEADER);
}

// ---------------------------------------------------------------------------------------
// k_fb_pdecode: one workgroup of FBP_NT lanes per unit.  A unit whose first block is Huffman
// coded (fixed or dynamic) and whose bits up to the next dynamic-header start fit the staging
// buffer has that block decoded lane-parallel, the k_inflate_pj way:
//   1. wave 0 reads the block header from the staged words, the workgroup fills 32-bit tables;
//   2. the block body [hs, he) (he = the unit's stop) is split into ranges of >= FBP_MINBITS
//      bits; each lane warms up FBP_WARM bits before its range (Huffman decoding re-synchronises
//      within a few tokens), then decodes through its range marking token starts and counting
//      token words and output bytes;
//   3. settle: a lane whose start is not where the previous range's path crossed in re-decodes
//      from there until it meets one of its own token starts (normally nobody, or one round);
//   4. ranges past the first one that reaches end-of-block are dropped; lanes that moved recount;
//   5. exclusive scans of words and bytes, then every lane writes its range's token words (the
//      TokSink format: literal runs of up to 3, matches) at its word offset.
// The unit then ends where the serial decoder would end it (BFINAL, the stop, or landing on
// another unit start); otherwise wave 0 continues with fb_serial from the block's end.  Anything
// the parallel pass cannot vouch for -- a stored, weak or oversized unit, a header error, no
// end-of-block before `he`, a bad code, no settlement, a copy from before the stream start in
// unit 0 -- makes wave 0 decode the whole unit with fb_serial instead, so results and error
// codes are the serial decoder's.
// ---------------------------------------------------------------------------------------
#ifndef DMX_FBP_NT
#define DMX_FBP_NT 1024
#endif
#ifndef DMX_FBP_IN
#define DMX_FBP_IN 14336
#endif
constexpr int FBP_NT = DMX_FBP_NT;
constexpr uint32_t FBP_IN = DMX_FBP_IN;  // staged words (a block body of up to ~56 KB: zlib's
                                      // blocks of 16 K symbols at up to ~27 bits each)
#ifndef DMX_FBP_MINBITS
#define DMX_FBP_MINBITS 96
#endif
constexpr uint32_t FBP_MINBITS = DMX_FBP_MINBITS;  // shortest range a lane decodes
#ifndef DMX_FBP_WARM
#define DMX_FBP_WARM 448
#endif
constexpr uint32_t FBP_WARM = DMX_FBP_WARM;  // warm-up bits before a range
constexpr uint32_t TK_NOP = 4;         // a fixed block's end of block + the next fixed header
constexpr int FBP_ROUNDS = 1024;  // a settle cascade (data that re-synchronises slowly) still
                                   // beats the serial decoder by far
// exact range starts of a region unit: the entries of its super block's 64 chunks x 8
// sub-chunks of 512 bits (k_fb_schunks, below)
constexpr uint32_t FBS_SUBS = 8;
constexpr uint32_t FBS_XS = 64 * FBS_SUBS;
static_assert(FBS_XS <= (uint32_t)FBP_NT, "one candidate start per thread");
struct FbpSmem {
    uint32_t in[FBP_IN + 8];  // stream words [ws, ws + nst), zero after; fb_serial's ring later
    uint32_t bmap[FBP_IN];    // token starts of the first pass (bit p = body bit p)
    uint32_t llut[1 << PJ_LL];
    uint32_t dlut[1 << PJ_LD];
    Tables T;
    uint32_t endp[FBP_NT];    // where range r's path crossed into range r + 1
    uint32_t wcnt[FBP_NT];    // words of range r, then its exclusive word offset
    uint32_t bcnt[FBP_NT];    // output bytes of range r, then its exclusive byte offset
    uint32_t part[2][FBP_NT / 64];
    uint32_t xs[FBS_XS + 1];  // exact range starts (region units: the chunk entries), body bits
    uint32_t nx;              // their count (0: ranges split evenly, warm-up + settle)
    uint32_t te2[2];
    uint32_t kind;            // 0 parallel, 1 serial from the unit start, 2 serial continuation,
                              // 3 an error the serial decoder would report (S.err), 4 again
    uint32_t btype, bfinal, hs, nst, nst1, words, bytes, err;  // nst1: words staged so far
    uint32_t midend;          // the unit stopped inside a block (soft stop)
    uint32_t crossed;         // the settled path passed a fixed-block header (TK_NOP)
    uint64_t ws, he, hecap, endbit;
    uint64_t vstate;          // the code in force (FB_STATE_*)
};
static_assert(sizeof(FbpSmem) <= 160 * 1024, "LDS");

// wave 0 of k_fb_pdecode: the block's code tables from the staged words (out of line: the
// header reader's registers would otherwise spill in the 1024-lane kernel)
__device__ __attribute__((noinline)) uint32_t fbp_header(Tables& T, uint32_t btype, const uint32_t* in,
                                                         uint64_t ws, uint32_t nst, uint64_t* hp,
                                                         uint64_t end_bits, bool rfc, uint64_t* stamps) {
    if (btype == 1) {
        load_fixed(T);
        return 0;
    }
    const StagedWords src{in, ws, nst};
    return fast_header(src, hp, end_bits, T, rfc, false, stamps);
}
// the same for the header of the block a mid-block unit starts in, read from HBM
__device__ __attribute__((noinline)) uint32_t fbp_header_g(Tables& T, const uint32_t* words, uint64_t nwords,
                                                           uint64_t end_bytes, uint64_t* hp, bool rfc) {
    return fast_header(BitInWords{nullptr, 0, 0, words, nwords, end_bytes}, hp, end_bytes * 8, T, rfc, false);
}

__global__ __launch_bounds__(FBP_NT) void k_fb_pdecode(FbDecodeArgs A) {
    __shared__ __attribute__((aligned(16))) FbpSmem S;
    constexpr int NW = FBP_NT / 64;
    const int t = threadIdx.x;
    // DMX_FB_DEBUG: cycles per phase (thread 0), summed over units in stats[16..]
    unsigned long long* const ph = A.stats ? reinterpret_cast<unsigned long long*>(A.stats + 16) : nullptr;
    uint64_t ph_last = ph && t == 0 ? clock64() : 0;
    const uint64_t ph_t0 = ph_last;
    auto stamp = [&](int k) {
        if (ph && t == 0) {
            const uint64_t now = clock64();
            atomicAdd(ph + k, (unsigned long long)(now - ph_last));
            ph_last = now;
        }
    };
    const int wave = t >> 6;
    const uint64_t u = A.u0 + blockIdx.x;
    const uint64_t start = A.starts[u];
    const uint32_t vm = A.vmode[u];
    const bool weak = (A.stops[u] & FB_STOP_WEAK) != 0;
    const bool soft = (A.stops[u] & FB_STOP_SOFT) != 0;
    const uint64_t stop = A.stops[u] & FB_STOP_MASK;
    const uint64_t base = A.misalign * 8;
    const uint64_t end_bytes = A.misalign + A.n;
    const uint64_t nwords = (end_bytes + 3) / 4;
    const uint64_t nbits = 8 * A.n;
    const bool rfc = (A.flags & DMX_CFG_RFC_STRICT) != 0;
    const bool stream_start = u == 0 && !(A.flags & DMX_IFLAG_PIECE);
    auto stage_rest = [&]() {  // the staging window past S.nst1 (all threads; the caller syncs)
        for (uint32_t i = S.nst1 + t; i < S.nst + 8; i += FBP_NT) {
            uint32_t v = 0;
            if (i < S.nst) {
                const uint64_t wi = S.ws + i;
                v = A.in_words[wi];
                const uint64_t lim = end_bytes - 4 * wi;
                if (lim < 4) v &= (1u << (8 * lim)) - 1u;
            }
            S.in[i] = v;
        }
    };
    auto hdr3 = [&](uint64_t b) -> uint32_t {  // the 3 header bits at aligned-image bit b
        const uint32_t w0 = A.in_words[b >> 5];
        const uint32_t w1 = (b >> 5) + 1 < nwords ? A.in_words[(b >> 5) + 1] : 0u;
        return __builtin_amdgcn_alignbit(w1, w0, (uint32_t)(b & 31)) & 7u;
    };
    // ---- 1. block type (the code in force), staging window ----
    if (t == 0) {
        uint32_t kind = 1;
        const uint64_t b = base + start;
        uint32_t btype, bfinal;
        uint64_t state;
        if (vm == FB_V_HEADER) {
            const uint32_t h = hdr3(b);
            btype = (h >> 1) & 3;
            bfinal = h & 1;
            state = (btype == 1 ? FB_STATE_FIXED : start) | (bfinal ? FB_STATE_FINAL : 0ull);
        } else {  // inside a block (FB_V_EXACT): the code of vhdr's block
            const uint64_t vh = A.vhdr[u];
            const uint32_t h = (vh & FB_STATE_FIXED) ? 2u : hdr3(base + (vh & FB_STATE_POS));
            btype = ((h >> 1) & 3) == 2 ? 2u : 1u;  // a stored or fixed first block: fixed blocks follow
            bfinal = btype == 2 ? (h & 1) : ((vh & FB_STATE_FIXED) && (vh & FB_STATE_FINAL) ? 1u : 0u);
            state = (btype == 1 ? FB_STATE_FIXED : (vh & FB_STATE_POS)) | (bfinal ? FB_STATE_FINAL : 0ull);
        }
        // The block run must end by he: first the stop (the next unit start), then -- if no end of
        // block comes before a hard stop: a false header hit inside the block -- as far as the
        // staging reaches.  Staged: as many words as fit.
        const uint64_t ws = b >> 5;
        const uint64_t hecap = min(nbits, (ws + FBP_IN - 16) * 32 - base);
        if (!weak && (btype == 1 || btype == 2) && start + (vm == FB_V_HEADER ? 3 : 0) < hecap) {
            kind = 0;
            S.ws = ws;
            S.nst = (uint32_t)(min(ws + FBP_IN - 13, nwords) - ws);
            S.he = min(stop, hecap);
            S.hecap = hecap;
            // the first attempt reads up to he (and a token's lookahead): stage that much; the
            // rest only for a second attempt (a C3 unit's block is ~15 KB of the 56 KB window)
            // (at least 160 words past the start: the header a wave reads first)
            S.nst1 = (uint32_t)min((uint64_t)S.nst, max(((base + S.he) >> 5) - ws + 16, (b >> 5) - ws + 160));
        }
        // a region head whose first block is not dynamic: the unit is empty, the region map
        // takes the run of blocks from its header on
        if ((A.stops[u] & FB_STOP_REGION) && vm == FB_V_HEADER && btype != 2) kind = 5;
        S.kind = kind;
        S.err = SEGF_ERR_DATA;
        S.btype = btype;
        S.bfinal = bfinal;
        S.vstate = state;
        S.midend = 0;
        S.crossed = 0;
    }
    __syncthreads();
    if (S.kind == 0) {
        const uint64_t ws = S.ws;
        const uint32_t nst = S.nst1;
        for (uint32_t i = t; i < nst + 8; i += FBP_NT) {
            uint32_t v = 0;
            if (i < nst) {
                const uint64_t wi = ws + i;
                v = A.in_words[wi];
                const uint64_t lim = end_bytes - 4 * wi;
                if (lim < 4) v &= (1u << (8 * lim)) - 1u;
            }
            S.in[i] = v;
        }
        __syncthreads();
        stamp(0);
        if (wave == 0) {
            uint64_t hp = base + start + 3;
            uint32_t err = 0;
            if (vm == FB_V_HEADER) {
                uint64_t hst[4] = {0, 0, 0, 0};  // DMX_FB_DEBUG: the header's phases
                err = fbp_header(S.T, S.btype, S.in, ws, nst, &hp, end_bytes * 8, rfc, ph ? hst : nullptr);
                if (ph && lane_id() == 0)
                    for (int k = 0; k < 4; k++) atomicAdd(ph + 10 + k, (unsigned long long)hst[k]);
            } else {
                if (S.btype == 1) {
                    load_fixed(S.T);
                } else {
                    uint64_t hq = base + (S.vstate & FB_STATE_POS) + 3;
                    err = fbp_header_g(S.T, A.in_words, nwords, end_bytes, &hq, rfc);
                }
                hp = base + start;  // the body starts at the unit's start bit
            }
            if (lane_id() == 0) {
                const uint64_t hs = hp - ws * 32;
                if (err) {  // the serial decoder fails here too: the unit's record says so
                    S.kind = 3;
                    S.err = err;
                } else if (base + S.hecap - ws * 32 <= hs) {
                    S.kind = 1u;
                    if (A.stats) atomicAdd(&A.stats[4], 1u);
                } else if (base + S.he - ws * 32 <= hs) {
                    S.he = S.hecap;  // the stop lies inside the header
                }
                S.hs = (uint32_t)hs;
            }
        }
        __syncthreads();
        stamp(1);
        if (S.kind == 0 && S.he == S.hecap) stage_rest();  // the stop lay inside the header
        if (S.kind == 0) {
            fill_lut32_wg<PJ_LL, false>(S.llut, S.T.lm, S.T.lsorted, t, FBP_NT);
            fill_lut32_wg<PJ_LD, true>(S.dlut, S.T.dm, S.T.dsorted, t, FBP_NT);
        }
        __syncthreads();
        stamp(2);
    }
    // a fixed-code block whose end of block is followed by a non-final fixed-block header runs on
    // into it (the same code): a run of fixed blocks decodes as one block
    const bool fixcont = S.btype == 1 && !S.bfinal;
    auto tok = [&](const uint32_t* win, uint32_t* pa, uint32_t* a, uint32_t* d) -> uint32_t {
        const uint32_t k = pj_token(win, pa, S.llut, S.dlut, S.T, a, d);
        if (k == TK_EOB && fixcont && (lds_peek32(win, *pa) & 7u) == 2u) {  // BFINAL 0, BTYPE 01
            *pa += 3;
            return TK_NOP;
        }
        return k;
    };
    uint32_t dbg_rounds = 0, dbg_attempts = 0;  // DMX_FB_DEBUG (thread 0)
    for (int attempt = 0; attempt < 2 && S.kind == 0; attempt++) {
        dbg_attempts++;
        const uint32_t* win = S.in;
        const uint32_t hs = S.hs, hlen = (uint32_t)(base + S.he - S.ws * 32 - hs);
        // A region unit's chunks each have a known entry on the true token path (k_fb_schunks):
        // its ranges start exactly there, with no warm-up, and settle at once.  (Evenly split
        // ranges inside a fixed-code run need not re-synchronise -- literal runs of one code
        // length stay misaligned -- and settled one range per round: 3.7 ms per 32 KB unit.)
        {
            constexpr uint32_t NX = FBS_XS;  // entries per super block (chunks x sub-chunks)
            const uint64_t body = S.ws * 32 + hs - base;  // stream bit of the body's first token
            const uint32_t cb = A.ucb ? A.ucb[u] : ~0u;
            const uint64_t x = (cb != ~0u && (uint32_t)t < NX) ? A.cbit[(uint64_t)cb * FBS_SUBS + t] : ~0ull;
            const bool v = x != ~0ull && x > body && x - body < hlen;
            const uint64_t m = __ballot(v);
            if ((t & 63) == 0) S.part[0][wave] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t before = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                const uint32_t c = S.part[0][w];
                before += w < wave ? c : 0u;
                tot += c;
            }
            if (v) S.xs[1 + before + __popcll(m & ((1ull << (t & 63)) - 1ull))] = (uint32_t)(x - body);
            if (t == 0) {
                S.xs[0] = 0;
                S.nx = cb != ~0u ? 1u + tot : 0u;
            }
        }
        __syncthreads();
        const uint32_t nx = S.nx;
        const uint32_t nl = nx ? nx : max(1u, min((uint32_t)FBP_NT, hlen / FBP_MINBITS));
        const uint32_t r = (uint32_t)((t & 63) * NW + wave);
        const uint32_t sp = r < nl ? (nx ? S.xs[r] : (uint32_t)(((uint64_t)hlen * r) / nl)) : hlen;
        const uint32_t sp1 = r + 1 < nl ? (nx ? S.xs[r + 1] : (uint32_t)(((uint64_t)hlen * (r + 1)) / nl)) : hlen;
        const uint32_t cw = hlen / 32 + 2;
        for (uint32_t i = t; i < cw; i += FBP_NT) S.bmap[i] = 0;
        if (t < 2) S.te2[t] = FBP_NT;
        __syncthreads();
        // ---- 2. warm-up, first pass ----
        uint32_t s0 = sp;
        if (r > 0 && r < nl && !nx) {
            int32_t p = (int32_t)sp - (int32_t)FBP_WARM;
            if (p < 0) p = 0;
            uint32_t pa = (uint32_t)((int32_t)hs + p);
            bool ok = true;
            while (p < (int32_t)sp) {
                uint32_t a, d;
                const uint32_t k = tok(win, &pa, &a, &d);
                if (k == TK_BAD || k == TK_EOB) { ok = false; break; }
                p = (int32_t)(pa - hs);
            }
            if (ok && p < (int32_t)sp1) s0 = (uint32_t)p;
        }
        uint32_t e1, st1 = 0, w1 = 0, b1 = 0;
        {
            uint32_t p = s0, pa = hs + s0, pn = 0;
            while (p < sp1) {
                atomicOr(&S.bmap[p >> 5], 1u << (p & 31));
                uint32_t a, d;
                const uint32_t k = tok(win, &pa, &a, &d);
                if (k == TK_BAD) { st1 = 2; break; }
                p = pa - hs;
                if (k == TK_EOB) { st1 = 1; break; }
                if (k == TK_NOP) continue;
                if (k == TK_LIT) {
                    if (pn == 3) { w1++; pn = 0; }
                    pn++;
                    b1++;
                } else if (a && d) {
                    w1 += pn ? 2u : 1u;
                    pn = 0;
                    b1 += a;
                }
            }
            if (pn) w1++;
            e1 = p;
        }
        stamp(3);
        // ---- 3. settle the range starts (k_inflate_pj's protocol) ----
        uint32_t s = s0, e = e1, st = st1;
        uint32_t te = FBP_NT;
        bool settled = false;
        for (int round = 0; round <= FBP_ROUNDS; round++) {
            S.endp[r] = e;
            if (st) atomicMin(&S.te2[round & 1], r);
            if (t == 0) S.te2[(round + 1) & 1] = FBP_NT;
            __syncthreads();
            te = S.te2[round & 1];
            const uint32_t want = r == 0 ? 0 : S.endp[r - 1];
            const bool redo = r > 0 && r <= te && want != s;
            if (ph && t == 0) atomicAdd(ph + 8, 1ull);  // DMX_FB_DEBUG: settle rounds
            dbg_rounds++;
            if (ph && redo) atomicAdd(ph + 9, 1ull);    // and lanes that redo
            if (!__syncthreads_or(redo)) {
                settled = true;
                break;
            }
            if (round == FBP_ROUNDS) break;
            const uint64_t rd0 = ph && t == 0 ? clock64() : 0;
            if (redo) {
                s = want;
                uint32_t p = want, pa = hs + want, stn = 0;
                bool merged = false;
                for (;;) {
                    if (p >= sp1) break;
                    if (p >= sp && ((S.bmap[p >> 5] >> (p & 31)) & 1u)) {
                        merged = true;
                        break;
                    }
                    uint32_t a, d;
                    const uint32_t k = tok(win, &pa, &a, &d);
                    if (k == TK_BAD) { stn = 2; break; }
                    p = pa - hs;
                    if (k == TK_EOB) { stn = 1; break; }
                }
                e = merged ? e1 : p;
                st = merged ? st1 : stn;
            }
            __syncthreads();
            if (ph && t == 0) atomicAdd(ph + 20, (unsigned long long)(clock64() - rd0));  // DMX_FB_DEBUG
        }
        stamp(4);
        // ---- 4. the block's end; recount ranges that moved ----
        if (t == 0 && !settled) {
            S.kind = 1u;
            if (A.stats) atomicAdd(&A.stats[5], 1u);
        } else if (t == 0 && te >= (uint32_t)FBP_NT) {
            if (soft && S.he == stop) {
                // the soft stop: the unit ends at the first token boundary at or past it, inside
                // the block run (the next unit starts there)
                S.midend = 1;
                S.endbit = S.ws * 32 + hs + S.endp[nl - 1] - base;
            } else {
                // no end of block before he: again up to the staging's end, else serially
                S.kind = S.he < S.hecap ? 4u : (1u);
                if (S.kind == 4) S.he = S.hecap;
                if (A.stats) atomicAdd(&A.stats[6], 1u);
            }
        }
        if (r == te && settled) {
            // a code that decodes to nothing, or an end past the stream: the serial decoder
            // stops with this error too
            const uint64_t pe_abs = S.ws * 32 + hs + e;
            if (st != 1 || pe_abs > end_bytes * 8) {
                S.kind = 3;
                S.err = st != 1 ? SEGF_ERR_DATA : SEGF_OVERREAD;
                if (A.stats) atomicAdd(&A.stats[7], 1u);
            }
            S.endbit = pe_abs - base;
        }
        __syncthreads();
        const uint32_t kk = S.kind;
        if (kk != 0) {
            __syncthreads();  // every lane has read it
            if (kk == 4) stage_rest();  // again up to the staging's end
            if (kk == 4 && t == 0) S.kind = 0;
            __syncthreads();
            continue;
        }
        if (r <= te && s != s0) {
            uint32_t p = s, pa = hs + s, pn = 0;
            w1 = b1 = 0;
            while (p < sp1) {
                uint32_t a, d;
                const uint32_t k = tok(win, &pa, &a, &d);
                p = pa - hs;
                if (k == TK_BAD || k == TK_EOB) break;
                if (k == TK_NOP) continue;
                if (k == TK_LIT) {
                    if (pn == 3) { w1++; pn = 0; }
                    pn++;
                    b1++;
                } else if (a && d) {
                    w1 += pn ? 2u : 1u;
                    pn = 0;
                    b1 += a;
                }
            }
            if (pn) w1++;
        }
        stamp(5);
        // ---- 5. scans, then the token words ----
        S.wcnt[r] = r <= te ? w1 : 0u;
        S.bcnt[r] = r <= te ? b1 : 0u;
        __syncthreads();
        const uint32_t cwv = S.wcnt[t], cbv = S.bcnt[t];
        const uint32_t iw = wave_incl_scan(cwv), ib = wave_incl_scan(cbv);
        if ((t & 63) == 63) {
            S.part[0][wave] = iw;
            S.part[1][wave] = ib;
        }
        __syncthreads();
        uint32_t bw = 0, bb = 0, tw = 0, tb = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint32_t x = S.part[0][w], y = S.part[1][w];
            bw += w < wave ? x : 0u;
            bb += w < wave ? y : 0u;
            tw += x;
            tb += y;
        }
        __syncthreads();  // every lane has read its counts
        S.wcnt[t] = bw + iw - cwv;
        S.bcnt[t] = bb + ib - cbv;
        const uint32_t cap = (uint32_t)(A.tokoff[u + 1] - A.tokoff[u]);
        if (t == 0) {
            S.words = tw;
            S.bytes = tb;
            if (tw > cap) {
                S.kind = 1u;
                if (A.stats) atomicAdd(&A.stats[8], 1u);
            }
        }
        __syncthreads();
        stamp(6);
        if (S.kind == 0 && r <= te) {
            uint32_t* tk = A.tok + A.tokoff[u] + S.wcnt[r];
            uint32_t o = S.bcnt[r];
            uint32_t p = s, pa = hs + s, pn = 0, pend = 0, nw = 0;
            bool drop = false;
            while (p < sp1) {
                uint32_t a, d;
                const uint32_t k = tok(win, &pa, &a, &d);
                p = pa - hs;
                if (k == TK_BAD || k == TK_EOB) break;
                if (k == TK_NOP) {
                    S.crossed = 1;
                    continue;
                }
                if (k == TK_LIT) {
                    if (pn == 3) {
                        tk[nw++] = (3u << 24) | pend;
                        pn = pend = 0;
                    }
                    pend |= a << (8 * pn);
                    pn++;
                    o++;
                } else if (a && d) {
                    if (stream_start && d > o) drop = true;  // the reference copies nothing
                    if (pn) {
                        tk[nw++] = (pn << 24) | pend;
                        pn = pend = 0;
                    }
                    tk[nw++] = 0x80000000u | (a << 15) | (d - 1);
                    o += a;
                }
            }
            if (pn) tk[nw++] = (pn << 24) | pend;
            if (drop) {
                S.kind = 1u;
                if (A.stats) atomicAdd(&A.stats[9], 1u);
            }
        }
        __syncthreads();
        stamp(7);
        // the unit ends after this block unless the serial decoder would go on; a fixed block
        // far from the stop ends it too (the host starts a lane-parallel unit at its header)
        if (t == 0 && S.kind == 0 && !S.bfinal && !S.midend) {
            const uint64_t pos = S.endbit;
            bool ends = pos >= stop ||
                        (((hdr3(base + pos) >> 1) & 3) == 1 && stop - pos > FB_SER_FIXED_MAX);
            if (!ends) {
                uint64_t lo = 0, hi = A.nunits;  // first listed start >= pos
                while (lo < hi) {
                    const uint64_t mid = (lo + hi) >> 1;
                    if (A.starts[mid] < pos) lo = mid + 1;
                    else hi = mid;
                }
                ends = lo < A.nunits && A.starts[lo] == pos;
            }
            if (!ends) S.kind = 2;
        }
        __syncthreads();
        break;
    }
    const uint32_t kind = S.kind;
    if (A.stats && t == 0 && kind != 5) atomicAdd(&A.stats[weak ? 3 : kind == 3 ? 0 : kind], 1u);
    const uint64_t rstart = start;
    if (kind == 0 || kind == 3 || kind == 5) {
        if (t == 0) {
            FbUnit rec;
            rec.start = rstart;
            rec.end = kind == 0 ? S.endbit : start;
            rec.size = kind == 0 ? S.bytes : 0;
            rec.ntok = kind == 0 ? S.words : 0;
            rec.hdr = kind == 0 && S.midend ? S.vstate : FB_AT_HEADER;
            rec.flags = kind == 3 ? S.err
                        : kind == 5 ? 0u
                                    : ((S.bfinal && !S.midend) ? SEGF_FINAL : 0u) | (S.crossed ? SEGF_CROSSED : 0u);
            A.units[u] = rec;
        }
    } else if (wave == 0) {
        const uint32_t crossed = S.crossed;
        if (kind == 1) fb_serial(A, u, S.T, S.in, start, 0, 0, true, vm == FB_V_EXACT ? A.vhdr[u] : FB_AT_HEADER);
        else fb_serial(A, u, S.T, S.in, S.endbit, S.words, S.bytes, false);
        if (lane_id() == 0) {
            A.units[u].start = rstart;
            if (kind == 2 && crossed) A.units[u].flags |= SEGF_CROSSED;
        }
    }
    // DMX_FB_DEBUG: the longest unit of each kind (wave 0's span), in ph[14..17]: lane-parallel,
    // serial from the start, serial after a parallel block, weak
    if (ph && t == 0) {
        const uint32_t slot = weak ? 3u : kind == 1 ? 1u : kind == 2 ? 2u : 0u;
        const uint64_t dur = clock64() - ph_t0;  // (the longest's settle rounds and attempts below it)
        atomicMax(ph + 14 + slot, (unsigned long long)((dur << 24) | (min(dbg_rounds, 4095u) << 4) | min(dbg_attempts, 15u)));
    }
}

// ---------------------------------------------------------------------------------------
// k_fb_replay
// ---------------------------------------------------------------------------------------
// One wavefront per unit on the chain.  Tokens are taken 64 at a time, cut so that a group
// writes at most FB_GROUP_MAX entries (a longer stored block is copied alone, in pieces).
// Inside a group (T = its output size, o = a token's offset in it):
//   1. "far" matches (d > FB_RING - T), in order, one wave copy each: their sources lie before
//      the group and are the only ones a write of this group could overwrite in the ring, so
//      they read first.  (A later far match's source is never written by an earlier one.)
//   2. literal runs, and matches whose source lies wholly before the group, one lane each.
//   3. stored blocks and the remaining matches, in order, one wave copy each.
//   4. the group's entries go to the 16-bit output image in HBM.
struct FbReplayArgs {
    const uint8_t* stream;       // stream byte 0
    const uint64_t* starts;      // unit start bits
    const uint32_t* chain;       // unit index of the k-th unit on the chain
    const uint64_t* offs;        // output offset of the k-th unit on the chain
    const uint64_t* tokoff;
    const uint32_t* tok;
    const FbUnit* units;
    uint16_t* img;               // 16-bit output image (total entries)
    uint32_t* err;               // set to 1 when a copy reaches before the stream start
    unsigned long long* ph;      // DMX_FB_DEBUG: k_fb_units cycles per phase, or nullptr
};

// ring copy of L entries from src (ring index) to dst, src < dst in stream order (dst - src =
// d); periodic when d < L.  Every lane reads its sources before any lane writes (per 64).
__device__ __forceinline__ void fb_ring_copy(uint16_t* ring, uint32_t dst, uint32_t d, uint32_t L) {
    const uint32_t lane = lane_id();
    if (d >= L) {
        for (uint32_t i0 = 0; i0 < L; i0 += 256) {
            uint16_t v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t i = i0 + 64 * k + lane;
                v[k] = i < L ? ring[(dst - d + i) & (FB_RING - 1)] : 0;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t i = i0 + 64 * k + lane;
                if (i < L) ring[(dst + i) & (FB_RING - 1)] = v[k];
            }
        }
        return;
    }
    // periodic: pattern of d entries, lane i writes entry i, i + P, ... with P a multiple of d
    const uint32_t P = d >= 64 ? d : d * (64 / d);
    uint16_t pat[4];
    // entries [0, P) of the copy come from the d source entries (index mod d)
    for (uint32_t i0 = 0; i0 < P; i0 += 256) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t i = i0 + 64 * k + lane;
            pat[k] = i < P ? ring[(dst - d + (i % d)) & (FB_RING - 1)] : 0;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t i = i0 + 64 * k + lane;
            for (uint32_t j = i; j < L && i < P; j += P) ring[(dst + j) & (FB_RING - 1)] = pat[k];
        }
    }
}

__global__ __launch_bounds__(64) void k_fb_replay(FbReplayArgs A) {
    __shared__ __attribute__((aligned(16))) uint16_t ring[FB_RING];
    const uint32_t lane = lane_id();
    const uint64_t ci = blockIdx.x;
    const uint32_t u = A.chain[ci];
    const FbUnit rec = A.units[u];
    const uint64_t off = A.offs[ci];
    const uint32_t* tk = A.tok + A.tokoff[u];
    const uint32_t n = rec.ntok;
    const uint64_t byte0 = A.starts[u] >> 3;  // stored offsets are relative to this byte
    uint16_t* const img = A.img + off;
    // the entries before the unit: markers 0x8000 | (b - 1) for "b bytes before the start"
    for (uint32_t i = lane; i < FB_RING; i += 64) ring[i] = (uint16_t)(0x8000u | (FB_RING - 1 - i));
    wave_sync();
    uint64_t pos = 0;   // output entries so far (ring index = pos mod FB_RING)
    bool bad = false;   // a copy reaching before the stream start
    uint32_t t0 = 0;
    // token words t0 + lane (wc) and t0 + 64 + lane (wn, loaded a group ahead: its latency
    // passes while the current group replays), word t0 - 1 (wl)
    uint32_t wc = lane < n ? tk[lane] : 0u;
    uint32_t wn = 64 + lane < n ? tk[64 + lane] : 0u;
    uint32_t wl = 0;
    auto advance = [&](uint32_t adv) {  // 1 <= adv <= 64
        const uint32_t idx = lane + adv;
        const uint32_t a = (uint32_t)__shfl((int)wc, (int)(idx & 63), 64);
        const uint32_t b = (uint32_t)__shfl((int)wn, (int)(idx & 63), 64);
        wl = (uint32_t)__shfl((int)wc, (int)(adv - 1), 64);
        wc = idx < 64 ? a : b;
        const uint32_t nx = t0 + adv + 64 + lane;
        wn = idx < 64 ? b : (nx < n ? tk[nx] : 0u);
        t0 += adv;
    };
    while (t0 < n) {
        const uint32_t ti = t0 + lane;
        const uint32_t w = wc;
        // the word after a stored header is its offset (any 32-bit value, bit 31 included):
        // lane ti - 1 is that header
        const uint32_t wprev = (uint32_t)__shfl((int)w, (int)lane - 1, 64);
        const uint32_t wp = lane == 0 ? wl : wprev;
        const bool isoff = (ti & 1) && !(wp >> 31) && ((wp >> 24) & 127) == 127 && ((ti - 1) & 1) == 0;
        const bool ism = (w >> 31) != 0 && !isoff;
        const uint32_t cnt = (w >> 24) & 127;
        const bool isst = !ism && !isoff && cnt == 127 && (ti & 1) == 0;
        const bool islit = !ism && !isst && !isoff && cnt >= 1 && cnt <= 3;
        uint32_t L = ism ? (w >> 15) & 0xFFFFu : isst ? (w & 0xFFFFFFu) : islit ? cnt : 0u;
        const uint32_t d = (w & 0x7FFFu) + 1;
        if (ti >= n) L = 0;
        uint32_t incl = wave_incl_scan(L);
        // cut the group at FB_GROUP_MAX entries (at least one token)
        const uint64_t over = __ballot(incl > FB_GROUP_MAX && ti < n);
        uint32_t ntk = over ? (uint32_t)__builtin_ctzll(over) : 64u;
        const uint32_t avail = n - t0 < 64 ? n - t0 : 64u;
        if (ntk > avail) ntk = avail;
        if (ntk == 0) {
            // a stored block larger than a group: copy it alone, in pieces of FB_GROUP_MAX
            const uint32_t len = (uint32_t)__builtin_amdgcn_readfirstlane((int)L);
            const uint32_t so = (uint32_t)__builtin_amdgcn_readlane((int)w, 1);
            const uint8_t* src = A.stream + byte0 + so;
            for (uint32_t p0 = 0; p0 < len; p0 += FB_GROUP_MAX) {
                const uint32_t m = min(FB_GROUP_MAX, len - p0);
                for (uint32_t i = lane; i < m; i += 64) ring[(pos + p0 + i) & (FB_RING - 1)] = src[p0 + i];
                wave_sync();
                for (uint32_t i = lane; i < m; i += 64) img[pos + p0 + i] = ring[(pos + p0 + i) & (FB_RING - 1)];
                wave_sync();
            }
            pos += len;
            advance(2);
            continue;
        }
        const bool inq = lane < ntk;
        if (!inq) L = 0;
        incl = wave_incl_scan(L);
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t o = incl - L;  // offset in the group
        const uint64_t gpos = pos + o;
        // a copy must stay inside the stream (reference: a too-far distance copies nothing,
        // which this path cannot express once sizes are fixed -> serial path)
        if (inq && ism && L && (uint64_t)d > off + gpos) bad = true;
        const bool far = inq && ism && L && d > FB_RING - T;
        const bool simple = inq && ism && L && !far && o + L <= d;  // source before the group
        // 1. far matches, in order
        uint64_t m = __ballot(far);
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t ok = (uint32_t)__builtin_amdgcn_readlane((int)o, k);
            const uint32_t Lk = (uint32_t)__builtin_amdgcn_readlane((int)L, k);
            const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)d, k);
            fb_ring_copy(ring, (uint32_t)((pos + ok) & (FB_RING - 1)), dk, Lk);
            wave_sync();
        }
        // 2. literal runs and matches with their source before the group
        if (islit && inq) {
            const uint32_t r = (uint32_t)(gpos & (FB_RING - 1));
            ring[r] = (uint16_t)(w & 0xFF);
            if (cnt > 1) ring[(r + 1) & (FB_RING - 1)] = (uint16_t)((w >> 8) & 0xFF);
            if (cnt > 2) ring[(r + 2) & (FB_RING - 1)] = (uint16_t)((w >> 16) & 0xFF);
        }
        if (simple) {
            const uint32_t r = (uint32_t)(gpos & (FB_RING - 1));
            for (uint32_t i = 0; i < L; i++) ring[(r + i) & (FB_RING - 1)] = ring[(r - d + i) & (FB_RING - 1)];
        }
        wave_sync();
        // 3. stored blocks and the remaining matches, in order
        m = __ballot(inq && L && ((ism && !far && !simple) || isst));
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t ok = (uint32_t)__builtin_amdgcn_readlane((int)o, k);
            const uint32_t Lk = (uint32_t)__builtin_amdgcn_readlane((int)L, k);
            const uint32_t wk = (uint32_t)__builtin_amdgcn_readlane((int)w, k);
            const uint32_t dst = (uint32_t)((pos + ok) & (FB_RING - 1));
            if (wk >> 31) {
                fb_ring_copy(ring, dst, (wk & 0x7FFFu) + 1, Lk);
            } else {
                // the offset word is token k + 1: in this group, or the first of the next
                const uint32_t so0 = (uint32_t)__shfl((int)w, (k + 1) & 63, 64);
                const uint32_t so1 = (uint32_t)__builtin_amdgcn_readlane((int)wn, 0);
                const uint32_t so = k + 1 < 64 ? so0 : so1;
                const uint8_t* src = A.stream + byte0 + so;
                for (uint32_t i = lane; i < Lk; i += 64) ring[(dst + i) & (FB_RING - 1)] = src[i];
            }
            wave_sync();
        }
        // 4. the group's entries to the image
        for (uint32_t i = lane; i < T; i += 64) img[pos + i] = ring[(pos + i) & (FB_RING - 1)];
        wave_sync();
        pos += T;
        advance(ntk);
    }
    if (__ballot(bad) && lane == 0) atomicOr(A.err, 1u);
}

// ---------------------------------------------------------------------------------------
// k_fb_units: the replay as pointer jumping, one 1024-lane workgroup per unit on the chain
// (replaces k_fb_replay's one wavefront, whose copies inside a 64-token group run one after
// another).  The unit's output is built in pieces of FBU_PS positions, all in LDS:
//   1. the token words, 1024 at a time (the next batch's words loaded while this one is
//      expanded): a block scan of their lengths gives each token's output offset.  A batch of
//      short tokens expands one token per lane; in a batch whose waves' longest tokens average
//      more than 40 positions each thread takes FBU_PS / 1024 consecutive positions of the piece, finds the
//      token of the first by binary search and walks on.  A literal gives a final
//      byte, a match for each byte the position it copies from (periodic copies point into
//      the first period) or -- before the unit -- the final marker 0x8000 | (b - 1).  (Round 4
//      expanded one token per lane: a wave waited for its longest match, 255K of ~330K cycles
//      per C3 unit.)  Stored blocks are copied by the whole workgroup from the stream.  A
//      batch that runs past the piece's end finishes the piece (2., 3.) and goes on in the next;
//   2. pointer jumping in the piece, in place, until every entry is final: a source before
//      the piece is final in one hop, since the ring R holds the last FBU_R resolved
//      positions (a match reaches at most 32 KiB back);
//   3. the piece's low 16 bits -- a byte or a marker, k_fb_replay's image format -- to the
//      16-bit image in HBM and to R.
// Round 4 kept a 32-bit image of the whole unit in HBM and jumped through it there: 16 bytes
// of HBM traffic per output byte (PMC on C3) and a dependent HBM load per hop; now the token
// words and the 2-byte image are the only HBM traffic.
// ---------------------------------------------------------------------------------------
constexpr int FBR_NT = 1024;
constexpr uint32_t FBR_FINAL = 0x80000000u;
constexpr uint32_t FBU_PS = 16384;  // piece positions (32-bit entries: 64 KiB of LDS)
constexpr uint32_t FBU_R = 32768;   // resolved ring (16-bit entries: 64 KiB)
constexpr uint32_t FBU_LIT = 1, FBU_MATCH = 2, FBU_STORED = 3;
#ifndef DMX_FBU_SPREAD
#define DMX_FBU_SPREAD 40
#endif
__global__ __launch_bounds__(FBR_NT) void k_fb_units(FbReplayArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t C[FBU_PS];
    __shared__ __attribute__((aligned(16))) uint16_t R[FBU_R];
    __shared__ uint32_t Gw[FBR_NT];      // spread batches: the token words,
    __shared__ uint32_t Go[FBR_NT + 1];  // their unit-relative output offsets (+ the batch end)
    __shared__ uint8_t Gk[FBR_NT];       // and kinds (FBU_*, 0: no output)
    __shared__ uint32_t part[FBR_NT / 64], pmax[FBR_NT / 64];
    __shared__ uint32_t slist[FBR_NT / 2][3];  // stored blocks of the batch: offset, length, source
    __shared__ uint32_t nst;
    constexpr int NW = FBR_NT / 64;
    const uint32_t t = threadIdx.x, wave = t >> 6;
    const uint64_t ci = blockIdx.x;
    const uint32_t u = A.chain[ci];
    const FbUnit rec = A.units[u];
    const uint64_t off = A.offs[ci];
    const uint32_t* tk = A.tok + A.tokoff[u];
    const uint32_t n = rec.ntok;
    const uint32_t usize = (uint32_t)rec.size;
    const uint8_t* sbase = A.stream + (A.starts[u] >> 3);  // stored offsets are relative to this byte
    uint16_t* const img = A.img + off;
    bool bad = false, open = false;
    uint32_t obase = 0;  // unit-relative output offset of the batch
    uint32_t pstart = 0; // the current piece: [pstart, pstart + FBU_PS)
    if (t == 0) nst = 0;
    uint64_t ph_last = A.ph && t == 0 ? clock64() : 0;
    auto stamp = [&](int k) {
        if (A.ph && t == 0) {
            const uint64_t now = clock64();
            atomicAdd(A.ph + k, (unsigned long long)(now - ph_last));
            ph_last = now;
        }
    };
    // pointer jumping in the piece's pn entries, then the piece to the image and to R
    auto finish_piece = [&](uint32_t pn) {
        __syncthreads();  // every entry of the piece written
        stamp(1);
        for (int round = 0; round < 32; round++) {
            bool pend = false;
            for (uint32_t x = t; x < pn; x += FBR_NT) {
                uint32_t v = C[x];
                if (v & FBR_FINAL) continue;
#pragma unroll 1
                for (int h = 0; h < 8 && !(v & FBR_FINAL); h++)
                    v = v < pstart ? (FBR_FINAL | R[v & (FBU_R - 1)]) : C[v - pstart];
                C[x] = v;  // at once: entries read later in the round see it
                pend |= !(v & FBR_FINAL);
            }
            if (A.ph && t == 0) atomicAdd(A.ph + 4, 1ull);
            if (!__syncthreads_or(pend)) break;
            if (round == 31) open = true;  // cannot happen: chains strictly go back
        }
        stamp(2);
        for (uint32_t x = t; x < pn; x += FBR_NT) {
            const uint16_t v = (uint16_t)C[x];
            img[pstart + x] = v;
            R[(pstart + x) & (FBU_R - 1)] = v;
        }
        __syncthreads();  // R and C reused
        stamp(3);
        pstart += pn;
    };
    uint32_t w = t < n ? tk[t] : 0u;
    uint32_t wp = t >= 1 && t - 1 < n ? tk[t - 1] : 0u;
    for (uint32_t c0 = 0; c0 < n; c0 += FBR_NT) {
        const uint32_t ti = c0 + t;
        // the next batch's words, loaded now
        const uint32_t tn = ti + FBR_NT;
        const uint32_t wn = tn < n ? tk[tn] : 0u;
        const uint32_t wpn = tn - 1 < n ? tk[tn - 1] : 0u;
        // the word after a stored header (at an even index) is its offset: any 32-bit value
        const bool isoff = (ti & 1) && !(wp >> 31) && ((wp >> 24) & 127) == 127;
        const bool ism = (w >> 31) != 0 && !isoff;
        const uint32_t cnt = (w >> 24) & 127;
        const bool isst = !ism && !isoff && cnt == 127 && !(ti & 1);
        const bool islit = !ism && !isst && !isoff && cnt >= 1 && cnt <= 3;
        uint32_t L = ism ? (w >> 15) & 0xFFFFu : isst ? (w & 0xFFFFFFu) : islit ? cnt : 0u;
        if (ti >= n) L = 0;
        // block-wide exclusive scan of the lengths; each wave's longest token
        const uint32_t inc = wave_incl_scan(L);
        uint32_t lmax = L;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) lmax = max(lmax, (uint32_t)__shfl_xor((int)lmax, o, 64));
        if ((t & 63) == 63) {
            part[wave] = inc;
            pmax[wave] = lmax;
        }
        __syncthreads();
        uint32_t before = 0, T = 0, smax = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t v = part[k];
            before += k < (int)wave ? v : 0u;
            T += v;
            smax += pmax[k];
        }
        const uint32_t go = obase + before + inc - L;
        const uint32_t d = (w & 0x7FFFu) + 1;
        if (ism && L && (uint64_t)d > off + go) bad = true;  // a copy from before the stream start
        const uint32_t gend = go + L;
        const uint32_t gk = !L ? 0u : islit ? FBU_LIT : ism ? FBU_MATCH : FBU_STORED;
        const uint32_t bend = obase + T;
        // one token per lane costs each wave its longest token; spreading the positions costs
        // ~16 stores per thread plus a binary search: spread when the waves' longest tokens
        // average more than DMX_FBU_SPREAD positions (image rows, runs)
        const bool spread = smax > (uint32_t)DMX_FBU_SPREAD * NW;
        if (spread) {
            Gw[t] = w;
            Go[t] = go;
            Gk[t] = (uint8_t)gk;
            if (t == 0) Go[FBR_NT] = bend;
        }
        if (isst && L) {
            const uint32_t k = atomicAdd(&nst, 1u);
            slist[k][0] = go;
            slist[k][1] = L;
            slist[k][2] = ti + 1 < n ? tk[ti + 1] : 0u;
        }
        __syncthreads();
        const uint32_t ns = nst;
        stamp(0);
        while (pstart < bend) {
            const uint32_t pe = min(pstart + FBU_PS, bend);  // this batch's part of the piece
            if (!spread) {
                // short tokens: one per lane
                const uint32_t lo = max(go, pstart), hi = min(gend, pe);
                if (gk == FBU_LIT) {
                    for (uint32_t x = lo; x < hi; x++) C[x - pstart] = FBR_FINAL | ((w >> (8 * (x - go))) & 0xFF);
                } else if (gk == FBU_MATCH && lo < hi) {
                    uint32_t rr = lo - go;
                    if (rr >= d) rr %= d;
                    for (uint32_t x = lo; x < hi; x++) {
                        const uint32_t src = go + rr - d;  // as signed: the source position
                        C[x - pstart] = (int32_t)src >= 0 ? src : (FBR_FINAL | 0x8000u | (uint32_t)(-(int32_t)src - 1));
                        if (++rr == d) rr = 0;
                    }
                }
            } else {
                // long tokens (a lane per token would wait for the longest): the batch's part of
                // the piece spread evenly over the workgroup; a thread finds the token of its
                // first position by binary search over the batch's offsets and walks on
                const uint32_t a0 = max(pstart, obase);
                const uint32_t cs = (pe - a0 + FBR_NT - 1) / FBR_NT;
                uint32_t x = a0 + t * cs;
                const uint32_t x1 = min(x + cs, pe);
                if (x < x1) {
                    uint32_t lo = 0, hi = FBR_NT;  // the last k with Go[k] <= x (it has output)
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (Go[mid] <= x) lo = mid;
                        else hi = mid;
                    }
                    uint32_t k = lo;
                    while (x < x1) {
                        const uint32_t tw = Gw[k], tgo = Go[k], tend = Go[k + 1], kind = Gk[k];
                        const uint32_t e = min(tend, x1);
                        if (kind == FBU_LIT) {
                            for (; x < e; x++) C[x - pstart] = FBR_FINAL | ((tw >> (8 * (x - tgo))) & 0xFF);
                        } else if (kind == FBU_MATCH) {
                            const uint32_t td = (tw & 0x7FFFu) + 1;
                            uint32_t rr = x - tgo;  // nonzero only in the first token of the range
                            if (rr >= td) rr %= td;
                            for (; x < e; x++) {
                                const uint32_t src = tgo + rr - td;  // as signed: the source position
                                C[x - pstart] = (int32_t)src >= 0 ? src : (FBR_FINAL | 0x8000u | (uint32_t)(-(int32_t)src - 1));
                                if (++rr == td) rr = 0;
                            }
                        } else {
                            x = e;  // a stored block (copied below), or no output
                        }
                        k++;
                    }
                }
            }
            for (uint32_t q = 0; q < ns; q++) {
                const uint32_t o = slist[q][0], len = slist[q][1];
                const uint32_t a = max(o, pstart), b = min(o + len, pe);
                const uint8_t* src = sbase + slist[q][2] + (a - o);
                for (uint32_t j = t; a + j < b; j += FBR_NT) C[a + j - pstart] = FBR_FINAL | src[j];
            }
            if (pe - pstart < FBU_PS && pe < usize) break;  // the piece goes on in the next batch
            finish_piece(pe - pstart);
        }
        __syncthreads();
        stamp(1);
        if (t == 0) nst = 0;
        obase = bend;
        w = wn;
        wp = wpn;
    }
    if (__syncthreads_or(bad || open) && t == 0) atomicOr(A.err, 1u);
}

// ---------------------------------------------------------------------------------------
// k_fb_tails: the serial window hand-off.  One workgroup; for every unit on the chain, in
// order, the markers of its last min(size, 32 KiB) entries are resolved against the last
// 32 KiB of output before it (kept in LDS), the bytes go to the output, and the window moves.
// The image entries of unit k + 1's tail are loaded into registers (32 per thread) while unit
// k is resolved, so the chain of units pays the HBM latency once, not once per unit.
// ---------------------------------------------------------------------------------------
constexpr int FB_TNT = 1024;
constexpr int FB_TPT = FB_RING / FB_TNT;  // tail entries per thread
__global__ __launch_bounds__(FB_TNT) void k_fb_tails(const uint16_t* __restrict__ img,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint64_t* __restrict__ sizes,
                                                     uint64_t nchain, uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t win[2][FB_RING];
    const uint32_t t = threadIdx.x;
    uint32_t cur = 0;
    for (uint32_t i = t; i < FB_RING; i += FB_TNT) win[0][i] = 0;
    // entry i of a tail is held by thread i % FB_TNT, slot i / FB_TNT
    struct Tail {
        uint64_t off, s;
        uint32_t v[FB_TPT];
    };
    auto load_tail = [&](uint64_t k, Tail& T) {
        if (k >= nchain) return;
        T.off = offs[k];
        T.s = sizes[k];
        const uint32_t tl = (uint32_t)min(T.s, (uint64_t)FB_RING);
        const uint16_t* src = img + T.off + (T.s - tl);
        uint32_t tq = t;  // opaque copy: the 32 indices are not hoisted out of the loop (spills)
        asm volatile("" : "+v"(tq));
#pragma unroll
        for (int j = 0; j < FB_TPT; j++) {
            const uint32_t i = tq + FB_TNT * j;
            T.v[j] = src[i < tl ? i : 0u];  // unconditional (the image has 8 spare entries)
        }
    };
    Tail ta, tb;
    load_tail(0, ta);
    __syncthreads();
    auto resolve = [&](const Tail& T) {
        const uint64_t off = T.off, s = T.s;
        const uint32_t tl = (uint32_t)min(s, (uint64_t)FB_RING);
        const uint64_t x0 = s - tl;  // first tail entry (unit-relative)
        const uint8_t* W = win[cur];
        uint8_t* N = win[cur ^ 1];
        // carry the part of the old window that stays (units shorter than the window)
        for (uint32_t i = t; i < FB_RING - tl; i += FB_TNT) N[i] = W[i + tl];
        uint32_t tq = t;
        asm volatile("" : "+v"(tq));
        // all window reads first (unconditional, so they pipeline), then the stores
        uint32_t bv[FB_TPT];
#pragma unroll
        for (int j = 0; j < FB_TPT; j++) {
            const uint32_t e = T.v[j];
            const uint32_t w = W[FB_RING - 1 - (e & 0x7FFFu)];
            bv[j] = e < 0x8000u ? e : w;
        }
#pragma unroll
        for (int j = 0; j < FB_TPT; j++) {
            const uint32_t i = tq + FB_TNT * j;
            if (i < tl) {
                out[off + x0 + i] = (uint8_t)bv[j];
                N[FB_RING - tl + i] = (uint8_t)bv[j];
            }
        }
        __syncthreads();
        cur ^= 1;
    };
    // two units per iteration, the register sets swapping roles
    for (uint64_t k = 0; k < nchain; k += 2) {
        load_tail(k + 1, tb);
        resolve(ta);
        if (k + 1 >= nchain) break;
        load_tail(k + 2, ta);
        resolve(tb);
    }
}

// ---------------------------------------------------------------------------------------
// Parallel window hand-off (replaces k_fb_tails when the chain has < 65536 units).
// Window k is the last FB_RING output positions before the end of unit k on the chain:
// W[k * FB_RING + i] is output position uend_k - FB_RING + i, as a 32-bit entry that is either
// a byte (bit 31 set) or the index of another window entry holding the same byte -- always in
// window k - 1 or earlier, so the references form a forest rooted at bytes:
//   k_fb_win_init   entries from the 16-bit image: a byte; a marker "b before unit k" -> entry
//                   FB_RING - b of window k - 1; a position before unit k's start (short units)
//                   -> the same position in window k - 1.
//   k_fb_win_jump   pointer jumping, up to FB_HOPS hops per entry per round, in place (an
//                   entry only ever moves further along its chain); a round that finds nothing
//                   unresolved lets every later round return at once.  The chain depth is at
//                   most the unit count, so ceil(log2(units)) + 1 rounds always suffice.
//   k_fb_final      every output byte: an image byte, or its marker's window entry.
// ---------------------------------------------------------------------------------------
constexpr uint32_t FB_WLIT = 0x80000000u;
#ifndef DMX_FB_HOPS
#define DMX_FB_HOPS 8
#endif
constexpr int FB_HOPS = DMX_FB_HOPS;
#ifndef DMX_FB_WIN_ROUNDS
#define DMX_FB_WIN_ROUNDS 2
#endif
constexpr uint32_t FB_WIN_ROUNDS = DMX_FB_WIN_ROUNDS;  // jump rounds launched (k_fb_final finishes the chains)
constexpr uint32_t FB_WIN_BLK = 4096;  // window entries per k_fb_win_init workgroup
__global__ __launch_bounds__(256) void k_fb_win_init(const uint16_t* __restrict__ img,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint64_t* __restrict__ sizes,
                                                     uint32_t* __restrict__ W) {
    const uint64_t k = blockIdx.x;
    const uint64_t uoff = offs[k], uend = uoff + sizes[k];
    const uint64_t wk = k * FB_RING;
    for (uint32_t i = blockIdx.y * FB_WIN_BLK + threadIdx.x; i < (blockIdx.y + 1) * FB_WIN_BLK; i += 256) {
        uint32_t v = FB_WLIT;  // before the stream start: never referenced by a valid stream
        if (uend + i >= FB_RING) {
            const uint64_t x = uend + i - FB_RING;
            if (x >= uoff) {
                const uint32_t e = img[x];
                if (e < 0x8000u) v = FB_WLIT | e;
                else if (k > 0) v = (uint32_t)(wk - FB_RING + FB_RING - 1 - (e & 0x7FFFu));
            } else {
                v = (uint32_t)(wk - FB_RING + (x + FB_RING - uoff));
            }
        }
        W[wk + i] = v;
    }
}

// Four entries per thread at a time: their hops are independent gathers, issued together.
__global__ __launch_bounds__(256) void k_fb_win_jump(uint32_t* W, uint64_t nent, uint32_t* open, int round) {
    if (round > 0 && __builtin_nontemporal_load(&open[round - 1]) == 0) return;
    bool left = false;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; i0 < nent; i0 += 4 * stride) {
        uint32_t v[4];
        bool in[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t i = i0 + k * stride;
            in[k] = i < nent;
            v[k] = in[k] ? W[i] : FB_WLIT;
        }
        const bool todo = !((v[0] & v[1] & v[2] & v[3]) & FB_WLIT);
        if (!todo) continue;
        bool chg[4];
#pragma unroll
        for (int k = 0; k < 4; k++) chg[k] = !(v[k] & FB_WLIT);
#pragma unroll 1
        for (int h = 0; h < FB_HOPS; h++) {
            uint32_t nv[4];
#pragma unroll
            for (int k = 0; k < 4; k++) nv[k] = W[(v[k] & FB_WLIT) ? 0u : v[k]];  // (entry 0: a valid index)
            bool open_k = false;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                v[k] = (v[k] & FB_WLIT) ? v[k] : nv[k];
                open_k |= !(v[k] & FB_WLIT);
            }
            if (!open_k) break;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (chg[k]) W[i0 + k * stride] = v[k];
            left |= in[k] && !(v[k] & FB_WLIT);
        }
    }
    if (__ballot(left) && lane_id() == 0) atomicOr(&open[round], 1u);
}

// ---------------------------------------------------------------------------------------
// k_fb_final: every entry (W != nullptr) or every entry before its unit's tail (after
// k_fb_tails).  One workgroup per FB_FIN_SPAN entries; the unit of the span's first entry is
// found by binary search over the chain offsets.
// ---------------------------------------------------------------------------------------
constexpr uint32_t FB_FIN_SPAN = 16384;
__global__ __launch_bounds__(256) void k_fb_final(const uint16_t* img, const uint64_t* offs,
                                                  const uint64_t* sizes, uint64_t nchain,
                                                  uint64_t total, const uint32_t* W, uint8_t* out,
                                                  uint32_t* err) {
    const uint64_t s0 = (uint64_t)blockIdx.x * FB_FIN_SPAN;
    if (s0 >= total) return;
    const uint64_t s1 = min(total, s0 + FB_FIN_SPAN);
    uint64_t lo = 0, hi = nchain;  // last unit with offs <= s0
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (offs[mid] <= s0) lo = mid;
        else hi = mid;
    }
    uint64_t k = lo;
    uint64_t uoff = offs[k], uend = uoff + sizes[k];
    if (W) {
        // four entries per thread at a time, 256 apart (a wave's image loads, window reads and
        // stores stay contiguous), their window reads issued together
        for (uint64_t x0 = s0 + threadIdx.x; x0 < s1; x0 += 4 * 256) {
            uint32_t e[4], wi[4];
#pragma unroll
            for (int j = 0; j < 4; j++) e[j] = x0 + 256 * j < s1 ? img[x0 + 256 * j] : 0u;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint64_t x = x0 + 256 * j;
                while (x >= uend && x < s1) {
                    k++;
                    uoff = offs[k];
                    uend = uoff + sizes[k];
                }
                // a marker's window entry (a marker before the stream start was flagged)
                wi[j] = e[j] >= 0x8000u && k > 0 ? (uint32_t)(k * FB_RING - ((e[j] & 0x7FFFu) + 1)) : 0xFFFFFFFFu;
            }
            uint32_t wv[4];
#pragma unroll
            for (int j = 0; j < 4; j++) wv[j] = wi[j] == 0xFFFFFFFFu ? FB_WLIT : W[wi[j]];
            // an entry the (at most FB_WIN_ROUNDS) jump rounds left open: follow it to its byte
#pragma unroll
            for (int j = 0; j < 4; j++) {  // (entries point strictly back: the walk ends; bounded anyway)
                for (uint32_t h = 0; h < (1u << 20) && !(wv[j] & FB_WLIT); h++) wv[j] = W[wv[j]];
                // the bound reached with the entry still open: no byte to write, so the stream
                // goes to the serial decoder instead
                if (!(wv[j] & FB_WLIT) && x0 + 256 * j < s1) atomicOr(err, 2u);
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (x0 + 256 * j < s1)
                    out[x0 + 256 * j] = e[j] < 0x8000u ? (uint8_t)e[j] : wi[j] != 0xFFFFFFFFu ? (uint8_t)wv[j] : (uint8_t)0;
        }
        return;
    }
    for (uint64_t x = s0 + threadIdx.x; x < s1; x += 256) {
        while (x >= uend) {
            k++;
            uoff = offs[k];
            uend = uoff + sizes[k];
        }
        const uint32_t v = img[x];
        const uint64_t b = (v & 0x7FFFu) + 1;  // a marker before the stream start was flagged
        {
            const uint64_t s = uend - uoff;
            if (x - uoff >= s - min(s, (uint64_t)FB_RING)) continue;  // tail: k_fb_tails wrote it
            out[x] = v < 0x8000u ? (uint8_t)v : (b <= uoff ? out[uoff - b] : (uint8_t)0);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Fixed-code regions: exact token boundaries without scanned block starts.
//
// A run of fixed-code blocks (zlib's Z_FIXED, the reference's own level-1/2 fixed chunks,
// realDecompress's prebuilt trees, inflate.hpp:280-283, 310-312) or one huge block has no
// dynamic header for the scan to find, and a decode that starts off the token path inside it
// need not get back on it: in literal runs of one code length (8-bit codes for bytes < 144)
// every misaligned start stays misaligned.  Guessing starts and repairing them round by round
// therefore does not converge.  Instead the region [E, T) -- from the block header E where the
// unit before it stopped, to the next dynamic-header start T -- is cut into chunks of FBS_CH
// bits, and for every chunk c and entry offset e < 32 (a fixed-code token is at most 31 bits:
// 8-bit length code + 5 extra + 5-bit distance code + 13 extra, so the token path enters every
// chunk within its first 31 bits) one lane decodes from bit c * FBS_CH + e to the first token
// boundary at or past the next chunk: a function from entries to entries.  The true path is
// that function's orbit from E.
//
// Node = (chunk, f, e): f is the BFINAL bit of the fixed block in force.  A lane starting at e
// does not know f; f only matters at the first end of block it meets, so one lane yields both
// nodes' results: with f = 1 the first end of block ends the stream, with f = 0 the next header
// is read.  End of block + the following headers are one token: stored blocks are skipped
// (the lane continues from the chunk their data ends in), BTYPE 3 blocks are empty (the
// reference has no case for them, inflate.hpp:292), a dynamic header ends the lane (a link
// when it is T, else no path), so every boundary is inside a fixed block.
//
// A node's result (32 bits): a next node (region chunk << 6 | f << 5 | e, bit 31 clear) or a
// terminal FBS_END (the final block ended), FBS_LINK (the dynamic header at T follows), FBS_FAIL
// (no valid path: past T, an over-read).  Chunk 0's node 0 is the region head: the block header
// at E (its other nodes are unreachable).
//
//   k_fb_smap   one workgroup per super block of FBS_K chunks (2^18 bits, staged in LDS): the
//               chunk map, then pointer jumping in LDS so that every node of the super block
//               maps to the first node of its path past the super block (or a terminal).
//   k_fb_swalk  one lane per region walks those jumps from the head: one dependent read per
//               super block; the node where the path enters each super block is recorded.
// The host starts one unit per visited super block at that node (FB_V_EXACT, fixed code, f),
// each ending softly at the next one's start: exact starts, so every link holds.
// ---------------------------------------------------------------------------------------
constexpr uint32_t FBS_CH = 4096;             // bits per chunk
constexpr uint32_t FBS_K = 64;                // chunks per super block
constexpr uint32_t FBS_SB = FBS_CH * FBS_K;   // 2^18 bits
constexpr uint32_t FBS_NODES = FBS_K * 64;    // nodes per super block
constexpr uint32_t FBS_SUB = FBS_SUBS;        // sub-chunks per chunk whose entries a lane records
constexpr uint32_t FBS_SUBB = FBS_CH / FBS_SUB;  // 512 bits
constexpr uint64_t FBS_SUB_NONE = (1ull << (5 * (FBS_SUB - 1))) - 1;  // every sub-entry 31 = none
// 512 threads (two chunks of 32 entries per wave, four tasks per thread): 52 KB of LDS leaves
// three workgroups, i.e. 24 waves, per CU (256 threads: 12 -- the lanes are LDS-latency-bound)
constexpr int FBS_NT = 512;
constexpr uint32_t FBS_STG = FBS_SB / 32 + 128;  // staged words: one before the super block, 4 KiB bits after
constexpr uint32_t FBS_TERM = 0x80000000u;
constexpr uint32_t FBS_END = FB_REGION_END, FBS_LINK = FB_REGION_LINK, FBS_FAIL = FBS_TERM | 3u;

struct FbsSmem {
    uint32_t stg[FBS_STG + 2];
    uint32_t lut[512];          // fixed lit/len code by the next 9 stream bits (lit_entry format)
    uint32_t J[FBS_NODES];
};

// 32 bits at stream bit p: from the staged words when they hold them, else from HBM (masked at
// the stream end; a stored block's data can carry a lane far past the staging)
struct FbsBits {
    const uint32_t* stg;
    uint64_t a0;        // aligned-image bit of stg[0]
    const uint32_t* w;  // aligned image
    uint64_t base, nwords, end_bytes;
    __device__ uint32_t word(uint64_t i) const {
        if (i >= nwords) return 0u;
        const uint32_t v = w[i];
        const uint64_t lim = end_bytes - 4 * i;
        return lim >= 4 ? v : v & ((1u << (8 * lim)) - 1u);
    }
    // aligned-image word i: staged when the staging holds it (FBS_STG + 2 words from a0)
    __device__ uint32_t wordx(uint64_t i) const {
        const uint64_t j = i - (a0 >> 5);
        return (i >= (a0 >> 5) && j < FBS_STG + 2) ? stg[j] : word(i);
    }
    __device__ uint32_t peek(uint64_t p) const {
        const uint64_t a = base + p;
        const uint64_t rel = a - a0;
        if (a >= a0 && rel < (uint64_t)(FBS_STG - 1) * 32) {
            const uint32_t i = (uint32_t)(rel >> 5);
            return __builtin_amdgcn_alignbit(stg[i + 1], stg[i], (uint32_t)(rel & 31));
        }
        const uint64_t i = a >> 5;
        return __builtin_amdgcn_alignbit(word(i + 1), word(i), (uint32_t)(a & 31));
    }
};

// One lane: the token path from stream bit p (hstate: p is the region head's block header)
// to the first fixed-code token boundary at or past the next chunk (chunk grid from E).
// *r0 / *r1: the result for entry f = 0 / f = 1.  The stream comes through a 64-bit register
// window holding >= 32 valid bits before every token (a fixed-code token is <= 31 bits), so a
// token costs one table read: literal or match by selects, the distance code from the same
// window.  (Round 5 re-read the stream per token, 2 + 2 LDS reads and 64-bit address math.)
__device__ void fbs_lane(const FbsBits& B, const uint32_t* lut, uint64_t p, bool hstate, uint64_t E,
                         uint64_t T, uint64_t nbits, uint32_t* r0, uint32_t* r1, uint64_t* subs) {
    uint64_t target = p - ((p - E) % FBS_CH) + FBS_CH;
    // sub-chunk entries: the first token boundary at or past each FBS_SUBB-bit mark of the chunk
    // (5 bits each: a token is <= 31 bits, so it is < 31 bits past the mark; 31 = not recorded)
    uint64_t sub_at = target - FBS_CH + FBS_SUBB, sb = FBS_SUB_NONE;
    uint32_t sk = 0;
    bool eob_seen = false;  // an end of block met with f unknown: the f = 1 entry ended there
    bool hdr = hstate;      // a header is next
    uint32_t fcur = 0;      // BFINAL of the last header read (valid once one was read)
    bool hdr_read = false;
    uint32_t res = 0;
    uint64_t w = 0, wi = 0;  // window: the bits from p on (nb valid), next word to load
    uint32_t nb = 0;
    auto seek = [&](uint64_t q) {
        const uint64_t a = B.base + q;
        wi = a >> 5;
        const uint32_t sh = (uint32_t)(a & 31);
        w = (((uint64_t)B.wordx(wi + 1) << 32) | B.wordx(wi)) >> sh;
        nb = 64 - sh;
        wi += 2;
    };
    seek(p);
    for (;;) {
        if (nb < 32) {
            w |= (uint64_t)B.wordx(wi) << nb;
            nb += 32;
            wi++;
        }
        if (hdr) {
            // block headers up to the next fixed block (stored data skipped, BTYPE 3 empty)
            if (p >= T || p + 3 > nbits) { res = (p == T && T < nbits) ? FBS_LINK : FBS_FAIL; break; }
            const uint32_t h = (uint32_t)w & 7u;
            const uint32_t bfinal = h & 1u, btype = h >> 1;
            if (btype == 2) { res = FBS_FAIL; break; }  // a dynamic header before T: not scanned
            p += 3;
            w >>= 3;
            nb -= 3;
            hdr_read = true;
            if (btype == 1) {
                fcur = bfinal;
                hdr = false;
                continue;
            }
            if (btype == 0) {
                p = (p + 7) & ~7ull;
                if (p + 32 > nbits) { res = FBS_FAIL; break; }
                const uint32_t len = B.peek(p) & 0xFFFFu;  // NLEN unchecked (inflate.hpp:293-303)
                p += 32 + 8ull * len;
                if (p > nbits) { res = FBS_FAIL; break; }
                seek(p);
            }
            if (bfinal) { res = FBS_END; break; }
            continue;
        }
        // a fixed-code token boundary
        if (p >= T) { res = FBS_FAIL; break; }
        if (p >= target) {
            const uint64_t rel = p - E;
            const uint64_t cc = rel / FBS_CH;
            const uint32_t off = (uint32_t)(rel % FBS_CH);
            if (off < 32) {
                res = (uint32_t)(cc << 6) | (off & 31u);
                break;
            }
            target = E + (cc + 1) * FBS_CH;  // a stored block's data ended deep inside a chunk
        }
        while (p >= sub_at && sk < FBS_SUB - 1) {
            const uint64_t o = p - sub_at;
            if (o < 31) sb = (sb & ~(31ull << (5 * sk))) | (o << (5 * sk));
            sk++;
            sub_at += FBS_SUBB;
        }
        // Fast path: tokens until the next event (T, the chunk target, a sub-chunk mark, the
        // stream end) or an end of block, from the staged words only, without branches: the
        // next word is always loaded one token ahead and merged by selects.  The general loop
        // below (one token per trip, every test, HBM words past the staging) takes the rest.
        {
            uint64_t ev = min(min(T, target), nbits + 1);
            if (sk < FBS_SUB - 1) ev = min(ev, sub_at);
            const uint64_t wb = B.a0 >> 5;  // aligned-image word of stg[0]
            if (p < ev && wi >= wb && wi - wb + 1 < (uint64_t)(FBS_STG + 2)) {
                const uint32_t* const stg = B.stg;
                uint32_t wl = (uint32_t)(wi - wb);
                uint32_t nxt = stg[wl];
                const uint32_t rem0 = (uint32_t)min(ev - p, (uint64_t)0x7FFFFFFF);
                uint32_t used = 0;
                for (;;) {
                    const uint32_t x9 = __builtin_bitreverse32((uint32_t)w) >> 23, x8 = x9 >> 1, x7 = x9 >> 2;
                    const bool c7 = x7 < 0x18u, c8a = (x8 >= 0x30u) & (x8 < 0xC0u), c8b = (x8 >= 0xC0u) & (x8 < 0xC8u);
                    const uint32_t cl = c7 ? 7u : (c8a | c8b) ? 8u : 9u;
                    const uint32_t sym = c7 ? 256u + x7 : c8a ? x8 - 0x30u : c8b ? 280u + x8 - 0xC0u : x9 - 256u;
                    if (sym == 256u) break;  // end of block: the general loop decodes it
                    const bool m = sym > 256u;
                    const uint32_t n1 = cl + (m ? len_extra(sym) : 0u);
                    const uint32_t ds = __builtin_bitreverse32((uint32_t)(w >> n1)) >> 27;
                    const uint32_t n = m ? n1 + 5 + (ds < 30 ? dist_extra(ds) : 0u) : cl;
                    used += n;
                    w >>= n;
                    nb -= n;
                    const bool need = nb < 32;
                    w |= need ? (uint64_t)nxt << nb : 0ull;
                    nb += need ? 32u : 0u;
                    wl += need ? 1u : 0u;
                    nxt = stg[min(wl, FBS_STG + 1)];
                    if (used >= rem0 || wl + 1 >= FBS_STG + 2) break;
                }
                p += used;
                wi = wb + wl;
                if (used) {
                    if (p > nbits) { res = FBS_FAIL; break; }
                    continue;  // the events at p
                }
            }
        }
        // the fixed lit/len code (RFC 1951 3.2.6) by arithmetic on the next 9 bits, MSB-first: no
        // table read on the token's dependency chain (the map is latency-bound)
        const uint32_t x9 = __builtin_bitreverse32((uint32_t)w) >> 23, x8 = x9 >> 1, x7 = x9 >> 2;
        const bool c7 = x7 < 0x18u, c8a = (x8 >= 0x30u) & (x8 < 0xC0u), c8b = (x8 >= 0xC0u) & (x8 < 0xC8u);
        const uint32_t cl = c7 ? 7u : (c8a | c8b) ? 8u : 9u;
        const uint32_t sym = c7 ? 256u + x7 : c8a ? x8 - 0x30u : c8b ? 280u + x8 - 0xC0u : x9 - 256u;
        const uint32_t ty = sym < 256u ? 0u : sym == 256u ? 1u : 2u;
        (void)lut;
        if (ty == 1) {  // end of block
            p += 7;
            w >>= 7;
            nb -= 7;
            if (!hdr_read) eob_seen = true;
            else if (fcur) { res = FBS_END; break; }
            hdr = true;
        } else {  // literal (ty 0) or length (ty 2) + distance, <= 31 bits of the window
            const bool m = ty == 2;
            const uint32_t n1 = cl + (m ? len_extra(sym) : 0u);  // (286 / 287: no extra bits)
            const uint32_t ds = __builtin_bitreverse32((uint32_t)(w >> n1)) >> 27;  // 5-bit distance code
            const uint32_t n = m ? n1 + 5 + (ds < 30 ? dist_extra(ds) : 0u) : cl;
            p += n;
            w >>= n;
            nb -= n;
        }
        if (p > nbits) { res = FBS_FAIL; break; }
    }
    if (!(res & FBS_TERM)) {
        *r0 = res | ((hdr_read ? fcur : 0u) << 5);
        *r1 = eob_seen ? FBS_END : (res | (1u << 5));
    } else {
        *r0 = res;
        *r1 = eob_seen ? FBS_END : res;
    }
    *subs = sb;
}

struct FbsArgs {
    const uint32_t* in_words;
    uint64_t misalign, n;
    const uint64_t* reg;    // per region: E, T, first super block (3 words)
    const uint32_t* sbreg;  // region of each super block
    uint32_t* J;            // FBS_NODES per super block
    uint32_t* visit;        // per super block: the node the path enters it at (~0: none)
    uint32_t* rstat;        // per region: the walk's terminal
    uint32_t nreg;
    uint32_t* Jraw;         // FBS_NODES per super block: the chunk map before pointer jumping
    uint64_t* Jsub;         // FBS_NODES per super block: each node's sub-chunk entries (5 bits each)
    uint64_t* cbit;         // FBS_K * FBS_SUB per super block: the stream bit the path enters each
                            // chunk and sub-chunk at (~0: not entered / not recorded)
};

__global__ __launch_bounds__(FBS_NT) void k_fb_smap(FbsArgs A) {
    __shared__ __attribute__((aligned(16))) FbsSmem S;
    const uint32_t t = threadIdx.x;
    const uint64_t sb = blockIdx.x;
    const uint32_t r = A.sbreg[sb];
    const uint64_t E = A.reg[3 * r], T = A.reg[3 * r + 1], lsb = sb - A.reg[3 * r + 2];
    const uint64_t base = A.misalign * 8;
    const uint64_t end_bytes = A.misalign + A.n, nwords = (end_bytes + 3) / 4, nbits = 8 * A.n;
    const uint64_t b0 = E + lsb * FBS_SB;  // first bit of the super block
    const uint64_t w0 = ((base + b0) >> 5) - ((base + b0) >= 32 ? 1 : 0);
    FbsBits B{S.stg, w0 * 32, A.in_words, base, nwords, end_bytes};
    for (uint32_t i = t; i < FBS_STG + 2; i += FBS_NT) S.stg[i] = B.word(w0 + i);
    for (uint32_t v = t; v < 512; v += FBS_NT) {
        // the fixed lit/len code (RFC 1951 3.2.6) by the next 9 stream bits, MSB-first code x
        const uint32_t x = __builtin_bitreverse32(v) >> 23;
        uint32_t sym, len;
        if ((x >> 2) < 0x18) sym = 256 + (x >> 2), len = 7;
        else if ((x >> 1) >= 0x30 && (x >> 1) <= 0xBF) sym = (x >> 1) - 0x30, len = 8;
        else if ((x >> 1) >= 0xC0 && (x >> 1) <= 0xC7) sym = 280 + (x >> 1) - 0xC0, len = 8;
        else sym = 144 + x - 0x190, len = 9;
        S.lut[v] = lit_entry(sym, len);
    }
    __syncthreads();
    // the chunk map: 32 lanes per chunk, entry e = lane & 31
    const uint32_t e = t & 31;
    for (uint32_t lc = t >> 5; lc < FBS_K; lc += FBS_NT / 32) {
        const uint64_t cc = lsb * FBS_K + lc;
        const uint64_t p = E + cc * FBS_CH + e;
        uint32_t r0 = FBS_FAIL, r1 = FBS_FAIL;
        uint64_t sub = FBS_SUB_NONE;
        if (cc == 0) {
            if (e == 0) fbs_lane(B, S.lut, p, true, E, T, nbits, &r0, &r1, &sub);
            r1 = FBS_FAIL;
        } else if (p < T) {
            fbs_lane(B, S.lut, p, false, E, T, nbits, &r0, &r1, &sub);
        }
        S.J[lc * 64 + e] = r0;
        S.J[lc * 64 + 32 + e] = r1;
        uint64_t* const Js = A.Jsub + sb * FBS_NODES + lc * 64;  // (f only matters past an end of block)
        Js[e] = sub;
        Js[32 + e] = sub;
    }
    __syncthreads();
    // the chunk map itself, for k_fb_schunks (every chunk's entry on the true path)
    uint32_t* const Jr = A.Jraw + sb * FBS_NODES;
    for (uint32_t i = t; i < FBS_NODES; i += FBS_NT) Jr[i] = S.J[i];
    // pointer jumping inside the super block: a path has at most one node per chunk
    const uint32_t lo = (uint32_t)(lsb * FBS_K);  // region chunk of local chunk 0
    for (int round = 0; round < 7; round++) {
        for (uint32_t i = t; i < FBS_NODES; i += FBS_NT) {
            uint32_t v = S.J[i];
            if (v & FBS_TERM) continue;
            const uint32_t c = v >> 6;
            if (c - lo < FBS_K) S.J[i] = S.J[(c - lo) * 64 + (v & 63u)];
        }
        __syncthreads();
    }
    uint32_t* Jg = A.J + sb * FBS_NODES;
    for (uint32_t i = t; i < FBS_NODES; i += FBS_NT) Jg[i] = S.J[i];
}

__global__ __launch_bounds__(64) void k_fb_swalk(FbsArgs A) {
    const uint32_t r = blockIdx.x;
    if (threadIdx.x != 0 || r >= A.nreg) return;
    const uint64_t sb0 = A.reg[3 * r + 2];
    uint32_t node = 0;  // the head: chunk 0, node 0
    A.visit[sb0] = 0;
    for (;;) {
        const uint32_t v = A.J[(sb0 + (node >> 6) / FBS_K) * FBS_NODES + ((node >> 6) % FBS_K) * 64 + (node & 63u)];
        if (v & FBS_TERM) {
            A.rstat[r] = v;
            return;
        }
        A.visit[sb0 + (v >> 6) / FBS_K] = v;
        node = v;
    }
}

// k_fb_schunks: one workgroup per super block follows the true path through its chunks from
// the node it enters at (k_fb_swalk's visit), in the chunk map staged in LDS; cbit gets the
// stream bit of every chunk's entry (~0 where the path does not enter), which k_fb_pdecode uses
// as exact range starts of the region units.
__global__ __launch_bounds__(64) void k_fb_schunks(FbsArgs A, uint64_t nsb) {
    __shared__ uint32_t J[FBS_NODES];
    const uint64_t sb = blockIdx.x;
    if (sb >= nsb) return;
    const uint32_t t = threadIdx.x;
    const uint32_t* const Jr = A.Jraw + sb * FBS_NODES;
    for (uint32_t i = t; i < FBS_NODES; i += 64) J[i] = Jr[i];
    uint64_t* const cb = A.cbit + sb * FBS_K * FBS_SUB;
    for (uint32_t i = t; i < FBS_K * FBS_SUB; i += 64) cb[i] = ~0ull;
    __syncthreads();
    if (t != 0) return;
    const uint32_t r = A.sbreg[sb];
    const uint64_t E = A.reg[3 * r], lsb = sb - A.reg[3 * r + 2];
    uint32_t v = A.visit[sb];
    for (uint32_t k = 0; k < FBS_K && v != ~0u && !(v & FBS_TERM); k++) {
        const uint32_t c = v >> 6;
        if (c / FBS_K != lsb) break;  // the path left the super block
        const uint32_t lc = c % FBS_K;
        const uint64_t c0 = E + (uint64_t)c * FBS_CH;
        cb[lc * FBS_SUB] = c0 + (v & 31u);
        const uint64_t sub = A.Jsub[sb * FBS_NODES + lc * 64 + (v & 63u)];
        for (uint32_t q = 1; q < FBS_SUB; q++) {
            const uint32_t o = (uint32_t)(sub >> (5 * (q - 1))) & 31u;
            if (o < 31) cb[lc * FBS_SUB + q] = c0 + q * FBS_SUBB + o;
        }
        v = J[lc * 64 + (v & 63u)];
    }
}
static_assert(FBS_K * FBS_SUB == FBS_XS, "k_fb_pdecode's exact starts");

uint64_t fb_region_super_bits() { return FBS_SB; }
uint32_t fb_region_entries() { return FBS_K * FBS_SUB; }
uint64_t fb_region_chunk_bits() { return FBS_CH; }
uint32_t fb_region_nodes() { return FBS_NODES; }

hipError_t launch_fb_regions(const uint32_t* in_words, uint64_t misalign, uint64_t n, const uint64_t* reg,
                             uint32_t nreg, const uint32_t* sbreg, uint64_t nsb, uint32_t* J, uint32_t* visit,
                             uint32_t* rstat, uint32_t* Jraw, uint64_t* Jsub, uint64_t* cbit, hipStream_t st) {
    if (!nreg || !nsb) return hipSuccess;
    const FbsArgs A{in_words, misalign, n, reg, sbreg, J, visit, rstat, nreg, Jraw, Jsub, cbit};
    (void)hipMemsetAsync(visit, 0xFF, nsb * 4, st);
    hipLaunchKernelGGL(k_fb_smap, dim3((uint32_t)nsb), dim3(FBS_NT), 0, st, A);
    hipLaunchKernelGGL(k_fb_swalk, dim3(nreg), dim3(64), 0, st, A);
    hipLaunchKernelGGL(k_fb_schunks, dim3((uint32_t)nsb), dim3(64), 0, st, A, nsb);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
uint64_t fb_scan_chunks(uint64_t n) { return (8 * n + FB_SCAN_BITS - 1) / FB_SCAN_BITS; }
uint32_t fb_hits_per_chunk() { return FB_HITS; }

hipError_t launch_fb_scan(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                          uint32_t* counts, uint64_t* hits, uint64_t* offs, uint64_t* nhits,
                          hipStream_t st) {
    const uint64_t nc = fb_scan_chunks(n);
    hipLaunchKernelGGL(k_fb_scan, dim3((uint32_t)nc), dim3(64), 0, st, in_words, misalign, n, counts, hits);
    return launch_scan_u32(counts, offs, nc, nhits, st);
}

hipError_t launch_fb_compact(const uint32_t* in_words, uint64_t misalign, uint64_t n, const uint32_t* counts,
                             const uint64_t* offs, const uint64_t* hits, uint64_t nchunks, uint64_t* list,
                             const uint64_t* pcount, uint64_t max_count, unsigned long long* ph, uint64_t* keep,
                             uint32_t* nkeep, uint32_t keep_cap, hipStream_t st) {
    hipLaunchKernelGGL(k_fb_compact, dim3((uint32_t)((nchunks + 255) / 256)), dim3(256), 0, st,
                       counts, offs, hits, nchunks, list);
    if (max_count) {
        // a wave per DMX_FBC_PER_WAVE candidates: its first 64, then refills as its lanes finish
        const uint32_t g = (uint32_t)((max_count + DMX_FBC_PER_WAVE - 1) / DMX_FBC_PER_WAVE);
        hipLaunchKernelGGL(k_fb_check, dim3(g), dim3(64), 0, st, in_words, misalign, n, list, pcount, ph, keep, nkeep,
                           keep_cap);
    }
    return hipGetLastError();
}

hipError_t launch_fb_decode(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                            const uint64_t* starts, const uint64_t* stops, const uint8_t* vmode,
                            const uint64_t* vhdr, uint64_t nunits, uint64_t u0, uint64_t count,
                            const uint64_t* tokoff, uint32_t* tok, FbUnit* units, uint32_t flags,
                            bool parallel, uint32_t* stats, const uint64_t* cbit, const uint32_t* ucb,
                            hipStream_t st) {
    if (!count) return hipSuccess;
    const FbDecodeArgs A{in_words, misalign, n, starts, stops, vmode, vhdr, nunits, u0, tokoff, tok, units, flags, stats,
                         cbit, ucb};
    if (parallel)
        hipLaunchKernelGGL(k_fb_pdecode, dim3((uint32_t)count), dim3(FBP_NT), 0, st, A);
    else
        hipLaunchKernelGGL(k_fb_decode, dim3((uint32_t)count), dim3(64), 0, st, A);
    return hipGetLastError();
}

uint64_t fb_window_entries(uint64_t nchain) { return nchain < 65536 ? nchain * FB_RING : 0; }
uint32_t fb_window_rounds(uint64_t nchain) {
    uint32_t r = 1;
    while ((1ull << (r - 1)) < nchain) r++;
    return r;
}

hipError_t launch_fb_resolve(const uint8_t* stream, const uint64_t* starts, const uint32_t* chain,
                             const uint64_t* offs, const uint64_t* sizes, uint64_t nchain,
                             const uint64_t* tokoff, const uint32_t* tok, const FbUnit* units,
                             uint16_t* img, uint64_t total, uint8_t* out, uint32_t* err,
                             uint32_t* win, uint32_t* open, bool workgroup, unsigned long long* ph,
                             hipStream_t st) {
    FbReplayArgs R{stream, starts, chain, offs, tokoff, tok, units, img, err, ph};
    if (workgroup)
        hipLaunchKernelGGL(k_fb_units, dim3((uint32_t)nchain), dim3(FBR_NT), 0, st, R);
    else
        hipLaunchKernelGGL(k_fb_replay, dim3((uint32_t)nchain), dim3(64), 0, st, R);
    if (win) {
        const uint64_t nent = fb_window_entries(nchain);
        hipLaunchKernelGGL(k_fb_win_init, dim3((uint32_t)nchain, FB_RING / FB_WIN_BLK), dim3(256), 0, st,
                           img, offs, sizes, win);
        // a few rounds resolve almost every entry (C3: the third finds nothing left); k_fb_final
        // follows the rest to their bytes instead of ceil(log2 units) + 1 early-returning launches
        const uint32_t rounds = std::min<uint32_t>(fb_window_rounds(nchain), FB_WIN_ROUNDS);
        (void)hipMemsetAsync(open, 0, rounds * 4, st);
        // one grid-striding wave of workgroups per round: a round with nothing left returns in
        // microseconds.  (Round 4 ran all rounds in one cooperative launch with a grid barrier
        // between them: on C3 that took 0.36 ms against ~0.2 ms for the separate launches.)
        const uint32_t g = (uint32_t)std::min<uint64_t>((nent + 255) / 256, 1024);
        for (uint32_t r = 0; r < rounds; r++)
            hipLaunchKernelGGL(k_fb_win_jump, dim3(g), dim3(256), 0, st, win, nent, open, (int)r);
    } else {
        hipLaunchKernelGGL(k_fb_tails, dim3(1), dim3(FB_TNT), 0, st, img, offs, sizes, nchain, out);
    }
    const uint64_t nb = (total + FB_FIN_SPAN - 1) / FB_FIN_SPAN;
    if (nb)
        hipLaunchKernelGGL(k_fb_final, dim3((uint32_t)nb), dim3(256), 0, st, img, offs, sizes, nchain, total,
                           (const uint32_t*)win, out, err);
    return hipGetLastError();
}

}  // namespace dmx
