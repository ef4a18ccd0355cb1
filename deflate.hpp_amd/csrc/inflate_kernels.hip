// inflate_kernels.hip -- MI355X (gfx950) INFLATE kernels.
//
// Segment-parallel path (streams made of byte-aligned independent segments, which is what
// libdmx's deflate emits and what any encoder's full-flush points produce):
//   k_marker_count / k_marker_write : find every "00 00 FF FF" (end of an empty stored block)
//                                     -> candidate segment starts, in order
//   k_inflate_segments<CAP>         : one wavefront per candidate, decodes into an LDS window
//                                     (the whole segment output), publishes its size through a
//                                     decoupled look-back, copies LDS -> HBM at its offset
//   k_inflate_validate              : candidate chain check (each segment must end exactly
//                                     where the next candidate starts, up to the BFINAL one)
// General path (any RFC 1951 stream, e.g. zlib's, whose blocks reference earlier blocks):
//   k_inflate_serial                : one wavefront decodes the whole stream with a 64 KiB
//                                     LDS ring window; run once to size, once to write.
//
// Decoding semantics follow the reference inflate exactly (inflate.hpp:226-322, common.hpp
// bit-trie) -- see oracle/inflate_oracle.c for the same rules stated on the CPU:
// first-length-wins code lookup (valid for over-subscribed and incomplete codes), separate
// lit/len and dist code-length loops with overshoot and "16 repeats the last literal length"
// (A-11/A-12; RFC behaviour with DMX_CFG_RFC_STRICT), length symbols 286+ = length 0,
// distance symbols 30+ = distance 0, distance > output so far copies nothing, NLEN unchecked,
// BTYPE 3 = empty block, trailing bytes ignored.
#include "../../include/dmx.h"
#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

constexpr int IF_NT = 64;  // one wavefront per segment decoder
constexpr int IF_STAGE = 512;  // input words staged in LDS per candidate (fits 4 decoders/CU)
constexpr int SEG_CAP = 32768;
constexpr int LUT_L = 9;  // primary lit/len lookup bits (32-bit entries, see lit_entry)
constexpr int LUT_D = 7;  // primary distance lookup bits (32-bit entries, see dist_entry)

struct TreeMeta {
    uint32_t lo[16], hi[16], cnt[16], offs[16];
};

struct Tables {
    uint32_t llut[1 << LUT_L];
    uint32_t dlut[1 << LUT_D];
    uint16_t plut[128];
    uint16_t lsorted[320];
    uint16_t dsorted[320];
    uint16_t psorted[32];
    uint8_t llen[320];
    uint8_t dlen[320];
    uint8_t plen[32];
    TreeMeta lm, dm, pm;
    int fixed_loaded;
};

// ---------------------------------------------------------------------------------------
// wave-uniform LSB-first bit reader over the input in HBM
// ---------------------------------------------------------------------------------------
struct BitIn {
    const uint32_t* w;
    uint64_t nwords, end_bytes, end_bits;
    uint64_t pos;  // bits consumed, relative to the aligned base
    uint64_t buf;  // LSB = next bit
    uint32_t cnt;  // valid bits in buf
    uint64_t wi;   // index of the word held in q0
    uint32_t q0, q1;  // raw words wi, wi + 1 (loaded two refills ahead of use)
    const uint32_t* sw;  // optional LDS copy of words [sws, sws + snw)
    uint64_t sws, snw;

    __device__ void init(const uint32_t* words, uint64_t misalign, uint64_t n) {
        w = words;
        end_bytes = misalign + n;
        end_bits = end_bytes * 8;
        nwords = (end_bytes + 3) / 4;
        sw = nullptr;
        sws = snw = 0;
    }
    __device__ void stage(const uint32_t* lds, uint64_t first, uint64_t count) {
        sw = lds;
        sws = first;
        snw = count;
    }
    // Staged words come from LDS.  Otherwise: unconditional load with a clamped index (no
    // branch, so the wait lands at first use); the decoder state is wave-uniform, so the input
    // is read through the scalar cache (s_load, constant address space).  Scalar loads share
    // lgkmcnt with LDS, so every table lookup also waits for them -- hence the staging.
    __device__ uint32_t raw(uint64_t i) const {
        if (i - sws < snw) return sw[i - sws];
        const __attribute__((address_space(4))) uint32_t* cw =
            (const __attribute__((address_space(4))) uint32_t*)w;
        return cw[i < nwords ? i : nwords - 1];
    }
    __device__ uint32_t mask(uint64_t i) const {  // bytes of word i inside the stream
        if (i >= nwords) return 0u;
        const uint64_t lim = end_bytes - 4 * i;
        return lim >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lim)) - 1u);
    }
    __device__ void refill() {
        if (cnt <= 32) {
            buf |= (uint64_t)(q0 & mask(wi)) << cnt;
            cnt += 32;
            wi++;
            q0 = q1;
            q1 = raw(wi + 1);
        }
    }
    __device__ void seek(uint64_t bitpos) {
        pos = bitpos;
        const uint64_t i = bitpos >> 5;
        buf = (uint64_t)((raw(i) & mask(i)) >> (bitpos & 31));
        cnt = 32 - (uint32_t)(bitpos & 31);
        wi = i + 1;
        q0 = raw(wi);
        q1 = raw(wi + 1);
        refill();
    }
    __device__ void ensure(uint32_t k) {  // k <= 33
        if (cnt < k) refill();
    }
    __device__ uint32_t peek(uint32_t k) const { return (uint32_t)buf & ((1u << k) - 1u); }
    __device__ void consume(uint32_t k) {
        buf >>= k;
        cnt -= k;
        pos += k;
    }
    __device__ uint32_t bits(uint32_t k) {  // k <= 16
        ensure(k);
        const uint32_t v = peek(k);
        consume(k);
        return v;
    }
    __device__ void align() {
        ensure(8);
        consume((8 - (uint32_t)(pos & 7)) & 7);
    }
    __device__ bool over() const { return pos > end_bits; }
    __device__ uint8_t byte_at(uint64_t b) const {  // b relative to the aligned base
        return (uint8_t)(w[b >> 2] >> ((b & 3) * 8));
    }
    __device__ uint32_t window32() {  // the next 32 bits (LSB first)
        ensure(32);
        return (uint32_t)buf;
    }
    __device__ uint64_t abspos() const { return pos; }
};

// ---------------------------------------------------------------------------------------
// canonical tables (reference FlatHuffmanTree::construct, common.hpp:104-145) as
// per-length [lo, hi] code ranges + symbols sorted by (length, value)
// ---------------------------------------------------------------------------------------
__device__ void build_tree(const uint8_t* lens, int nsym, uint16_t* sorted, TreeMeta& m) {
    const int lane = lane_id();
    const uint64_t ltmask = (1ull << lane) - 1ull;
    uint32_t cnt[16];
#pragma unroll
    for (int k = 0; k < 16; k++) cnt[k] = 0;
    for (int c = 0; c < nsym; c += 64) {
        const int s = c + lane;
        const uint32_t L = s < nsym ? lens[s] : 0;
#pragma unroll
        for (int k = 1; k < 16; k++) cnt[k] += __popcll(__ballot(L == (uint32_t)k));
    }
    uint32_t lo[16], offs[16];
    uint32_t code = 0, off = 0;
    lo[0] = 0;
    offs[0] = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
        code = (code + (k > 1 ? cnt[k - 1] : 0)) << 1;
        lo[k] = code;
        offs[k] = off;
        off += cnt[k];
    }
    uint32_t run[16];
#pragma unroll
    for (int k = 0; k < 16; k++) run[k] = 0;
    for (int c = 0; c < nsym; c += 64) {
        const int s = c + lane;
        const uint32_t L = s < nsym ? lens[s] : 0;
        uint32_t dst = 0;
#pragma unroll
        for (int k = 1; k < 16; k++) {
            const uint64_t b = __ballot(L == (uint32_t)k);
            if (L == (uint32_t)k) dst = offs[k] + run[k] + __popcll(b & ltmask);
            run[k] += __popcll(b);
        }
        if (L) sorted[dst] = (uint16_t)s;
    }
    if (lane < 16) {
        uint32_t vlo = 0, vc = 0, vo = 0;
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (lane == k) { vlo = lo[k]; vc = cnt[k]; vo = offs[k]; }
        m.lo[lane] = vlo;
        m.cnt[lane] = vc;
        m.hi[lane] = vlo + vc - 1;
        m.offs[lane] = vo;
    }
    wave_sync();
}

// the reference's lookup rule for key (k, x): the last-inserted code c in [lo_k, hi_k] with
// c == x (mod 2^k) (common.hpp:95-100 overwrites on collision); for prefix codes c == x.
__device__ __forceinline__ bool key_hit(const TreeMeta& m, uint32_t k, uint32_t x, uint32_t* c) {
    if (!m.cnt[k] || x > m.hi[k]) return false;
    const uint32_t cm = x + (((m.hi[k] - x) >> k) << k);
    if (cm < m.lo[k]) return false;
    *c = cm;
    return true;
}

// 32-bit decode entries: bits 0-3 code length, 4-5 class (0 literal, 1 end of block, 2 length),
// 6-9 extra-bit count, 16-31 literal byte / length base / distance base.  Length symbols 286+
// decode as length 0 and distance symbols 30+ as distance 0 (no copy, inflate.hpp:243-270).
__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t len) {
    if (sym < 256) return len | (sym << 16);
    if (sym == 256) return len | (1u << 4);
    if (sym > 285) return len | (2u << 4);
    return len | (2u << 4) | (len_extra(sym) << 6) | (len_base(sym) << 16);
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t ds, uint32_t len) {
    if (ds >= 30) return len;
    return len | (dist_extra(ds) << 6) | (dist_base(ds) << 16);
}

template <int PB, bool DIST>
__device__ void fill_lut32(uint32_t* lut, const TreeMeta& m, const uint16_t* sorted) {
    uint32_t lo[PB + 1], hi[PB + 1], cn[PB + 1], of[PB + 1];
#pragma unroll
    for (int k = 1; k <= PB; k++) {
        lo[k] = m.lo[k];
        hi[k] = m.hi[k];
        cn[k] = m.cnt[k];
        of[k] = m.offs[k];
    }
    for (int wv = lane_id(); wv < (1 << PB); wv += 64) {
        const uint32_t v = bitrev(wv, PB);
        uint32_t idx = 0, len = 0;
#pragma unroll
        for (int k = 1; k <= PB; k++) {
            const uint32_t x = v >> (PB - k);
            if (!len && cn[k] && x <= hi[k]) {
                const uint32_t cm = x + (((hi[k] - x) >> k) << k);
                if (cm >= lo[k]) {
                    idx = of[k] + cm - lo[k];
                    len = k;
                }
            }
        }
        lut[wv] = len ? (DIST ? dist_entry(sorted[idx], len) : lit_entry(sorted[idx], len)) : 0u;
    }
}

// precode LUT: the stored code must also equal the bits read (inflate.hpp:175)
__device__ void fill_prelut(uint16_t* lut, const TreeMeta& m, const uint16_t* sorted) {
    for (int wv = lane_id(); wv < 128; wv += 64) {
        const uint32_t v = bitrev(wv, 7);
        uint16_t e = 0;
        for (int k = 1; k <= 7; k++) {
            uint32_t c;
            const uint32_t x = v >> (7 - k);
            if (key_hit(m, k, x, &c) && c == x) {
                e = (uint16_t)(sorted[m.offs[k] + c - m.lo[k]] | (k << 9));
                break;
            }
        }
        lut[wv] = e;
    }
}

// codes longer than the primary table: test lengths kfrom..15 in order
__device__ __forceinline__ bool slow_decode(const TreeMeta& m, const uint16_t* sorted,
                                            uint32_t peek15, int kfrom, uint32_t* sym,
                                            uint32_t* len) {
    const uint32_t v = bitrev(peek15, 15);
    for (int k = kfrom; k <= 15; k++) {
        uint32_t c;
        if (key_hit(m, k, v >> (15 - k), &c)) {
            *sym = sorted[m.offs[k] + c - m.lo[k]];
            *len = k;
            return true;
        }
    }
    return false;
}

__device__ void load_fixed(Tables& T) {
    const int lane = lane_id();
    for (int s = lane; s < 288; s += 64) T.llen[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
    if (lane < 32) T.dlen[lane] = 5;
    wave_sync();
    build_tree(T.llen, 288, T.lsorted, T.lm);
    build_tree(T.dlen, 32, T.dsorted, T.dm);
    fill_lut32<LUT_L, false>(T.llut, T.lm, T.lsorted);
    fill_lut32<LUT_D, true>(T.dlut, T.dm, T.dsorted);
    wave_sync();
}


// ---------------------------------------------------------------------------------------
// Wave-level dynamic header reader (inflate.hpp:136-224).  Reference mode: the lit/len and
// distance code lengths are two sequences, each with its own count and overshoot (entries keep
// their index as the symbol value), and 16 repeats the last literal length, which starts at 0
// per sequence (A-11, A-12); RFC mode: one sequence, 16 repeats the previous length.  The 64 lanes hold a 2048-bit window of the stream, one word each; every step
// decodes the precode symbol (and its repeat bits) at 64 consecutive bit offsets at once, and
// the true symbol chain is then walked with v_readlane -- a few scalar instructions per code
// length instead of a dependent bit-reader refill + table lookup.
// ---------------------------------------------------------------------------------------
struct BitInWords {  // the words a BitIn reads (LDS-staged range, else HBM), masked at the end
    const uint32_t* sw;
    uint64_t sws, snw;
    const uint32_t* w;
    uint64_t nwords, end_bytes;
    __device__ uint32_t word(uint64_t i) const {
        if (i >= nwords) return 0u;
        const uint32_t v = i - sws < snw ? sw[i - sws] : w[i];
        const uint64_t lim = end_bytes - 4 * i;
        return lim >= 4 ? v : v & ((1u << (8 * lim)) - 1u);
    }
};
struct StagedWords {  // words [ws, ws + nw) staged in LDS (already masked)
    const uint32_t* w;
    uint64_t ws, nw;
    __device__ uint32_t word(uint64_t i) const { return (i >= ws && i < ws + nw) ? w[i - ws] : 0u; }
};
__device__ __forceinline__ BitInWords reader_words(const BitIn& br) {
    return BitInWords{br.sw, br.sws, br.snw, br.w, br.nwords, br.end_bytes};
}

// Wave-uniform bit reader over a candidate staged whole in LDS (words [ws, ws + nw), masked at
// the stream end, zero-padded): a 32-bit relative position and one ds_read2 + alignbit per
// 32-bit window, instead of BitIn's 64-bit buffer and refill bookkeeping.
struct StageReader {
    const uint32_t* w;
    uint64_t ws;
    uint32_t nw;
    uint32_t p;     // bits relative to ws * 32
    uint32_t endp;  // stream end, same origin (clamped)
    uint64_t end_bytes, end_bits;

    __device__ void init(const uint32_t* lds, uint64_t first, uint32_t count, uint64_t misalign, uint64_t n) {
        w = lds;
        ws = first;
        nw = count;
        end_bytes = misalign + n;
        end_bits = end_bytes * 8;
        const uint64_t e = end_bits - first * 32;
        endp = e > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)e;
    }
    __device__ uint32_t window32() const {
        const uint32_t i = p >> 5;
        return __builtin_amdgcn_alignbit(w[i + 1], w[i], p & 31);
    }
    __device__ void ensure(uint32_t) {}
    __device__ void consume(uint32_t k) { p += k; }
    __device__ uint32_t bits(uint32_t k) {
        const uint32_t v = window32() & ((1u << k) - 1u);
        p += k;
        return v;
    }
    __device__ void align() { p = (p + 7) & ~7u; }
    __device__ bool over() const { return p > endp; }
    __device__ uint64_t abspos() const { return ws * 32 + p; }
    __device__ void seek(uint64_t abs) { p = (uint32_t)(abs - ws * 32); }
    __device__ uint8_t byte_at(uint64_t b) const {
        const uint32_t r = (uint32_t)(b - ws * 4);
        return (uint8_t)(w[r >> 2] >> ((r & 3) * 8));
    }
    __device__ StagedWords words() const { return StagedWords{w, ws, nw}; }
};

__device__ __forceinline__ StagedWords reader_words(const StageReader& br) { return br.words(); }

// 32 bits at window bit b; every lane passes its own b (all lanes must be active)
__device__ __forceinline__ uint32_t win_bits(uint32_t win, uint32_t b) {
    const int i = (int)(b >> 5);
    const uint32_t lo = __shfl(win, i), hi = __shfl(win, i + 1);
    return __builtin_amdgcn_alignbit(hi, lo, b & 31);
}
__device__ __forceinline__ uint32_t win_bits_u(uint32_t win, uint32_t b) {  // b wave-uniform
    const int i = (int)(b >> 5);
    const uint32_t lo = __builtin_amdgcn_readlane(win, i), hi = __builtin_amdgcn_readlane(win, i + 1);
    return __builtin_amdgcn_alignbit(hi, lo, b & 31);
}

template <class Src>
__device__ uint32_t fast_header(const Src& src, uint64_t* pos_io, uint64_t end_bits, Tables& T,
                                bool rfc, bool fill, uint64_t* stamps = nullptr) {
    const int lane = lane_id();
    uint64_t t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
#define FH_STAMP(k)                                              \
    if (stamps) {                                                \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();        \
        stamps[k] += t1 - t0;                                    \
        t0 = t1;                                                 \
    }
    uint64_t w0 = *pos_io >> 5;
    uint32_t rp = (uint32_t)(*pos_io & 31);
    uint32_t win = src.word(w0 + lane);
    const uint32_t h = win_bits_u(win, rp);
    const uint32_t hlit = h & 31, hdist = (h >> 5) & 31, hclen = (h >> 10) & 15;
    rp += 14;
    const uint32_t pv = win_bits(win, rp + 3 * (uint32_t)(lane < 19 ? lane : 0)) & 7;
    if (lane < 32) T.plen[lane] = 0;
    wave_sync();
    if (lane < (int)hclen + 4) T.plen[kPerm[lane]] = (uint8_t)pv;
    rp += 3 * (hclen + 4);
    if (w0 * 32 + rp > end_bits) return SEGF_OVERREAD;
    wave_sync();
    build_tree(T.plen, 19, T.psorted, T.pm);
    fill_prelut(T.plut, T.pm, T.psorted);
    wave_sync();
    FH_STAMP(0);
    const uint32_t na = 257 + hlit, nd = 1 + hdist;
    const uint32_t cap = rfc ? na + nd : 300;
    uint32_t target = rfc ? na + nd : na;
    uint32_t seq = 0, i = 0, last = 0, nl = 0, ndd = 0;
    for (;;) {
        if (rp + 64 + 46 > 2048) {  // keep 64 offsets + 46 bits of lookahead in the window
            w0 += rp >> 5;
            rp &= 31;
            win = src.word(w0 + lane);
        }
        const uint32_t v = win_bits(win, rp + lane);
        const uint32_t e = T.plut[v & 127];
        const uint32_t sym = e & 511, len = e >> 9;
        const uint32_t ex = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
        const uint32_t xv = (v >> len) & ((1u << ex) - 1u);
        const uint32_t rep_l = sym < 16 ? 1u : sym == 18 ? 11u + xv : 3u + xv;
        const uint32_t tl = e ? len + ex : 0u;  // symbol + repeat bits; 0 = no precode symbol
        const uint64_t end_rel64 = end_bits > w0 * 32 ? end_bits - w0 * 32 : 0;
        const uint32_t end_rel = end_rel64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)end_rel64;
        // serial part: the chain of true symbol starts in this window (one readlane per symbol)
        uint64_t M = 0;
        uint32_t p = 0;
        while (p < 64) {
            M |= 1ull << p;
            const uint32_t t = __builtin_amdgcn_readlane(tl, p);
            if (!t) break;  // no precode symbol: reported below if it is reached
            p += t;
        }
        // parallel part, in chain order: run index (prefix sum of repeats), sequence switch and
        // end, the value a 16 repeats, errors, then the writes
        const bool onp = (M >> lane) & 1ull;
        const uint64_t below = (1ull << lane) - 1ull;
        const uint32_t rep = onp && e ? rep_l : 0u;
        const uint32_t incl = wave_incl_scan(rep);
        const uint32_t excl = incl - rep;
        const uint64_t sw = __ballot(onp && i + incl >= target);
        int b1 = sw ? __builtin_ctzll(sw) : 64;  // first lane that completes the current sequence
        int endl = 64;                           // last processed lane (64: the window continues)
        int b2 = 64;
        uint32_t incl_b1 = b1 < 64 ? __builtin_amdgcn_readlane(incl, b1) : 0u;
        const bool switching = !rfc && seq == 0 && b1 < 64;
        if (b1 < 64) {
            if (!switching) {
                endl = b1;
            } else {  // reference mode: the distance lengths start after lane b1
                const uint64_t sw2 = __ballot(onp && lane > b1 && incl - incl_b1 >= nd);
                b2 = sw2 ? __builtin_ctzll(sw2) : 64;
                if (b2 < 64) endl = b2;
            }
        }
        const bool proc = onp && lane <= endl;
        const bool in2 = switching && lane > b1;          // lane belongs to the distance sequence
        const uint32_t idx = in2 ? excl - incl_b1 : i + excl;
        const uint32_t sq = in2 ? 1u : seq;
        // value a 16 repeats: the nearest earlier lane of the same sequence that sets "last"
        // (reference: literal lengths only; RFC: any non-16 symbol), else the carried value
        const uint32_t symv = sym < 16 ? sym : 0u;
        const uint64_t qual = __ballot(onp && (rfc ? sym != 16 : sym < 16));
        const uint64_t seq2m = switching ? ~((2ull << b1) - 1ull) : ~0ull;  // distance-sequence lanes
        const uint64_t qb = (in2 ? qual & seq2m : qual) & below;
        const uint32_t src = qb ? 63u - (uint32_t)__builtin_clzll(qb) : 0u;
        const uint32_t qv = (uint32_t)__shfl((int)symv, (int)src, 64);
        const uint32_t lastv = qb ? qv : (in2 ? 0u : last);
        const uint32_t val = sym < 16 ? sym : sym == 16 ? lastv : 0u;
        // errors, in the reference's order per symbol (inflate.hpp:166-206)
        uint32_t lerr = 0;
        if (proc) {
            if (!e) lerr = SEGF_ERR_DATA;
            else if (sym == 16 && rfc && idx == 0) lerr = SEGF_ERR_DATA;
            else if (rp + (uint32_t)lane + tl > end_rel) lerr = SEGF_OVERREAD;
            else if (idx + rep_l > cap && (rfc || val != 0)) lerr = SEGF_ERR_DATA;
        }
        const uint64_t em = __ballot(lerr != 0);
        const uint32_t err = em ? __builtin_amdgcn_readlane(lerr, __builtin_ctzll(em)) : 0u;
        // writes: entries idx < cap keep the value (reference: overshoot entries keep their index
        // as the symbol value); long runs are written by the whole wave
        const bool mine = proc && e;
        const bool longr = mine && rep_l > 8;
        if (mine && !longr) {
            for (uint32_t jj = 0; jj < rep_l; jj++) {
                const uint32_t k = idx + jj;
                if (k < cap) {
                    if (!rfc) (sq ? T.dlen : T.llen)[k] = (uint8_t)val;
                    else if (k < na) T.llen[k] = (uint8_t)val;
                    else T.dlen[k - na] = (uint8_t)val;
                }
            }
        }
        uint64_t lm = __ballot(longr);
        while (lm) {
            const int l = __builtin_ctzll(lm);
            lm &= lm - 1;
            const uint32_t il = __builtin_amdgcn_readlane(idx, l);
            const uint32_t vl = __builtin_amdgcn_readlane(val, l);
            const uint32_t rl = __builtin_amdgcn_readlane(rep_l, l);
            const uint32_t ql = __builtin_amdgcn_readlane(sq, l);
            for (uint32_t jj = lane; jj < rl; jj += 64) {
                const uint32_t k = il + jj;
                if (k < cap) {
                    if (!rfc) (ql ? T.dlen : T.llen)[k] = (uint8_t)vl;
                    else if (k < na) T.llen[k] = (uint8_t)vl;
                    else T.dlen[k - na] = (uint8_t)vl;
                }
            }
        }
        if (err) return err;
        // carry to the next window
        const uint64_t procm = __ballot(proc);
        const int lastl = 63 - __builtin_clzll(procm);  // last processed lane (lane 0 always is)
        const uint32_t inc_last = __builtin_amdgcn_readlane(incl, lastl);
        const uint64_t qp = qual & procm & seq2m;  // setters in the sequence that continues
        if (rfc) {
            last = __builtin_amdgcn_readlane(val, lastl);
        } else if (qp) {
            last = __builtin_amdgcn_readlane(symv, 63 - __builtin_clzll(qp));
        } else if (switching) {
            last = 0;
        }
        if (endl < 64) {  // the header ends inside this window
            if (rfc) {
                nl = na;
                ndd = nd;
            } else if (switching) {
                nl = min(i + incl_b1, 300u);
                ndd = min(inc_last - incl_b1, 300u);
            } else {
                ndd = min(i + inc_last, 300u);
            }
            rp += (uint32_t)endl + __builtin_amdgcn_readlane(tl, endl);
            break;
        }
        if (switching) {
            nl = min(i + incl_b1, 300u);
            seq = 1;
            target = nd;
            i = inc_last - incl_b1;
        } else {
            i += inc_last;
        }
        rp += p;
    }
    if (rfc) {
        nl = na;
        ndd = nd;
    }
    *pos_io = w0 * 32 + rp;
    wave_sync();
    FH_STAMP(1);
    build_tree(T.llen, nl, T.lsorted, T.lm);
    build_tree(T.dlen, ndd, T.dsorted, T.dm);
    wave_sync();
    FH_STAMP(2);
    if (fill) {
        fill_lut32<LUT_L, false>(T.llut, T.lm, T.lsorted);
        fill_lut32<LUT_D, true>(T.dlut, T.dm, T.dsorted);
    }
    wave_sync();
    FH_STAMP(3);
#undef FH_STAMP
    return 0;
}

// periodic LZ77 copy: out[pos + i] = out[pos - dist + (i mod dist)], i < L (equal to the
// reference's byte-serial overlapping copy, inflate.hpp:268-270); every source byte lies
// before pos, so all lanes copy independently.
// Four independent byte reads per lane are issued before the writes (one LDS latency per
// 256 bytes); the modulo bookkeeping needs a division only for distances below 64.
template <uint32_t MASK>
__device__ __forceinline__ void lz_copy_lds(uint8_t* win, uint32_t pos, uint32_t L, uint32_t dist) {
    const uint32_t lane = lane_id();
    const uint32_t src = pos - dist;
    if (dist >= L) {
        for (uint32_t i0 = 0; i0 < L; i0 += 256) {
            uint8_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + u * 64 + lane;
                v[u] = i < L ? win[(src + i) & MASK] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + u * 64 + lane;
                if (i < L) win[(pos + i) & MASK] = v[u];
            }
        }
    } else {
        uint32_t r = dist >= 64 ? lane : lane % dist;
        const uint32_t step = dist >= 64 ? 64 : 64 % dist;
        for (uint32_t i0 = 0; i0 < L; i0 += 256) {
            uint8_t v[4];
            uint32_t rr[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                rr[u] = r;
                r += step;
                if (r >= dist) r -= dist;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + u * 64 + lane;
                v[u] = i < L ? win[(src + rr[u]) & MASK] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + u * 64 + lane;
                if (i < L) win[(pos + i) & MASK] = v[u];
            }
        }
    }
}

// output sink of the segment-parallel path: the segment's bytes in LDS
struct SegSink {
    uint8_t* win;
    uint32_t pos;
    bool stream_start;
    uint32_t err;
    __device__ bool literal(uint32_t b) {
        if (pos >= SEG_CAP) { err |= SEGF_OVERFLOW; return false; }
        if (lane_id() == 0) win[pos] = (uint8_t)b;
        pos++;
        return true;
    }
    __device__ bool copy(uint32_t L, uint32_t dist) {
        if (L == 0 || dist == 0) return true;
        if (dist > pos) {
            if (stream_start) return true;  // reference: nothing to copy
            err |= SEGF_XREF;
            return false;
        }
        if (pos + L > SEG_CAP) { err |= SEGF_OVERFLOW; return false; }
        lz_copy_lds<0xFFFFFFFFu>(win, pos, L, dist);
        pos += L;
        return true;
    }
    template <class BR>
    __device__ bool stored(const BR& br, uint64_t b0, uint32_t len) {
        if (pos + len > SEG_CAP) { err |= SEGF_OVERFLOW; return false; }
        for (uint32_t i = lane_id(); i < len; i += 64) win[pos + i] = br.byte_at(b0 + i);
        pos += len;
        return true;
    }
};

// output sink of the serial path: 64 KiB LDS ring window + the output in HBM
struct RingSink {
    uint8_t* ring;
    uint64_t pos;
    uint8_t* out;
    uint64_t cap;
    bool count_only;
    uint32_t err;
    __device__ bool literal(uint32_t b) {
        if (!count_only) {
            if (lane_id() == 0) {
                ring[pos & 0xFFFF] = (uint8_t)b;
                if (pos < cap) out[pos] = (uint8_t)b;
            }
        }
        pos++;
        return true;
    }
    __device__ bool copy(uint32_t L, uint32_t dist) {
        if (L == 0 || dist == 0 || dist > pos) return true;
        if (!count_only) {
            const uint32_t lane = lane_id();
            const uint64_t src = pos - dist;
            uint32_t r = dist >= L ? lane : (dist >= 64 ? lane : lane % dist);
            const uint32_t step = dist >= L ? 64 : (dist >= 64 ? 64 : 64 % dist);
            const bool wrap = dist < L;
            for (uint32_t i = lane; i < L; i += 64) {
                const uint8_t v = ring[(src + r) & 0xFFFF];
                ring[(pos + i) & 0xFFFF] = v;
                if (pos + i < cap) out[pos + i] = v;
                r += step;
                if (wrap && r >= dist) r -= dist;
            }
        }
        pos += L;
        return true;
    }
    template <class BR>
    __device__ bool stored(const BR& br, uint64_t b0, uint32_t len) {
        if (!count_only) {
            for (uint32_t i = lane_id(); i < len; i += 64) {
                const uint8_t v = br.byte_at(b0 + i);
                ring[(pos + i) & 0xFFFF] = v;
                if (pos + i < cap) out[pos + i] = v;
            }
        }
        pos += len;
        return true;
    }
};

// decompressHuffmanBlock (inflate.hpp:226-275) with 32-bit table entries: one 32-bit window
// per half token (code + extra bits), no per-symbol base / extra arithmetic.
template <class BR, class Sink>
__device__ uint32_t decode_huffman(BR& br, const Tables& T, Sink& sk) {
    for (;;) {
        uint32_t v = br.window32();
        uint32_t e = T.llut[v & ((1u << LUT_L) - 1)];
        if (!e) {
            uint32_t sym, len;
            if (!slow_decode(T.lm, T.lsorted, v & 0x7FFF, LUT_L + 1, &sym, &len)) return SEGF_ERR_DATA;
            e = lit_entry(sym, len);
        }
        const uint32_t cl = e & 15, ty = (e >> 4) & 3;
        if (ty == 0) {
            br.consume(cl);
            if (br.over()) return SEGF_OVERREAD;
            if (!sk.literal(e >> 16)) return sk.err;
            continue;
        }
        if (ty == 1) {
            br.consume(cl);
            return br.over() ? SEGF_OVERREAD : 0;
        }
        const uint32_t ex = (e >> 6) & 15;
        const uint32_t L = (e >> 16) + ((v >> cl) & ((1u << ex) - 1u));
        br.consume(cl + ex);
        v = br.window32();
        uint32_t de = T.dlut[v & ((1u << LUT_D) - 1)];
        if (!de) {
            uint32_t ds, dl;
            if (!slow_decode(T.dm, T.dsorted, v & 0x7FFF, LUT_D + 1, &ds, &dl)) return SEGF_ERR_DATA;
            de = dist_entry(ds, dl);
        }
        const uint32_t dl = de & 15, dx = (de >> 6) & 15;
        const uint32_t dist = (de >> 16) + ((v >> dl) & ((1u << dx) - 1u));
        br.consume(dl + dx);
        if (br.over()) return SEGF_OVERREAD;
        if (!sk.copy(L, dist)) return sk.err;
    }
}

// realDecompress (inflate.hpp:277-322).  With stop_at_marker the segment ends at an empty,
// non-final stored block whose NLEN is FFFF (the "00 00 FF FF" the scanner keyed on).
template <class BR, class Sink>
__device__ uint32_t inflate_blocks(BR& br, Tables& T, Sink& sk, bool rfc, bool stop_at_marker,
                                   uint64_t* end_byte, bool* fin, uint64_t* hdr_cycles = nullptr) {
    *fin = false;
    for (;;) {
        br.ensure(3);
        const uint32_t bfinal = br.bits(1);
        const uint32_t btype = br.bits(2);
        if (br.over()) return SEGF_OVERREAD;
        if (btype == 0) {
            br.align();
            br.ensure(32);
            const uint32_t len = br.bits(16);
            const uint32_t nlen = br.bits(16);
            if (br.over()) return SEGF_OVERREAD;
            const uint64_t b0 = br.abspos() >> 3;
            if (stop_at_marker && !bfinal && len == 0 && nlen == 0xFFFF) {
                *end_byte = b0;
                return 0;
            }
            if (b0 + len > br.end_bytes) return SEGF_OVERREAD;
            if (!sk.stored(br, b0, len)) return sk.err;
            br.seek(br.abspos() + 8ull * len);
            wave_sync();
        } else if (btype == 1) {
            if (!T.fixed_loaded) {
                load_fixed(T);
                T.fixed_loaded = 1;
            }
            const uint32_t err = decode_huffman(br, T, sk);
            if (err) return err;
        } else if (btype == 2) {
            T.fixed_loaded = 0;
            const uint64_t h0 = hdr_cycles ? __builtin_amdgcn_s_memtime() : 0;
            uint64_t hp = br.abspos();
            uint32_t err = fast_header(reader_words(br), &hp, br.end_bits, T, rfc, true,
                                       hdr_cycles ? hdr_cycles + 1 : nullptr);
            if (hdr_cycles) *hdr_cycles += __builtin_amdgcn_s_memtime() - h0;
            if (err) return err;
            br.seek(hp);
            err = decode_huffman(br, T, sk);
            if (err) return err;
        }  // btype 3: no-op block (inflate.hpp:292 has no case 3)
        if (bfinal) {
            *fin = true;
            *end_byte = (br.abspos() + 7) >> 3;
            return 0;
        }
    }
}

// ---------------------------------------------------------------------------------------
// marker scan: candidates = {0} U {p : 4 <= p < n, in[p-4..p) == 00 00 FF FF}
// ---------------------------------------------------------------------------------------
constexpr int MK_NT = 256;
constexpr uint64_t MK_TILE = MK_NT * 16;

__device__ __forceinline__ uint32_t mk_word(const uint32_t* w, uint64_t nwords, int64_t i) {
    return (i >= 0 && (uint64_t)i < nwords) ? w[i] : 0u;
}

// marker bitmask for the 16 aligned positions [16g, 16g + 16)
__device__ __forceinline__ uint32_t mk_scan16(const uint32_t* w, uint64_t misalign, uint64_t n,
                                              uint64_t g) {
    const uint64_t nwords = (misalign + n + 3) / 4;
    uint32_t W[5];
    W[0] = mk_word(w, nwords, (int64_t)(4 * g) - 1);
#pragma unroll
    for (int k = 0; k < 4; k++) W[k + 1] = mk_word(w, nwords, (int64_t)(4 * g + k));
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t x = __builtin_amdgcn_alignbyte(W[(i >> 2) + 1], W[i >> 2], i & 3);
        const uint64_t P = 16 * g + i;  // aligned position of the candidate
        const bool ok = x == 0xFFFF0000u && P >= misalign + 4 && P < misalign + n;
        mask |= ok ? (1u << i) : 0u;
    }
    return mask;
}

__global__ __launch_bounds__(MK_NT) void k_marker_count(const uint32_t* w, uint64_t misalign,
                                                        uint64_t n, uint32_t* tile_counts) {
    __shared__ uint32_t red[MK_NT / 64];
    const uint64_t g = (uint64_t)blockIdx.x * MK_NT + threadIdx.x;
    const uint32_t c = __popc(mk_scan16(w, misalign, n, g));
    const uint32_t s = wave_sum(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(MK_NT) void k_marker_write(const uint32_t* w, uint64_t misalign,
                                                        uint64_t n, const uint64_t* tile_offs,
                                                        uint64_t* cands) {
    __shared__ uint32_t part[MK_NT / 64];
    const uint64_t g = (uint64_t)blockIdx.x * MK_NT + threadIdx.x;
    uint32_t mask = mk_scan16(w, misalign, n, g);
    const uint32_t c = __popc(mask);
    const uint32_t inc = wave_incl_scan(c);
    if ((threadIdx.x & 63) == 63) part[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < (int)(threadIdx.x >> 6); i++) base += part[i];
    uint64_t o = 1 + tile_offs[blockIdx.x] + base + inc - c;
    while (mask) {
        const int i = __builtin_ctz(mask);
        mask &= mask - 1;
        cands[o++] = 16 * g + i - misalign;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cands[0] = 0;
}

uint64_t marker_tiles(uint64_t n, uint64_t misalign) {
    return (misalign + n + MK_TILE - 1) / MK_TILE + 0;
}

hipError_t launch_marker_count(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                               uint32_t* tile_counts, uint64_t ntiles, hipStream_t st) {
    hipLaunchKernelGGL(k_marker_count, dim3((uint32_t)ntiles), dim3(MK_NT), 0, st, in_words,
                       misalign, n, tile_counts);
    return hipGetLastError();
}

hipError_t launch_marker_write(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                               const uint64_t* tile_offs, uint64_t ntiles, uint64_t* cands,
                               uint64_t*, hipStream_t st) {
    hipLaunchKernelGGL(k_marker_write, dim3((uint32_t)ntiles), dim3(MK_NT), 0, st, in_words,
                       misalign, n, tile_offs, cands);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// segment-parallel decode with decoupled look-back for the output offsets
// ---------------------------------------------------------------------------------------
constexpr unsigned long long LB_A = 1ull << 62, LB_P = 2ull << 62, LB_V = (1ull << 62) - 1;

__global__ __launch_bounds__(IF_NT) void k_inflate_segments(InflateArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t win[SEG_CAP + 16];
    __shared__ Tables T;
    __shared__ uint32_t stg[IF_STAGE];
    __shared__ unsigned long long s_j, s_excl;
    const int lane = threadIdx.x;
    // dynamic segment index: workgroups that start earlier take earlier segments, so a
    // look-back only ever waits on a workgroup that is already running
    if (lane == 0) s_j = atomicAdd(A.ticket, 1u);
    if (lane == 0) T.fixed_loaded = 0;
    __syncthreads();
    const uint64_t j = s_j;
    if (j >= A.ncand) return;
    if (A.mode == 3 && !(A.recs[j].flags & SEGF_EXOTIC)) return;  // patch pass: declined ones only
    DMX_PHASE(A.dbg, j, 0);
    const uint64_t start = A.cands[j];
    uint64_t hdr_cycles[5] = {0, 0, 0, 0, 0};

    // stage IF_STAGE - 2 words from the candidate on in LDS (masked at the stream end, two zero
    // words after).  When the next candidate lies inside the stage the segment is read by
    // StageReader; if that read ever came within 32 bits of the stage end (a false marker made
    // the segment look short), or the segment is long, it is read by BitIn.
    const uint64_t end_bytes = A.misalign + A.n;
    const uint64_t nwords = (end_bytes + 3) / 4;
    const uint64_t ws = (A.misalign + start) >> 2;
    const uint64_t nextb = j + 1 < A.ncand ? A.cands[j + 1] : A.n;
    const uint64_t we = min((A.misalign + nextb + 3) / 4 + 2, nwords);
    const uint32_t nst = (uint32_t)min((uint64_t)IF_STAGE - 2, nwords - ws);
    const bool to_end = ws + nst == nwords;
    for (uint32_t i = lane; i < nst + 2; i += IF_NT) {
        uint32_t v = 0;
        if (i < nst) {
            const uint64_t wi = ws + i;
            v = A.in_words[wi];
            const uint64_t lim = end_bytes - 4 * wi;
            if (lim < 4) v &= (1u << (8 * lim)) - 1u;
        }
        stg[i] = v;
    }
    __syncthreads();
    SegSink sk{win, 0, j == 0, 0};
    uint64_t end_byte = 0;
    bool fin = false;
    const bool rfc = (A.flags & DMX_CFG_RFC_STRICT) != 0;
    uint32_t err = 0;
    bool staged = we - ws + 2 <= (uint64_t)nst + 2;
    if (staged) {
        StageReader br;
        br.init(stg, ws, nst, A.misalign, A.n);
        br.seek((A.misalign + start) * 8);
        err = inflate_blocks(br, T, sk, rfc, true, &end_byte, &fin, A.dbg ? hdr_cycles : nullptr);
        if (!to_end && br.p + 32 > nst * 32) staged = false;  // read past the stage: redo
    }
    if (!staged) {
        sk.pos = 0;
        sk.err = 0;
        fin = false;
        end_byte = 0;
        T.fixed_loaded = 0;
        wave_sync();
        BitIn br;
        br.init(A.in_words, A.misalign, A.n);
        br.stage(stg, ws, nst);
        br.seek((A.misalign + start) * 8);
        err = inflate_blocks(br, T, sk, rfc, true, &end_byte, &fin, A.dbg ? hdr_cycles : nullptr);
    }
    const uint32_t size = err ? 0 : sk.pos;
    DMX_PHASE(A.dbg, j, 1);
    if (A.dbg && lane_id() == 0)
        for (int k = 0; k < 5; k++) A.dbg[j * kPhaseSlots + 8 + k] = hdr_cycles[k];

    if (lane == 0) {
        uint64_t excl = 0;
        if (A.mode == 3) {
            excl = j * (uint64_t)A.slot;  // the workgroup decoder's slot
        } else if (A.mode == 0) {
            // speculative: every segment before the final one has this segment's size (what
            // libdmx's deflate emits); the final one takes segment 0's size.  Checked after
            // the kernel by k_inflate_validate; a miss re-runs in look-back mode.
            if (j == 0) {
                __hip_atomic_store(&A.status[0], LB_P | size, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (!fin) {
                excl = j * (uint64_t)size;
            } else {
                uint32_t spins = 0;
                unsigned long long v;
                while (((v = __hip_atomic_load(&A.status[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 62) == 0) {
                    if (++spins > (1u << 24)) { err |= SEGF_TIMEOUT; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                excl = j * (v & LB_V);
            }
        } else if (j == 0) {
            __hip_atomic_store(&A.status[0], LB_P | size, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            // decoupled look-back over the candidates before this one
            __hip_atomic_store(&A.status[j], LB_A | size, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint64_t k = j - 1;
            uint32_t spins = 0;
            for (;;) {
                const unsigned long long v =
                    __hip_atomic_load(&A.status[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long f = v >> 62;
                if (f == 0) {
                    if (++spins > (1u << 24)) {
                        err |= SEGF_TIMEOUT;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                excl += v & LB_V;
                if (f == 2) break;
                k--;
            }
            __hip_atomic_store(&A.status[j], LB_P | (excl + size), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        s_excl = excl;
        DMX_PHASE(A.dbg, j, 2);
        A.recs[j].end_byte = end_byte - A.misalign;
        A.recs[j].out_size = size;
        A.recs[j].flags = err | (fin ? SEGF_FINAL : 0u);
        A.recs[j].offset = excl;
    }
    __syncthreads();
    if (err) return;
    const uint64_t excl = s_excl;
    if (excl >= A.cap) return;
    const uint32_t nb = (uint32_t)min((uint64_t)size, A.cap - excl);
    uint8_t* dst = A.out + excl;
    if ((((uintptr_t)dst) & 15) == 0) {
        const uint32_t nv = nb / 16;
        const uint4* s4 = reinterpret_cast<const uint4*>(win);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint32_t i = lane; i < nv; i += 64) d4[i] = s4[i];
        for (uint32_t i = nv * 16 + lane; i < nb; i += 64) dst[i] = win[i];
    } else {
        for (uint32_t i = lane; i < nb; i += 64) dst[i] = win[i];
    }
    DMX_PHASE(A.dbg, j, 3);
}

// ---------------------------------------------------------------------------------------
// k_inflate_pj<SEG, NT>: one workgroup of NT lanes per candidate segment of up to SEG bytes.
//   1. wave 0 reads BTYPE; a stored segment is copied HBM -> HBM; a Huffman segment's
//      compressed words are staged in LDS (every later bit read is an LDS read), then wave 0
//      reads the block header and the workgroup fills the lookup tables;
//   2. the segment's Huffman bits are split into nl equal ranges; lane t decodes tokens from
//      the start of its range (an arbitrary bit: Huffman decoding self-synchronises within a
//      few tokens) until its path crosses into the next range, keeping the first PJ_K token
//      boundaries it passed;
//   3. settle: lane t restarts where lane t-1's path left its range and decodes until it
//      reaches a boundary of its own first path (merged: the rest of its count is known) --
//      repeated until every range starts where the previous one ended (normally one round);
//   4. exclusive scan of the per-lane output counts, then every lane re-decodes its range and
//      writes P[x] for each output byte x: 0x8000 | byte for a literal, or the position the
//      byte is copied from (LZ77 copy out[o + i] = out[o - d + (i mod d)], always < x);
//   5. pointer jumping P[x] = P[P[x]] until every entry is a literal (chains halve per round);
//   6. the low bytes of P go to HBM with 16-byte stores at the segment's slot j * SEG.
// Everything else -- several blocks in one segment, an output above SEG, compressed data
// above the staging buffer, a split that does not settle -- is flagged SEGF_EXOTIC and the
// stream is redone by k_inflate_segments, so results never depend on this path's coverage.
// ---------------------------------------------------------------------------------------
constexpr uint32_t PJ_LIT = 0x8000u;
constexpr int PJ_ROUNDS = 64;
constexpr uint32_t PJ_MINBITS = 256;
constexpr int PJ_LL = 12;  // lit/len lookup bits
constexpr int PJ_LD = 10;  // distance lookup bits

template <int SEG, int NT>
struct PjSmem {
    static constexpr int IN_WORDS = (SEG + 2048) / 4 + 8;
    uint16_t P[SEG];
    uint32_t in[IN_WORDS];  // the candidate's compressed words, in[0] = stream word ws
    uint32_t llut[1 << PJ_LL];  // 32-bit entries (lit_entry / dist_entry)
    uint32_t dlut[1 << PJ_LD];
    Tables T;
    uint32_t endp[NT];      // where range r's current path crossed into range r+1; later the
                            // exclusive output offset of range r
    uint32_t cntr[NT];      // output bytes of range r
    uint32_t part[NT / 64];
    uint32_t te2[2];        // first range whose path ends (EOB / no code), alternating words
    uint32_t dcount[4];     // developer counters (DMX_PHASES)
    uint64_t ws;            // first staged stream word
    uint32_t nst;           // staged words
    uint32_t hs;            // first Huffman bit, relative to ws * 32
    uint32_t hlen;          // bits split among the lanes
    uint32_t kind;          // 0 Huffman, 1 stored, 2 done (empty segment / error)
    uint32_t btype;
    uint32_t bfinal;
    uint32_t err;
    uint32_t slen;
    uint64_t sb0;
    uint32_t total;
    uint64_t end_byte;
};

// 32 bits at bit p of the staged words (LSB = bit p)
__device__ __forceinline__ uint32_t lds_peek32(const uint32_t* w, uint32_t p) {
    const uint32_t i = p >> 5;
    return __builtin_amdgcn_alignbit(w[i + 1], w[i], p & 31);
}

// primary lookup table over PB bits with 32-bit entries, filled by the whole workgroup
template <int PB, bool DIST>
__device__ void fill_lut32_wg(uint32_t* lut, const TreeMeta& m, const uint16_t* sorted, int tid, int nthr) {
    uint32_t lo[16], hi[16], cn[16], of[16];
#pragma unroll
    for (int k = 1; k < 16; k++) {
        lo[k] = m.lo[k];
        hi[k] = m.hi[k];
        cn[k] = m.cnt[k];
        of[k] = m.offs[k];
    }
    for (int wv = tid; wv < (1 << PB); wv += nthr) {
        const uint32_t v = bitrev(wv, PB);
        uint32_t idx = 0, len = 0;
#pragma unroll
        for (int k = 1; k <= PB && k < 16; k++) {
            const uint32_t x = v >> (PB - k);
            if (!len && cn[k] && x <= hi[k]) {
                const uint32_t cm = x + (((hi[k] - x) >> k) << k);
                if (cm >= lo[k]) {
                    idx = of[k] + cm - lo[k];
                    len = k;
                }
            }
        }
        lut[wv] = len ? (DIST ? dist_entry(sorted[idx], len) : lit_entry(sorted[idx], len)) : 0u;
    }
}

enum : uint32_t { TK_LIT = 0, TK_MATCH = 1, TK_EOB = 2, TK_BAD = 3 };

// one token of decompressHuffmanBlock (inflate.hpp:226-275) at bit *p of the staged words:
// a literal (*a = byte), a match (*a = length, *d = distance; 0 for symbols 286+ / 30+), the
// end of block, or no code.  A literal reads one 32-bit window, a match two; the 32-bit table
// entries carry class, code length, base and extra-bit count.
__device__ __forceinline__ uint32_t pj_token(const uint32_t* w, uint32_t* p, const uint32_t* llut,
                                             const uint32_t* dlut, const Tables& T, uint32_t* a,
                                             uint32_t* d) {
    uint32_t v = lds_peek32(w, *p);
    uint32_t e = llut[v & ((1u << PJ_LL) - 1)];
    if (!e) {
        uint32_t sym, len;
        if (!slow_decode(T.lm, T.lsorted, v & 0x7FFF, PJ_LL + 1, &sym, &len)) return TK_BAD;
        e = lit_entry(sym, len);
    }
    const uint32_t cl = e & 15, ty = (e >> 4) & 3;
    if (ty == 0) {
        *p += cl;
        *a = e >> 16;
        return TK_LIT;
    }
    if (ty == 1) {
        *p += cl;
        return TK_EOB;
    }
    const uint32_t ex = (e >> 6) & 15;
    *a = (e >> 16) + ((v >> cl) & ((1u << ex) - 1u));
    *p += cl + ex;
    v = lds_peek32(w, *p);
    uint32_t de = dlut[v & ((1u << PJ_LD) - 1)];
    if (!de) {
        uint32_t ds, dl;
        if (!slow_decode(T.dm, T.dsorted, v & 0x7FFF, PJ_LD + 1, &ds, &dl)) return TK_BAD;
        de = dist_entry(ds, dl);
    }
    const uint32_t dl = de & 15, dx = (de >> 6) & 15;
    *d = (de >> 16) + ((v >> dl) & ((1u << dx) - 1u));
    *p += dl + dx;
    return TK_MATCH;
}

__device__ __forceinline__ uint32_t tok_bytes(uint32_t k, uint32_t a, uint32_t d) {
    return k == TK_LIT ? 1u : (k == TK_MATCH && a && d) ? a : 0u;
}

template <int SEG, int NT>
__global__ __launch_bounds__(NT) void k_inflate_pj(InflateArgs A) {
    using Smem = PjSmem<SEG, NT>;
    __shared__ __attribute__((aligned(16))) Smem S;
    constexpr int NW = NT / 64;
    const int t = threadIdx.x;
    const int wave = t >> 6;
    const uint64_t j = blockIdx.x;
    const bool rfc = (A.flags & DMX_CFG_RFC_STRICT) != 0;
    const uint64_t obase = j * (uint64_t)SEG;
    const uint64_t end_bytes = A.misalign + A.n;
    DMX_PHASE(A.dbg, j, 0);

    // ---- 1. block type (wave 0), stored segments ----
    if (wave == 0) {
        BitIn br;
        br.init(A.in_words, A.misalign, A.n);
        br.seek((A.misalign + A.cands[j]) * 8);
        br.ensure(3);
        const uint32_t bfinal = br.bits(1);
        const uint32_t btype = br.bits(2);
        uint32_t kind = 2, err = 0;
        uint64_t end_byte = 0, sb0 = 0, ws = 0;
        uint32_t slen = 0, nst = 0;
        if (br.over()) {
            err = SEGF_OVERREAD;
        } else if (btype == 0) {
            br.align();
            br.ensure(32);
            const uint32_t len = br.bits(16);
            const uint32_t nlen = br.bits(16);
            sb0 = br.pos >> 3;
            if (br.over()) {
                err = SEGF_OVERREAD;
            } else if (!bfinal && len == 0 && nlen == 0xFFFF) {
                end_byte = sb0;  // the segment is just the marker
            } else if (sb0 + len > br.end_bytes) {
                err = SEGF_OVERREAD;
            } else if (len > (uint32_t)SEG) {
                err = SEGF_EXOTIC;
            } else if (bfinal) {
                kind = 1;
                slen = len;
                end_byte = sb0 + len;
            } else {
                // the next block must be the marker: 000 + 5 pad bits, 00 00 FF FF
                const uint64_t m = sb0 + len;
                if (m + 5 <= br.end_bytes && (br.byte_at(m) & 7) == 0 && br.byte_at(m + 1) == 0 &&
                    br.byte_at(m + 2) == 0 && br.byte_at(m + 3) == 0xFF && br.byte_at(m + 4) == 0xFF) {
                    kind = 1;
                    slen = len;
                    end_byte = m + 5;
                } else {
                    err = SEGF_EXOTIC;
                }
            }
        } else if (btype == 3) {
            err = SEGF_EXOTIC;
        } else {
            // stage words [ws, we): the candidate through the word after the next candidate
            ws = (A.misalign + A.cands[j]) >> 2;
            const uint64_t next = j + 1 < A.ncand ? A.cands[j + 1] : A.n;
            const uint64_t we = min((A.misalign + next + 3) / 4 + 1, br.nwords);
            if (we - ws + 4 > (uint64_t)Smem::IN_WORDS) {
                err = SEGF_EXOTIC;
            } else {
                kind = 0;
                nst = (uint32_t)(we - ws);
            }
        }
        if (lane_id() == 0) {
            S.kind = err ? 2 : kind;
            S.err = err;
            S.btype = btype;
            S.bfinal = bfinal;
            S.end_byte = end_byte;
            S.slen = slen;
            S.sb0 = sb0;
            S.ws = ws;
            S.nst = nst;
            S.total = kind == 1 ? slen : 0;
            S.dcount[0] = S.dcount[1] = S.dcount[2] = S.dcount[3] = 0;
        }
    }
    __syncthreads();
    const uint32_t kind = S.kind;

    if (kind == 1) {
        const uint32_t len = S.slen;
        const uint64_t b0 = S.sb0;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(A.in_words);
        for (uint32_t i = t; i < len; i += NT)
            if (obase + i < A.cap) A.out[obase + i] = src[b0 + i];
    } else if (kind == 0) {
        // ---- stage the compressed words (masked at the stream end), 4 words of zeros after ----
        const uint64_t ws = S.ws;
        const uint32_t nst = S.nst;
        for (uint32_t i = t; i < nst + 4; i += NT) {
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
        // ---- block header (wave 0) ----
        if (wave == 0) {
            uint64_t hp = (A.misalign + A.cands[j]) * 8 + 3;
            uint32_t err = 0;
            if (S.btype == 1) {
                load_fixed(S.T);
            } else {
                const StagedWords src{S.in, ws, nst};
                err = fast_header(src, &hp, end_bytes * 8, S.T, rfc, false);
            }
            if (lane_id() == 0) {
                const uint64_t hs = hp - ws * 32;
                const uint64_t he = j + 1 < A.ncand ? (A.misalign + A.cands[j + 1] - 4) * 8 - 3 - ws * 32
                                                    : (uint64_t)nst * 32;
                if (!err && (he <= hs || he > (uint64_t)nst * 32)) err = SEGF_EXOTIC;
                S.err = err;
                S.hs = (uint32_t)hs;
                S.hlen = err ? 0 : (uint32_t)(he - hs);
            }
        }
        __syncthreads();
        DMX_PHASE(A.dbg, j, 1);
        if (!S.err) {
            fill_lut32_wg<PJ_LL, false>(S.llut, S.T.lm, S.T.lsorted, t, NT);
            fill_lut32_wg<PJ_LD, true>(S.dlut, S.T.dm, S.T.dsorted, t, NT);
        }
        __syncthreads();
    }
    if (kind == 0 && !S.err) {
        const uint32_t* win = S.in;
        const uint32_t hs = S.hs;
        const uint32_t hlen = S.hlen;
        // ranges of at least PJ_MINBITS (a few dozen tokens) so that a path started at an
        // arbitrary bit re-synchronises inside its own range; range r belongs to thread
        // (r % NW) * 64 + r / NW so that a short segment's ranges spread over every wave
        const uint32_t nl = max(1u, min((uint32_t)NT, hlen / PJ_MINBITS));
        const uint32_t r = (uint32_t)((t & 63) * NW + wave);
        const uint32_t sp = r < nl ? (uint32_t)(((uint64_t)hlen * r) / nl) : hlen;
        const uint32_t sp1 = r + 1 < nl ? (uint32_t)(((uint64_t)hlen * (r + 1)) / nl) : hlen;
        // P is free until the emit pass: it holds the first pass's token-start bitmap, then
        // (from word cw0) the running output count after each of a range's first ccap tokens,
        // entry k of range r at cw0 * 2 + k * NT + r (u16)
        uint32_t* bmap = reinterpret_cast<uint32_t*>(S.P);
        const uint32_t cw0 = hlen / 32 + 2;
        const uint32_t ccap = min(64u, (uint32_t)(SEG / 2 - cw0) * 2 / NT);
        uint16_t* cbuf = S.P + cw0 * 2;
        for (uint32_t i = t; i < cw0; i += NT) bmap[i] = 0;
        if (t < 2) S.te2[t] = NT;
        __syncthreads();
        // ---- 2. first pass over the ranges (positions relative to hs) ----
        uint32_t qc = sp, cc = 0;  // token boundary ccap of the first pass, its count
        uint32_t e1, cnt1 = 0, st1 = 0, nb = 0;
        {
            uint32_t p = sp, pa = hs + sp;
            while (p < sp1) {
                atomicOr(&bmap[p >> 5], 1u << (p & 31));
                uint32_t a, d;
                const uint32_t k = pj_token(win, &pa, S.llut, S.dlut, S.T, &a, &d);
                if (k == TK_BAD) { st1 = 2; break; }
                p = pa - hs;
                if (k == TK_EOB) { st1 = 1; break; }
                cnt1 += tok_bytes(k, a, d);
                if (nb < ccap) cbuf[nb * NT + r] = (uint16_t)cnt1;
                if (++nb == ccap) { qc = p; cc = cnt1; }
            }
            e1 = p;
        }
        DMX_PHASE(A.dbg, j, 2);
        // ---- 3. settle the range starts ----
        // per round: [publish end, first ending range] | read te, want | or-barrier | redo |
        // barrier.  Every shared word is written and read on opposite sides of a barrier; the
        // first-ending-range minimum alternates between two words (one reset per round).
        uint32_t s = sp, e = e1, cnt = cnt1, st = st1;
        uint32_t te = NT;
        bool settled = false;
        uint32_t settle_rounds = 0;
        for (int round = 0; round <= PJ_ROUNDS; round++) {
            S.endp[r] = e;
            if (st) atomicMin(&S.te2[round & 1], r);
            if (t == 0) S.te2[(round + 1) & 1] = NT;
            __syncthreads();
            te = S.te2[round & 1];
            const uint32_t want = r == 0 ? 0 : S.endp[r - 1];
            const bool redo = r > 0 && r <= te && want != s;
            settle_rounds = round;
            if (!__syncthreads_or(redo)) {
                settled = true;
                break;
            }
            if (round == PJ_ROUNDS) break;
            if (redo) {
                // decode from the true start until the path meets a token start of this
                // range's first pass (from there on both paths are the same)
                s = want;
                uint32_t p = want, pa = hs + want, acc = 0, stn = 0, dbg_tok = 0, dbg_walk = 0;
                bool merged = false;
                for (;;) {
                    if (p >= sp1) break;
                    if (p >= sp && ((bmap[p >> 5] >> (p & 31)) & 1u)) {
                        merged = true;
                        break;
                    }
                    uint32_t a, d;
                    dbg_tok++;
                    const uint32_t k = pj_token(win, &pa, S.llut, S.dlut, S.T, &a, &d);
                    if (k == TK_BAD) { stn = 2; break; }
                    p = pa - hs;
                    if (k == TK_EOB) { stn = 1; break; }
                    acc += tok_bytes(k, a, d);
                }
                if (merged) {
                    // first-pass bytes of the tokens before p: p is token boundary kb of the
                    // first pass (kb = its marks in [sp, p)); counts of boundaries past ccap
                    // are re-walked from boundary ccap
                    uint32_t kb = 0;
                    for (uint32_t wi = sp >> 5; wi <= (p >> 5); wi++) {
                        uint32_t m = bmap[wi];
                        if (wi == (sp >> 5)) m &= ~0u << (sp & 31);
                        if (wi == (p >> 5)) m &= (1u << (p & 31)) - 1u;
                        kb += __builtin_popcount(m);
                    }
                    uint32_t before = 0;
                    if (kb == 0) {
                        before = 0;
                    } else if (kb <= ccap) {
                        before = cbuf[(kb - 1) * NT + r];
                    } else {
                        uint32_t pw = qc, pwa = hs + qc, cum = cc;
                        while (pw < p) {
                            uint32_t a, d;
                            dbg_walk++;
                            const uint32_t k = pj_token(win, &pwa, S.llut, S.dlut, S.T, &a, &d);
                            pw = pwa - hs;
                            cum += tok_bytes(k, a, d);
                            if (k == TK_BAD || k == TK_EOB) break;
                        }
                        if (pw != p) atomicOr(&S.err, SEGF_EXOTIC);  // cannot happen
                        before = cum;
                    }
                    cnt = acc + cnt1 - before;
                    e = e1;
                    st = st1;
                } else {
                    e = p;
                    cnt = acc;
                    st = stn;
                }
                if (A.dbg) {
                    atomicAdd(&S.dcount[0], dbg_tok);
                    atomicAdd(&S.dcount[3], dbg_walk);
                    atomicAdd(&S.dcount[merged ? 1 : 2], 1u);
                }
            }
            __syncthreads();
        }
        if (t == 0 && !settled) S.err |= SEGF_EXOTIC;
        DMX_PHASE(A.dbg, j, 3);
        if (A.dbg && t == 0) {
            A.dbg[j * kPhaseSlots + 9] = settle_rounds;
            A.dbg[j * kPhaseSlots + 11] = S.dcount[0];
            A.dbg[j * kPhaseSlots + 12] = S.dcount[1];
            A.dbg[j * kPhaseSlots + 13] = S.dcount[2];
            A.dbg[j * kPhaseSlots + 14] = nl;
            A.dbg[j * kPhaseSlots + 15] = S.dcount[3];
        }
        if (r == te) {
            if (st == 2) {
                S.err |= SEGF_ERR_DATA;
            } else {
                // end of block: BFINAL ends the stream, else the marker block must follow
                const uint32_t pe = hs + e;
                const uint64_t pe_abs = S.ws * 32 + pe;
                if (pe_abs > end_bytes * 8) {
                    S.err |= SEGF_OVERREAD;
                } else if (S.bfinal) {
                    S.end_byte = (pe_abs + 7) >> 3;
                } else {
                    const uint32_t h3 = lds_peek32(win, pe) & 7;
                    const uint32_t m = (pe + 3 + 7) >> 3;  // byte offset in the staged words
                    const uint8_t* sb = reinterpret_cast<const uint8_t*>(win);
                    if (h3 == 0 && m + 4 <= S.nst * 4 && sb[m] == 0 && sb[m + 1] == 0 &&
                        sb[m + 2] == 0xFF && sb[m + 3] == 0xFF && S.ws * 4 + m + 4 <= end_bytes)
                        S.end_byte = S.ws * 4 + m + 4;
                    else
                        S.err |= SEGF_EXOTIC;
                }
            }
        }
        // no end of block before the split end: several blocks, or the next candidate is not
        // this segment's end
        if (te >= (uint32_t)NT && t == 0) S.err |= SEGF_EXOTIC;
        const uint32_t mycnt = r <= te ? cnt : 0u;
        // ---- 4. scan in range order, then emit ----
        S.cntr[r] = mycnt;
        __syncthreads();
        const uint32_t cv = S.cntr[t];
        const uint32_t inc = wave_incl_scan(cv);
        if ((t & 63) == 63) S.part[wave] = inc;
        __syncthreads();
        uint32_t base = 0, total = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint32_t v = S.part[w];
            base += w < wave ? v : 0u;
            total += v;
        }
        S.endp[t] = base + inc - cv;  // exclusive output offset of range t
        if (t == 0) {
            S.total = total;
            if (total > (uint32_t)SEG) S.err |= SEGF_EXOTIC;  // larger segments: other decoder
        }
        __syncthreads();
        if (!S.err) {
            // wave-uniform token loop: matches of 16+ bytes are expanded by the whole wave
            uint32_t o = S.endp[r];
            uint32_t p = s, pa = hs + s;
            bool act = r <= te && mycnt != 0;
            uint32_t bad = 0;
            uint32_t* P2 = reinterpret_cast<uint32_t*>(S.P);
            const uint32_t lane = t & 63;
            for (;;) {
                const bool live = act && p < sp1;
                if (!__ballot(live)) break;
                uint32_t k = TK_EOB, a = 0, d = 0;
                if (live) {
                    k = pj_token(win, &pa, S.llut, S.dlut, S.T, &a, &d);
                    p = pa - hs;
                    if (k == TK_LIT) S.P[o++] = (uint16_t)(PJ_LIT | a);
                    if (k == TK_EOB || k == TK_BAD) act = false;
                }
                bool mt = live && k == TK_MATCH && a && d;
                if (mt && d > o) {  // before the segment: cross-segment or stream-start reference
                    bad = j == 0 ? SEGF_EXOTIC : SEGF_XREF;
                    act = false;
                    mt = false;
                }
                const bool longm = mt && a >= 16;
                if (mt && !longm) {
                    const uint32_t src = o - d;
                    uint32_t rr = 0;
                    for (uint32_t i = 0; i < a; i++) {
                        S.P[o + i] = (uint16_t)(src + rr);
                        if (++rr == d) rr = 0;
                    }
                }
                uint64_t lm = __ballot(longm);
                while (lm) {
                    const int l = __builtin_ctzll(lm);
                    lm &= lm - 1;
                    const uint32_t ol = __builtin_amdgcn_readlane(o, l);
                    const uint32_t dl = __builtin_amdgcn_readlane(d, l);
                    const uint32_t al = __builtin_amdgcn_readlane(a, l);
                    const uint32_t src = ol - dl;
                    if (dl >= al) {
                        for (uint32_t i = lane; i < al; i += 64) S.P[ol + i] = (uint16_t)(src + i);
                    } else {
                        uint32_t rr = lane % dl;
                        const uint32_t step = 64 % dl;
                        for (uint32_t i = lane; i < al; i += 64) {
                            S.P[ol + i] = (uint16_t)(src + rr);
                            rr += step;
                            if (rr >= dl) rr -= dl;
                        }
                    }
                }
                if (mt) o += a;
            }
            (void)P2;
            if (bad) atomicOr(&S.err, bad);
        }
        __syncthreads();
        DMX_PHASE(A.dbg, j, 4);
        // ---- 5. pointer jumping ----
        if (!S.err) {
            uint32_t* P2 = reinterpret_cast<uint32_t*>(S.P);
            const uint32_t npair = (total + 1) / 2;
            bool open = true;
            for (int round = 0; round < 24 && open; round++) {
                uint32_t any = 0;
                for (uint32_t i0 = t; i0 < npair; i0 += 4 * NT) {
                    uint32_t v[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t i = i0 + u * NT;
                        v[u] = i < npair ? P2[i] : (PJ_LIT | (PJ_LIT << 16));
                    }
                    uint32_t lo[4], hi[4];
                    bool plo[4], phi[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t i = i0 + u * NT;
                        lo[u] = v[u] & 0xFFFF;
                        hi[u] = v[u] >> 16;
                        plo[u] = !(lo[u] & PJ_LIT);
                        phi[u] = !(hi[u] & PJ_LIT) && 2 * i + 1 < total;
                        if (plo[u]) lo[u] = S.P[lo[u]];
                        if (phi[u]) hi[u] = S.P[hi[u]];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t i = i0 + u * NT;
                        if (plo[u] | phi[u]) {
                            if (!phi[u]) hi[u] = v[u] >> 16;
                            if (!plo[u]) lo[u] = v[u] & 0xFFFF;
                            P2[i] = lo[u] | (hi[u] << 16);
                            any |= (plo[u] && !(lo[u] & PJ_LIT)) || (phi[u] && !(hi[u] & PJ_LIT));
                        }
                    }
                }
                open = __syncthreads_or(any) != 0;
                if (A.dbg && t == 0) A.dbg[j * kPhaseSlots + 10] = round + 1;
            }
            if (open && t == 0) S.err |= SEGF_EXOTIC;
            __syncthreads();
        }
        DMX_PHASE(A.dbg, j, 5);
        // ---- 6. low bytes of P to the slot ----
        if (!S.err) {
            const uint32_t nb16 = total / 16;
            uint8_t* dst = A.out + obase;
            const bool vec = (((uintptr_t)dst) & 15) == 0 && obase + total <= A.cap;
            const uint4* P4 = reinterpret_cast<const uint4*>(S.P);
            if (vec) {
                for (uint32_t i = t; i < nb16; i += NT) {
                    const uint4 a = P4[2 * i], b = P4[2 * i + 1];
                    uint4 o;
                    o.x = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                    o.y = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                    o.z = __builtin_amdgcn_perm(b.y, b.x, 0x06040200u);
                    o.w = __builtin_amdgcn_perm(b.w, b.z, 0x06040200u);
                    reinterpret_cast<uint4*>(dst)[i] = o;
                }
                for (uint32_t i = nb16 * 16 + t; i < total; i += NT) dst[i] = (uint8_t)S.P[i];
            } else {
                for (uint32_t i = t; i < total; i += NT)
                    if (obase + i < A.cap) dst[i] = (uint8_t)S.P[i];
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        const uint32_t err = S.err;
        A.recs[j].end_byte = S.end_byte - A.misalign;
        A.recs[j].out_size = err ? 0 : S.total;
        A.recs[j].flags = err | (S.bfinal && !err ? SEGF_FINAL : 0u);
        A.recs[j].offset = obase;
    }
    DMX_PHASE(A.dbg, j, 6);
}

hipError_t launch_inflate_pj(const InflateArgs& A, uint32_t seg, hipStream_t st, hipEvent_t ev0,
                             hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, st);
    if (seg == 16384)
        hipLaunchKernelGGL((k_inflate_pj<16384, 256>), dim3((uint32_t)A.ncand), dim3(256), 0, st, A);
    else
        hipLaunchKernelGGL((k_inflate_pj<32768, 512>), dim3((uint32_t)A.ncand), dim3(512), 0, st, A);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// Candidate chain check.  Valid iff, up to the first BFINAL segment k, every segment decoded
// without error and ended exactly at the next candidate.  Speculative mode additionally needs
// every segment before k to have segment 0's size (else status 1: re-run with look-back).
__global__ __launch_bounds__(1024) void k_inflate_validate(InflateArgs A, InflateResult* res) {
    __shared__ unsigned long long kmin, bmin, umin, xmin, xcnt;
    const int t = threadIdx.x;
    if (t == 0) { kmin = ~0ull; bmin = ~0ull; umin = ~0ull; xmin = ~0ull; xcnt = 0; }
    __syncthreads();
    // mode 2 (k_inflate_lanes) placed segment j at j * 32768
    const uint32_t size0 = A.mode >= 2 ? A.slot : A.recs[0].out_size;
    for (uint64_t j = t; j < A.ncand; j += 1024) {
        const SegRecord r = A.recs[j];
        if (r.flags & SEGF_EXOTIC) {  // k_inflate_pj declined this candidate
            atomicMin(&xmin, (unsigned long long)j);
            atomicAdd(&xcnt, 1ull);
            continue;
        }
        const bool fin = (r.flags & SEGF_FINAL) != 0;
        const bool err = (r.flags & ~SEGF_FINAL) != 0;
        const bool chain = (j + 1 < A.ncand) && r.end_byte == A.cands[j + 1];
        if (fin) atomicMin(&kmin, (unsigned long long)j);
        if (err || (!fin && !chain)) atomicMin(&bmin, (unsigned long long)j);
        if (!fin && r.out_size != size0) atomicMin(&umin, (unsigned long long)j);
    }
    __syncthreads();
    if (t == 0) {
        const uint64_t k = kmin;
        res->fin_index = (uint32_t)k;
        res->exotic = xcnt;
        if (xmin < A.ncand) {
            res->status = 1;
            res->total = 0;
        } else if (k < A.ncand && bmin > k) {
            if (A.mode != 1 && umin < k) {
                res->status = 1;
                res->total = 0;
            } else {
                res->status = 0;
                res->total = A.recs[k].offset + A.recs[k].out_size;
            }
        } else {
            res->total = 0;
            res->status = 2;
        }
    }
}

// ---------------------------------------------------------------------------------------
// serial path: the whole stream by one wavefront (sizes first, then bytes)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(IF_NT) void k_inflate_serial(InflateArgs A, int count_only,
                                                          InflateResult* res) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[65536];
    __shared__ Tables T;
    if (threadIdx.x == 0) T.fixed_loaded = 0;
    __syncthreads();
    BitIn br;
    br.init(A.in_words, A.misalign, A.n);
    br.seek(A.misalign * 8);
    RingSink sk{ring, 0, A.out, A.cap, count_only != 0, 0};
    uint64_t end_byte = 0;
    bool fin = false;
    const uint32_t err =
        inflate_blocks(br, T, sk, (A.flags & DMX_CFG_RFC_STRICT) != 0, false, &end_byte, &fin);
    if (threadIdx.x == 0) {
        res->total = sk.pos;
        res->status = err == 0 ? 0 : (err & SEGF_OVERREAD) ? DMX_ERR_OVERREAD : DMX_ERR_DATA;
        res->fin_index = 0;
    }
}

hipError_t launch_inflate_segments(const InflateArgs& A, hipStream_t st, hipEvent_t ev0,
                                   hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, st);
    hipLaunchKernelGGL(k_inflate_segments, dim3((uint32_t)A.ncand), dim3(IF_NT), 0, st, A);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

hipError_t launch_inflate_validate(const InflateArgs& A, InflateResult* res, hipStream_t st) {
    hipLaunchKernelGGL(k_inflate_validate, dim3(1), dim3(1024), 0, st, A, res);
    return hipGetLastError();
}

hipError_t launch_inflate_serial(const InflateArgs& A, int count_only, InflateResult* res,
                                 hipStream_t st) {
    hipLaunchKernelGGL(k_inflate_serial, dim3(1), dim3(IF_NT), 0, st, A, count_only, res);
    return hipGetLastError();
}

}  // namespace dmx
