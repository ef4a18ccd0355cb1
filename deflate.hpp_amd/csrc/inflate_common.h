// inflate_common.h -- device code shared by the inflate kernels (inflate_kernels.hip,
// inflate_blocks.hip): bit readers, canonical-code tables with the reference's lookup rule,
// the lane-parallel dynamic-header reader, and the generic block loop over an output sink.
// Decoding semantics follow the reference inflate (inflate.hpp:136-322, common.hpp bit-trie).
#pragma once
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
template <class Meta>  // (TreeMeta in any address space)
__device__ __forceinline__ bool key_hit(const Meta& m, uint32_t k, uint32_t x, uint32_t* c) {
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
template <class Meta, class Sorted>  // (LDS tables through a flat or an LDS pointer)
__device__ __forceinline__ bool slow_decode(const Meta& m, const Sorted* sorted,
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

// Wave-uniform bit reader over a sliding LDS ring of the stream (fb_serial, k_inflate_serial).  BitIn reads
// through the scalar cache, and scalar loads share lgkmcnt with LDS, so every table lookup
// waited for the next stream word (~1000 cycles per symbol on C3).  Here the wave copies the
// stream into a ring of FB_RW words ahead of the reader, FB_RC words at a time, so every bit
// read is an LDS read.  Invariant after seek / refill: words [wi - 1, wi + FB_AHEAD) are in
// the ring (fast_header reads up to ~140 words past its start).  All lanes call every method
// together (the decoder state is wave-uniform).
constexpr uint32_t FB_RW = 1024, FB_RC = 512, FB_AHEAD = 320;
struct RingIn {
    const uint32_t* w;
    uint64_t nwords, end_bytes, end_bits;
    uint32_t* ring;
    uint64_t rb;    // ring holds words [rb, rb + FB_RW) at ring[i % FB_RW]
    uint64_t pos;   // bits consumed, relative to the aligned base
    uint64_t buf;   // LSB = next bit
    uint32_t cnt;   // valid bits in buf
    uint64_t wi;    // next word to shift into buf

    __device__ void init(const uint32_t* words, uint64_t misalign, uint64_t n, uint32_t* lds) {
        w = words;
        end_bytes = misalign + n;
        end_bits = end_bytes * 8;
        nwords = (end_bytes + 3) / 4;
        ring = lds;
        rb = ~0ull >> 1;
    }
    __device__ void fill(uint64_t from, uint64_t to) {  // words [from, to), masked at the end
        for (uint64_t i = from + lane_id(); i < to; i += 64) {
            uint32_t v = 0;
            if (i < nwords) {
                v = w[i];
                const uint64_t lim = end_bytes - 4 * i;
                if (lim < 4) v &= (1u << (8 * lim)) - 1u;
            }
            ring[i % FB_RW] = v;
        }
        wave_sync();
    }
    __device__ uint32_t word(uint64_t i) const { return ring[i % FB_RW]; }
    __device__ void refill() {
        if (cnt <= 32) {
            if (wi + FB_AHEAD >= rb + FB_RW) {  // slide: the oldest FB_RC words make room
                fill(rb + FB_RW, rb + FB_RW + FB_RC);
                rb += FB_RC;
            }
            buf |= (uint64_t)word(wi) << cnt;
            cnt += 32;
            wi++;
        }
    }
    __device__ void seek(uint64_t bitpos) {
        pos = bitpos;
        const uint64_t i = bitpos >> 5;
        if (i < rb || i + 1 + FB_AHEAD >= rb + FB_RW) {
            rb = i;
            fill(i, i + FB_RW);
        }
        buf = (uint64_t)(word(i) >> (bitpos & 31));
        cnt = 32 - (uint32_t)(bitpos & 31);
        wi = i + 1;
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
    __device__ uint32_t window32() {
        ensure(32);
        return (uint32_t)buf;
    }
    __device__ uint64_t abspos() const { return pos; }
    __device__ uint8_t byte_at(uint64_t b) const {  // b relative to the aligned base (stored data)
        return (uint8_t)(w[b >> 2] >> ((b & 3) * 8));
    }
};
struct RingWords {
    const uint32_t* ring;
    __device__ uint32_t word(uint64_t i) const { return ring[i % FB_RW]; }
};
__device__ __forceinline__ RingWords reader_words(const RingIn& br) { return RingWords{br.ring}; }

// ---------------------------------------------------------------------------------------
// lane-parallel token decoding over LDS-staged words (k_inflate_pj, k_fb_pdecode): every lane
// decodes its own bit range with 32-bit tables of PJ_LL / PJ_LD primary bits
// ---------------------------------------------------------------------------------------
constexpr int PJ_LL = 12;  // lit/len lookup bits
constexpr int PJ_LD = 10;  // distance lookup bits

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

// decompressHuffmanBlock (inflate.hpp:226-275) with 32-bit table entries: one 32-bit window
// per half token (code + extra bits), no per-symbol base / extra arithmetic.
// soft: stop (SEGF_SOFT) at the first token boundary at or past this reader position (path 5's
// units that end inside a block; ~0 = never), or where the sink is full()
template <class BR, class Sink>
__device__ uint32_t decode_huffman(BR& br, const Tables& T, Sink& sk, uint64_t soft = ~0ull) {
    for (;;) {
        if (br.abspos() >= soft || sk.full()) return SEGF_SOFT;
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

// One Huffman-coded block of inflate_blocks: the generic decoder; a sink with its own block
// decoder (the serial path's FlushSink) provides an overload that ADL finds at instantiation.
template <class BR, class Sink>
__device__ __forceinline__ uint32_t decode_block(BR& br, const Tables& T, Sink& sk) {
    return decode_huffman(br, T, sk);
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
            const uint32_t err = decode_block(br, T, sk);
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
            err = decode_block(br, T, sk);
            if (err) return err;
        }  // btype 3: no-op block (inflate.hpp:292 has no case 3)
        if (bfinal) {
            *fin = true;
            *end_byte = (br.abspos() + 7) >> 3;
            return 0;
        }
    }
}

// per-lane LSB-first bit reader over the stream in HBM: a 64-bit bit buffer fed from a ring
// of eight 16-byte quads held in VGPRs (quad q of the stream lives in Q[q & 7]).  Loads are
// issued only in wave-wide top-ups (every lane refills all its consumed quads at once, one
// memory latency for the wave), never one lane at a time: s_waitcnt is per wave, so a lane's
// lone reload would stall all 64.  Positions are bytes from blk (the 16-byte aligned base);
// bytes at or past E read as zero.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GUint4;  // global, not flat: a flat
                                                               // load also counts in lgkmcnt
#ifndef DMX_LN_RING_LOW
#define DMX_LN_RING_LOW 16
#endif
constexpr uint32_t LN_RING_LOW = DMX_LN_RING_LOW;  // top up when fewer words than this are buffered

struct LaneIn {
    GUint4* blk;     // the candidate's first 16-byte quad: all positions below are 32-bit,
    uint32_t nblk, E;  // relative to it (E clamped to 2^26 bytes, far beyond any accepted segment)
    u32x4 Q0, Q1, Q2, Q3, Q4, Q5, Q6, Q7;
    uint32_t fq;  // quads [.., fq) are in the ring
    uint32_t wi;  // index of the next word to shift into bb
    uint32_t nb;  // valid bits in bb
    uint64_t bb;
    // clamped to the last block (refill() zeroes bytes past E), so the load is unconditional
    // within the lanes that issue it
    __device__ __forceinline__ u32x4 fetch(uint32_t b) const { return blk[min(b, nblk - 1)]; }
    __device__ __forceinline__ bool low() const { return fq * 4 < wi + LN_RING_LOW; }
    // load quads [fq, wi/4 + 8): slot k gets the quad q == k (mod 8) in that range, or --
    // when there is none -- its current quad again (same bytes), so all eight loads are
    // unconditional.  The addresses are pinned in registers of their own before the first
    // load: computed inside the loads' registers, each would first wait for the previous
    // top-up's load there (vmcnt(0), which also drains the loads just issued).
    __device__ __forceinline__ void topup() {
        const uint32_t lim = (wi >> 2) + 8, last = nblk - 1;
        uint64_t a[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
            uint32_t q = fq + ((k - fq) & 7u);
            if (q >= lim) q -= 8;
            a[k] = reinterpret_cast<uint64_t>(blk + min(q, last));
        }
        asm volatile("" : : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
                     "v"(a[6]), "v"(a[7]));
        Q0 = *reinterpret_cast<GUint4*>(a[0]);
        Q1 = *reinterpret_cast<GUint4*>(a[1]);
        Q2 = *reinterpret_cast<GUint4*>(a[2]);
        Q3 = *reinterpret_cast<GUint4*>(a[3]);
        Q4 = *reinterpret_cast<GUint4*>(a[4]);
        Q5 = *reinterpret_cast<GUint4*>(a[5]);
        Q6 = *reinterpret_cast<GUint4*>(a[6]);
        Q7 = *reinterpret_cast<GUint4*>(a[7]);
        fq = lim;
    }
    __device__ __forceinline__ uint32_t word() const {
        const uint32_t qs = (wi >> 2) & 7, ws = wi & 3;
        const bool b0 = qs & 1, b1 = qs & 2, b2 = qs & 4;
        const u32x4 p01 = b0 ? Q1 : Q0, p23 = b0 ? Q3 : Q2, p45 = b0 ? Q5 : Q4, p67 = b0 ? Q7 : Q6;
        const u32x4 p03 = b1 ? p23 : p01, p47 = b1 ? p67 : p45;
        const u32x4 q = b2 ? p47 : p03;
        return (ws & 2) ? ((ws & 1) ? q.w : q.z) : ((ws & 1) ? q.y : q.x);
    }
    __device__ __forceinline__ void refill() {  // requires nb <= 32 and a word in the ring
        uint32_t w = word();
        const uint32_t wb = wi * 4;
        if (wb + 4 > E) w = wb >= E ? 0u : (w & ((1u << (8 * (E - wb))) - 1u));
        bb |= (uint64_t)w << nb;
        nb += 32;
        wi++;
    }
    __device__ void seek(uint32_t abyte) {
        wi = abyte >> 2;
        fq = wi >> 2;
        topup();
        bb = 0;
        nb = 0;
        refill();
        refill();
        const uint32_t sk = (abyte & 3) * 8;
        bb >>= sk;
        nb -= sk;
    }
    __device__ __forceinline__ void ensure(uint32_t k) {  // k <= 32
        if (nb < k) refill();
    }
    __device__ __forceinline__ uint32_t bits(uint32_t n) {  // n <= 32, after ensure(n)
        const uint32_t v = n ? (uint32_t)(bb & ((1ull << n) - 1ull)) : 0u;
        bb >>= n;
        nb -= n;
        return v;
    }
    __device__ __forceinline__ void consume(uint32_t n) {
        bb >>= n;
        nb -= n;
    }
    __device__ __forceinline__ uint32_t bitpos() const { return wi * 32 - nb; }
    __device__ __forceinline__ void align() { consume((uint32_t)(-bitpos()) & 7u); }  // next byte
};

}  // namespace dmx
