// deflate_kernels.hip -- MI355X (gfx950) DEFLATE encoder kernels.
//
// One 1024-thread workgroup (16 waves) compresses one independent segment (32 KiB, or 16 KiB)
// entirely out of LDS, the way the reference compresses one 32 KiB chunk with a fresh LZ77 state
// (realCompress, /root/reference/include/deflate.hpp:680-752):
//
//   load (16 B/lane coalesced)  -> LDS byte image of the segment
//   match rounds                -> a fingerprinted {latest, first-in-round} hash table in LDS,
//                                  rounds of 2048 positions (a consecutive pair per thread):
//                                  cand[p] = distance to the first occurrence of p's 4-byte key
//                                  earlier in the same round, else to the latest one in earlier
//                                  rounds   (replaces LZ77::getMatches deflate.hpp:310-383)
//   level 3                     -> a depth-16 search along the chains of those candidates
//                                  (replaces getMatchesSlow :268-304)
//   parse walk                  -> 258-byte chunk per quad of lanes, greedy (level 2) or one-step
//                                  lazy (level 3); matches never cross a chunk edge, so chunks
//                                  parse independently; token starts -> LDS bitmap
//   histogram                   -> token ranges balanced over the threads, LDS atomics
//                                  (constructDynamicHuffmanTree :402-418)
//   code lengths                -> block-parallel length-limited Huffman
//                                  (FlatHuffmanTree::generateCodeLengths common.hpp:322-404)
//   canonical codes             -> (FlatHuffmanTree::construct common.hpp:104-145)
//   dynamic header              -> parallel RLE of the two code-length sequences, precode
//                                  (writeDynamicHuffmanTree deflate.hpp:544-626)
//   bit pack                    -> per-thread bit counts, block scan, owned-range word stores into
//                                  an LDS bit image (compressBuffer deflate.hpp:630-674,
//                                  Bitstream :80-159)
//   store                       -> dynamic / fixed / stored, whichever is smallest
//                                  (deflate.hpp:739-746), then an empty stored block so every
//                                  segment ends byte-aligned (segments concatenate bytewise).
//
// k_scan_part + k_scan_apply scan the per-segment sizes and k_compact concatenates the segment slots.
#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

constexpr int DF_NT = 1024;    // threads per workgroup (16 waves)
#ifndef DMX_DF_CHUNK
#define DMX_DF_CHUNK 258
#endif
constexpr int DF_CHUNK = DMX_DF_CHUNK;  // bytes per parse lane: one maximal match per chunk, and not a
                               // multiple of 256, so the lanes' chunk starts spread over the LDS
                               // banks (at 256 every lane of a wave hit one bank per matchlen read)
constexpr int df_hash_bits(int seg) {  // hash bits of each of the two match tables: 11 at 16 KiB
    return seg >= 32768 ? 12 : 11;     // keeps that variant at <= 80 KiB of LDS (two per CU)
}
// Code-length limits of the emitted lit/len and distance codes.  RFC 1951 allows 15; 9 and 6
// keep every code inside the one-level lookup tables of the lane decoder
// (inflate_lanes.hip: 512 + 64 entries per segment in LDS) at < 1% ratio cost.
#ifndef DMX_LIT_MAXBITS
#define DMX_LIT_MAXBITS 9
#define DMX_DIST_MAXBITS 6
#endif
constexpr int DF_LIT_MAXBITS = DMX_LIT_MAXBITS;
constexpr int DF_DIST_MAXBITS = DMX_DIST_MAXBITS;
#ifndef DMX_L3_DEPTH
#define DMX_L3_DEPTH 16
#endif
constexpr int DF_L3_DEPTH = DMX_L3_DEPTH;  // level 3: candidate-chain links searched per position
#ifndef DMX_L3_LONG
#define DMX_L3_LONG 16
#endif
constexpr uint32_t DF_L3_LONG = DMX_L3_LONG;  // level 3: a first link this long ends the chain search
#ifndef DMX_L3_ROUND
#define DMX_L3_ROUND 128
#endif
constexpr uint32_t DF_L3_ROUND = DMX_L3_ROUND;  // level 3: positions per link-building round
// Level 3 links: the level-2 candidates (first occurrence in the round, else the latest before
// it) by default; 1 = the single-wave link rounds of DF_L3_ROUND positions (latest occurrence
// before the position's round), which cannot see an occurrence inside the same round.
#ifndef DMX_L3_LINK_ROUNDS
#define DMX_L3_LINK_ROUNDS 0
#endif
constexpr bool DF_L3_LINK_ROUNDS = DMX_L3_LINK_ROUNDS != 0;
// Level 3: positions per match round (the level-2 rounds take 2 * DF_NT = 2048)
#ifndef DMX_L3_U
#define DMX_L3_U 3
#endif
// level 3's chain search: 1 = the tail test as one unaligned 4-byte LDS read, 2 = also the match
// lengths by unaligned 8-byte reads, 3 = those but the first link's length by aligned words
// (0 = aligned words and alignbyte throughout)
[[maybe_unused]] constexpr int DF_L3_U = DMX_L3_U;
#ifndef DMX_L3_RP
#define DMX_L3_RP 512
#endif
constexpr uint32_t DF_L3_RP = DMX_L3_RP;
// level 2: run-continuation test of the match rounds (see run_rounds).  Measured on 1 GiB (ms):
// repeat 4.18 -> 3.40, zeros 3.88 -> 3.26, bmp 4.05 -> 3.48, mixed 6.67 -> 6.60; the bookkeeping
// costs text 8.89 -> 9.14 and random 5.48 -> 5.71 (no runs there)
#ifndef DMX_DF_SKIP
#define DMX_DF_SKIP 1
#endif
constexpr bool DF_SKIP = DMX_DF_SKIP != 0;
// the front kernel counts the symbols (the emission kernel skips its histogram pass)
#ifndef DMX_DF_HIST
#define DMX_DF_HIST 0
#endif
// (round 4's DMX_EM_PREF -- token words loaded two blocks ahead -- measured no gain, DESIGN
// 4.1, and was removed in round 6 with the per-part token sources of 64 KiB blocks)
// level 2: half-size parse chunks for segments without a run (see the parse walk)
#ifndef DMX_DF_ADAPT
#define DMX_DF_ADAPT 0
#endif
// token-word count of a segment without any match (k_deflate_emit then reads its input's bytes)
constexpr uint32_t EM_ALL_LITERALS = 0xFFFFFFFFu;

// ---------------------------------------------------------------------------------------
// block primitives
// ---------------------------------------------------------------------------------------

// threadIdx.x behind an empty volatile asm: the persistent segment loop would otherwise hoist
// every thread-dependent address of every phase out of the loop (all live at once: spills)
__device__ __forceinline__ int df_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// exclusive block scan of one value per thread; returns the prefix, *total gets the sum
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    const int t = df_tid(), w = t >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if ((t & 63) == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < DF_NT / 64; i++) {
        const uint32_t s = scratch[i];
        if (i < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// Length-limited code lengths for freq[0..nsym) (nsym <= 512), written to lens[].  One
// wavefront, registers only:
//  1. keys (f << 9 | 511 - sym) sorted descending (register bitonic network) -> rank order
//  2. L = round(log2(F/f)) clamped to [1, maxbits]
//  3. Kraft repair: while sum 2^-L > 1 lengthen the least frequent codes, longest class first
//  4. slack fill: per class of equal length (shortest first) shorten the most frequent codes
//     while the Kraft budget allows; repeat until the code is complete.
// Zero or one used symbol -> two codes of length 1 (complete code, as zlib emits).
// Stands in for FlatHuffmanTree::generateCodeLengths (common.hpp:322-404), a serial
// priority-queue Huffman; this one stays within ~1% of optimal.
// Kraft repair and slack fill on the class sizes cnt[1..15] of a code whose lengths are
// non-decreasing in frequency rank: lengthen the last (least frequent) members of a class while
// the code is over-full, then shorten the first (most frequent) members while slack remains.
// Ends with a complete code (Kraft sum exactly 2^maxbits), as zlib and the reference require.
__device__ __forceinline__ void fit_classes(uint32_t (&cnt)[17], int maxbits) {
    // Kraft sums in units of 2^-maxbits (<= 288 * 2^8: 32-bit); every class weight is a power
    // of two, so the divisions are shifts
    const int32_t U = 1 << maxbits;
    int32_t K = 0;
#pragma unroll
    for (int L = 1; L <= 15; L++) K += L <= maxbits ? (int32_t)cnt[L] << (maxbits - L) : 0;
    while (K > U) {
#pragma unroll
        for (int L = 14; L >= 1; L--) {
            if (L < maxbits && K > U && cnt[L]) {
                const int sh = maxbits - L - 1;  // gain of one lengthening: 2^sh
                const uint32_t need = (uint32_t)((K - U + (1 << sh) - 1) >> sh);
                const uint32_t k = min(need, cnt[L]);
                cnt[L] -= k;
                cnt[L + 1] += k;
                K -= (int32_t)k << sh;
            }
        }
    }
    uint32_t R = (uint32_t)(U - K);
    for (int pass = 0; pass < 64 && R; pass++) {
        bool changed = false;
#pragma unroll
        for (int L = 2; L <= 15; L++) {
            if (L <= maxbits && cnt[L] && (1u << (maxbits - L)) <= R) {
                const uint32_t k = min(cnt[L], R >> (maxbits - L));
                cnt[L] -= k;
                cnt[L - 1] += k;
                R -= k << (maxbits - L);
                changed = true;
            }
        }
        if (!changed) break;
    }
}

// initial length round(log2(F/f)) clamped to [1, maxbits] (0 for f == 0)
__device__ __forceinline__ uint32_t init_len(uint32_t f, uint32_t F, int maxbits) {
    if (!f) return 0;
    // floor(log2(F / f)) without a division: F / f lies in [2^(e-1), 2^(e+1)) for e = the
    // difference of the leading-bit positions, and is >= 2^e exactly when f << e <= F
    const uint32_t e = (uint32_t)(__clz(f) - __clz(F));
    const uint32_t L0 = e - (((uint64_t)f << e) > F ? 1u : 0u);
    const uint64_t a = (uint64_t)f << (L0 + 1);
    const uint32_t L = L0 + ((a * a <= 2ull * F * F) ? 1u : 0u);
    return max(1u, min((uint32_t)maxbits, L));
}

// the same for at most 64 symbols (precode, distance code): one key per lane, 64-key sort
__device__ void wave_build_lengths64(const uint32_t* freq, int nsym, int maxbits, uint8_t* lens) {
    const int lane = lane_id();
    const uint32_t f = lane < nsym ? freq[lane] : 0;
    uint32_t key = f ? (f << 9) | (511 - lane) : 0;
    if (lane < nsym) lens[lane] = 0;
    const uint32_t F = wave_sum(f);
    const uint64_t nzm = __ballot(f != 0);
    if (__popcll(nzm) <= 1) {
        const uint32_t u = nzm ? 64 - __clzll(nzm) : 0;  // highest used symbol + 1
        if (lane == 0) {
            if (u == 0) { lens[0] = 1; lens[1] = 1; }
            else { lens[u - 1] = 1; lens[u - 1 == 0 ? 1 : 0] = 1; }
        }
        return;
    }
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            uint32_t o;
            switch (stride) {
                case 1: o = xor_lane<1>(key); break;
                case 2: o = xor_lane<2>(key); break;
                case 4: o = xor_lane<4>(key); break;
                case 8: o = xor_lane<8>(key); break;
                case 16: o = xor_lane<16>(key); break;
                default: o = xor_lane<32>(key); break;
            }
            const bool lower = (lane & stride) == 0;
            const bool desc = (lane & size) == 0;
            key = (lower == desc) ? max(key, o) : min(key, o);
        }
    }
    const uint32_t L0 = init_len(key >> 9, F, maxbits);
    uint32_t cnt[17];
    cnt[0] = cnt[16] = 0;
#pragma unroll
    for (int L = 1; L <= 15; L++) cnt[L] = __popcll(__ballot(L0 == (uint32_t)L));
    fit_classes(cnt, maxbits);
    uint32_t S = 0, L = 0;
#pragma unroll
    for (int l = 1; l <= 15; l++) {
        L += (uint32_t)lane >= S ? 1u : 0u;
        S += cnt[l];
    }
    if (key >> 9) lens[511 - (key & 511)] = (uint8_t)L;
}

// Canonical codes (RFC 1951 3.2.2; reference FlatHuffmanTree::construct common.hpp:104-145),
// stored bit-reversed for the LSB-first bit packer: codes[s] = (len << 16) | rev(code).
// One wavefront; per-length counts and ranks come from ballots over 64-symbol chunks.
__device__ void wave_assign_codes(const uint8_t* lens, int nsym, uint32_t* codes) {
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
    uint32_t next[16];
    uint32_t code = 0;
    next[0] = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
        code = (code + (k > 1 ? cnt[k - 1] : 0)) << 1;
        next[k] = code;
    }
    for (int c = 0; c < nsym; c += 64) {
        const int s = c + lane;
        const uint32_t L = s < nsym ? lens[s] : 0;
        uint32_t my = 0;
#pragma unroll
        for (int k = 1; k < 16; k++) {
            const uint64_t b = __ballot(L == (uint32_t)k);
            if (L == (uint32_t)k) my = next[k] + __popcll(b & ltmask);
            next[k] += __popcll(b);
        }
        if (s < nsym) codes[s] = L ? (L << 16) | bitrev(my, L) : 0;
    }
}

// common prefix of the bytes at p and q, up to maxl; 16 bytes per step (five independent word
// reads per side, one LDS latency per step).  The segment buffer is zero-padded past its end.
__device__ __forceinline__ uint32_t matchlen(const uint32_t* w, uint32_t p, uint32_t q,
                                             uint32_t maxl) {
    uint32_t L = 0;
    while (L < maxl) {
        const uint32_t ip = (p + L) >> 2, sp = (p + L) & 3, iq = (q + L) >> 2, sq = (q + L) & 3;
        uint32_t a[5], b[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            a[k] = w[ip + k];
            b[k] = w[iq + k];
        }
        uint32_t x = 0, off = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t d = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sp) ^
                               __builtin_amdgcn_alignbyte(b[k + 1], b[k], sq);
            if (!x && d) {
                x = d;
                off = 4 * k;
            }
        }
        if (x) {
            L += off + ((uint32_t)__builtin_ctz(x) >> 3);
            break;
        }
        L += 16;
    }
    return min(L, maxl);
}

// gfx950 LDS takes unaligned 4- and 8-byte reads as one instruction each
typedef uint32_t df_u32u __attribute__((aligned(1)));
typedef uint64_t df_u64u __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t lds_rd32u(const uint32_t* w, uint32_t p) {
    return *reinterpret_cast<const df_u32u*>(reinterpret_cast<const uint8_t*>(w) + p);
}
__device__ __forceinline__ uint64_t lds_rd64u(const uint32_t* w, uint32_t p) {
    return *reinterpret_cast<const df_u64u*>(reinterpret_cast<const uint8_t*>(w) + p);
}
// matchlen with two unaligned 8-byte reads per side per 16 bytes (4 LDS reads instead of 10)
__device__ __forceinline__ uint32_t matchlen_u(const uint32_t* w, uint32_t p, uint32_t q, uint32_t maxl) {
    uint32_t L = 0;
    while (L < maxl) {
        const uint64_t x0 = lds_rd64u(w, p + L) ^ lds_rd64u(w, q + L);
        const uint64_t x1 = lds_rd64u(w, p + L + 8) ^ lds_rd64u(w, q + L + 8);
        if (x0) {
            L += (uint32_t)__builtin_ctzll(x0) >> 3;
            break;
        }
        if (x1) {
            L += 8 + ((uint32_t)__builtin_ctzll(x1) >> 3);
            break;
        }
        L += 16;
    }
    return min(L, maxl);
}

// matchlen by the four lanes of a quad (all four call it with the same p, q, maxl): lane
// `sub` compares bytes [L + 16 sub, L + 16 sub + 16), so one LDS latency covers 64 bytes.
// Reads up to 84 bytes past p + L: beyond maxl they only meet the segment's zero padding or
// the next LDS array, and the result is clamped to maxl.  Same value as matchlen().
__device__ __forceinline__ uint32_t matchlen4(const uint32_t* w, uint32_t p, uint32_t q,
                                              uint32_t maxl, uint32_t sub) {
    uint32_t L = 0;
    while (L < maxl) {
        const uint32_t o = L + 16 * sub;
        const uint32_t ip = (p + o) >> 2, sp = (p + o) & 3, iq = (q + o) >> 2, sq = (q + o) & 3;
        uint32_t a[5], b[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            a[k] = w[ip + k];
            b[k] = w[iq + k];
        }
        uint32_t x = 0, off = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t d = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sp) ^
                               __builtin_amdgcn_alignbyte(b[k + 1], b[k], sq);
            if (!x && d) {
                x = d;
                off = 4 * k;
            }
        }
        // the quad's first mismatch: a min over the quad by two DPP steps (no LDS round trip)
        uint32_t v = x ? 16 * sub + off + ((uint32_t)__builtin_ctz(x) >> 3) : 64u;
        v = min(v, xor_lane<1>(v));
        v = min(v, xor_lane<2>(v));
        if (v < 64) {
            L += v;
            break;
        }
        L += 64;
    }
    return min(L, maxl);
}

__device__ __forceinline__ uint8_t data_byte(const uint32_t* w, uint32_t p) {
    return (uint8_t)(w[p >> 2] >> ((p & 3) * 8));
}

// fixed Huffman code lengths (RFC 1951 3.2.6; reference generateFixedCodes common.hpp:442-482)
__device__ __forceinline__ uint32_t fixed_lit_len(uint32_t s) {
    return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
}
__device__ __forceinline__ uint32_t fixed_lit_code(uint32_t s) {
    uint32_t c = s < 144 ? 0x30 + s : s < 256 ? 0x190 + (s - 144) : s < 280 ? s - 256 : 0xC0 + (s - 280);
    return bitrev(c, fixed_lit_len(s));
}

// RLE plan of one run of code lengths (v, r): zero runs use 18/17, others v then 16s.
// Never a 16 after a 17/18, and sequences never span HLIT/HDIST (the reference
// inflate decodes the two sequences separately, inflate.hpp:216-220, and repeats the last
// *literal* length on 16, inflate.hpp:181).
struct RunPlan {
    uint32_t n18, last18, n17, r17, nlit, n16, last16;  // last18/last16: length of final repeat
};
__device__ __forceinline__ RunPlan plan_run(uint32_t v, uint32_t r) {
    RunPlan p = {0, 0, 0, 0, 0, 0, 0};
    if (v == 0) {
        p.n18 = r / 138;
        p.last18 = 138;
        uint32_t rem = r % 138;
        if (rem >= 11) { p.n18++; p.last18 = rem; }
        else if (rem >= 3) { p.n17 = 1; p.r17 = rem; }
        else p.nlit = rem;
    } else {
        uint32_t q = r - 1;
        p.nlit = 1;
        p.n16 = q / 6;
        p.last16 = 6;
        uint32_t rem = q % 6;
        if (rem >= 3) { p.n16++; p.last16 = rem; }
        else p.nlit += rem;
    }
    return p;
}

// ---------------------------------------------------------------------------------------
// the segment kernel: 1024 threads (16 waves) per segment, one workgroup per CU
// ---------------------------------------------------------------------------------------
template <int SEG>
struct DfSmem {
    static constexpr int NWALK = (SEG + DF_CHUNK - 1) / DF_CHUNK;
    static constexpr int NWALK_MAX = DMX_DF_ADAPT ? (SEG + DF_CHUNK / 2 - 1) / (DF_CHUNK / 2) : NWALK;
    static constexpr int HB = df_hash_bits(SEG);
    static constexpr int HT = 1 << HB;  // entries per hash table
    static constexpr int UW = 2 * HT;
    uint32_t data32[SEG / 4 + 32];  // + 128 B: matchlen4 reads up to 84 B past a match end
    alignas(16) uint16_t cand[SEG + 8];
    // the match rounds' HT pairs {head, first} (one ds_read_b64 per lookup)
    alignas(16) uint32_t U[UW];
    uint32_t mmap[SEG / 32];    // "a verified match of >= 3 starts here" (match rounds)
    uint32_t tokmap[SEG / 32];  // token-start bitmap (parse walk; chunks share boundary words)
    uint16_t lasttok[NWALK_MAX + 1];  // last token start of each parse chunk
    uint32_t scan[4 * DF_NT / 64];
    uint32_t sh[64];  // 44: run candidate, 46: mismatch tag, 48..62: divisor-period tags
    uint32_t hist[DMX_DF_HIST ? 320 : 1];  // the segment's symbol counts (see deflate_tok_stride)
};

// Persistent workgroups: the next segment of this workgroup (seg + gridDim.x) is loaded straight
// into the LDS byte image (global_load_lds, no registers) once the current segment's bytes are
// dead -- after its token words are written -- so its memory latency passes during the stores
// and the loop's bookkeeping.  The loop's closing
// __syncthreads waits for it (an LDS-DMA load counts on vmcnt).
template <int SEG>
__device__ __forceinline__ bool df_prefetch_next(const DeflateArgs& A, uint64_t seg, DfSmem<SEG>& S) {
    const uint64_t nbase = (seg + gridDim.x) * (uint64_t)SEG;
    const bool go = seg + gridDim.x < A.nseg && nbase + SEG <= A.n &&
                    ((reinterpret_cast<uintptr_t>(A.in + nbase) & 15) == 0);
    if (go) {
        const int t = df_tid();
        const uint4* src = reinterpret_cast<const uint4*>(A.in + nbase) + t;
        // one wave-instruction writes 64 x 16 B contiguously from a wave-uniform LDS base
        uint4* dst = reinterpret_cast<uint4*>(S.data32) + (t & ~63);
#pragma unroll
        for (int k = 0; k < SEG / (16 * DF_NT); k++)
            __builtin_amdgcn_global_load_lds(src + k * DF_NT, (__attribute__((address_space(3))) void*)(dst + k * DF_NT),
                                             16, 0, 0);
    }
    return go;
}

// Token ranges: after the parse, thread t owns tokens [t K, (t + 1) K) of the segment in
// position order (K = ceil(tokens / DF_NT)), found from per-word token counts of the token-start
// bitmap.  Every thread then walks the same number of tokens (a wave iterates K times, not the
// maximum over its lanes of a position range's token count), and its bits form one contiguous
// range of the block's bitstream.
struct TokRange {
    uint32_t w, m, n;  // bitmap word of the first token, its bits from that token on, tokens
};
__device__ __forceinline__ uint32_t next_tok(const uint32_t* tokmap, uint32_t& w, uint32_t& m) {
    while (!m) m = tokmap[++w];
    const uint32_t p = w * 32 + __builtin_ctz(m);
    m &= m - 1;
    return p;
}

// L3: level 3 (chain search, lazy parse) -- a separate instantiation, so the level-2 kernel
// carries none of that code (the 1024-thread kernel's register allocation and code size)
template <int SEG, bool L3>
__device__ __forceinline__ void deflate_segment(const DeflateArgs& A, DfSmem<SEG>& S, uint64_t seg,
                                                bool& staged) {
    [[maybe_unused]] constexpr int NWALK = DfSmem<SEG>::NWALK;
    constexpr int HT = DfSmem<SEG>::HT;
    constexpr int NMAP = SEG / 32;
    const int t = df_tid();
    const uint64_t base = seg * (uint64_t)SEG;
    const uint32_t nb = (uint32_t)min((uint64_t)SEG, A.n - base);
    constexpr int level = L3 ? 3 : 2;  // (the front kernel runs at levels 2 and 3 only)
    uint8_t* const dbytes = reinterpret_cast<uint8_t*>(S.data32);
    DMX_PHASE(A.dbg, seg, 0);

    // ---- load the segment into LDS (16 B per lane when aligned) ------------------------
    {
        const uint8_t* src = A.in + base;
        const uint32_t nvec = nb / 16;
        if (staged) {  // loaded during the previous segment (df_prefetch_next)
        } else if ((((uintptr_t)src) & 15) == 0) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src);
            uint4* d4 = reinterpret_cast<uint4*>(S.data32);
            for (uint32_t i = t; i < nvec; i += DF_NT) d4[i] = s4[i];
            for (uint32_t i = nvec * 16 + t; i < nb; i += DF_NT) dbytes[i] = src[i];
        } else {
            for (uint32_t i = t; i < nb; i += DF_NT) dbytes[i] = src[i];
        }
        // zero padding after the data (match compares read up to 8 bytes past)
        for (uint32_t i = nb + t; i < ((nb + 3) & ~3u) + 32; i += DF_NT) dbytes[i] = 0;
        if (t < NMAP) S.tokmap[t] = 0;
        if (t == 0) S.sh[46] = 0;  // the match rounds' mismatch tag (run continuation)
        if (t >= 48 && t < 63) S.sh[t] = 0;  // its divisor-period tags
        if (DMX_DF_HIST && t < 320) S.hist[t] = 0;
        if (level >= 2)
            for (int i = t; i < 2 * HT; i += DF_NT) S.U[i] = 0;
    }
    __syncthreads();
    DMX_PHASE(A.dbg, seg, 1);
    staged = false;

    if (level != 0) {
        bool any_skip = false;  // (uniform) the run continuation took a round of this segment
        // ---- match candidates: rounds of 2*DF_NT positions, two per thread ---------------
        if (level >= 2) {
            // Table entries carry a fingerprint of the 4-byte key (product bits below the hash
            // bits), so a lookup verifies its candidate without reading the candidate's bytes:
            //   first = round(4) | 0x7FFF - p (15) | fp13      (atomicMax: earliest p in round;
            //           shorter level-3 rounds: round(4 + e) and fp(13 - e))
            //   head  = p + 1 (16) | fp16                       (atomicMax: latest p, 0 = none)
            // stored as {head, first} pairs, one ds_read_b64 per lookup.  A fingerprint match
            // that is not a key match is rare; the parse walk then finds a match length < 3
            // and emits a literal.  Thread t handles the consecutive positions p0 = r0 + 2t and
            // p0 + 1 of each round: both keys come from one pair of words, both candidates go
            // out as one 32-bit store, and the neighbour tests that skip redundant table updates
            // are mostly in-thread.  A position's latest-occurrence update waits one round (a
            // lookup must not see later positions of its own round); the first occurrence in a
            // round is resolved by the round number in the entry.
            constexpr uint32_t HB = DfSmem<SEG>::HB;
            const uint2* const tab = reinterpret_cast<const uint2*>(S.U);
            uint32_t* const cand32 = reinterpret_cast<uint32_t*>(S.cand);
            uint32_t ph0 = 0, ph1 = 0, pp0 = 0, pf0 = 0, pf1 = 0;  // previous round: hashes, p0, fp16s
            bool pok0 = false, pok1 = false;
            constexpr uint32_t NOH = 0xFFFFFFFFu;  // "no hash" for the neighbour compares
            if (level == 3 && DF_L3_LINK_ROUNDS) {
                // Level 3 builds links for the chain search below: rounds of DF_L3_ROUND
                // positions, each position linked to the latest occurrence of its key before
                // its round (or to its pair partner, in-thread), so consecutive links skip at
                // most one round -- the hash chain of the reference's getMatchesSlow scan
                // (deflate.hpp:268-304) in a form the parallel rounds can build.
                const bool act = t < DF_L3_ROUND / 2;
                for (uint32_t r0 = 0; r0 < nb; r0 += DF_L3_ROUND) {
                    const uint32_t p0 = r0 + 2 * t, p1 = p0 + 1;
                    uint32_t h0 = NOH, h1 = NOH, fa0 = 0, fa1 = 0, k0 = 0, k1 = 1;
                    bool ok0 = false, ok1 = false;
                    if (act) {
                        const uint32_t wa = S.data32[p0 >> 2], wb = S.data32[(p0 >> 2) + 1];
                        k0 = __builtin_amdgcn_alignbyte(wb, wa, p0 & 3);
                        k1 = __builtin_amdgcn_alignbyte(wb, wa, (p0 & 3) + 1);
                        const uint32_t prod0 = k0 * 0x1E35A7BDu, prod1 = k1 * 0x1E35A7BDu;
                        ok0 = p0 + 4 <= nb;
                        ok1 = p1 + 4 <= nb;
                        h0 = ok0 ? prod0 >> (32 - HB) : NOH;
                        h1 = ok1 ? prod1 >> (32 - HB) : NOH;
                        fa0 = (prod0 >> (32 - HB - 16)) & 0xFFFFu;
                        fa1 = (prod1 >> (32 - HB - 16)) & 0xFFFFu;
                        const uint32_t hn = (uint32_t)__builtin_amdgcn_update_dpp((int)NOH, (int)(pok0 ? ph0 : NOH), 0x101, 0xF, 0xF, false);
                        if (pok0 && ph0 != (pok1 ? ph1 : NOH)) atomicMax(&S.U[2 * ph0], ((pp0 + 1) << 16) | pf0);
                        if (pok1 && ph1 != hn) atomicMax(&S.U[2 * ph1], ((pp0 + 2) << 16) | pf1);
                    }
                    __syncthreads();
                    if (act) {
                        const uint32_t e0 = tab[ok0 ? h0 : 0u].x, e1 = tab[ok1 ? h1 : 0u].x;
                        const uint32_t c0 = ok0 && e0 && (e0 & 0xFFFFu) == fa0 ? p0 + 1u - (e0 >> 16) : 0u;
                        uint32_t c1 = ok1 && e1 && (e1 & 0xFFFFu) == fa1 ? p1 + 1u - (e1 >> 16) : 0u;
                        if (ok1 && ok0 && k1 == k0) c1 = 1;
                        cand32[p0 >> 1] = c0 | (c1 << 16);
                    }
                    ph0 = h0;
                    ph1 = h1;
                    pp0 = p0;
                    pf0 = fa0;
                    pf1 = fa1;
                    pok0 = ok0;
                    pok1 = ok1;
                    __syncthreads();
                }
            } else {
                // One round; cur receives this round's hashes for the next round's latest-occurrence
                // updates, prev holds the previous round's.  Rounds go in pairs with the two states
                // swapping roles (no register copies), and rounds that lie wholly inside the
                // segment skip the bounds tests (`full`, a constant in each call).  Rounds of RP
                // positions: 2 * DF_NT at level 2; level 3 may use shorter rounds (DF_L3_RP, the
                // first RP / 2 threads active) so the first-in-round links skip fewer occurrences
                // for its chain search, with a wider round number and a narrower fingerprint.
                struct RoundState {
                    uint32_t h0, h1, p0, f0, f1;
                    bool ok0, ok1;
                };
                bool skipped = false;  // a round skipped by the run continuation (uniform)
                auto run_rounds = [&](auto rpc) {
                    constexpr uint32_t RP = decltype(rpc)::value;
                    constexpr uint32_t NR = SEG / RP;
                    constexpr uint32_t TAGB = NR <= 16 ? 4 : NR <= 32 ? 5 : NR <= 64 ? 6 : 7;
                    static_assert(NR <= 128, "round number is at most 7 bits");
                    constexpr uint32_t FPB = 17 - TAGB;  // fingerprint bits in the first entry
                    const bool act = RP >= 2 * DF_NT || t < (int)(RP / 2);
                    const uint32_t tt = RP >= 2 * DF_NT ? (uint32_t)t : (uint32_t)t & (RP / 2 - 1);
                    // Run continuation (level 2): after a round in which at least 120 of the last
                    // 128 positions found a candidate, the next round tests the rest of the segment at one
                    // distance d (the candidate of that round's last position): the words at q and
                    // q - d, neighbouring lanes on neighbouring words (no bank conflicts), the first
                    // mismatch by an LDS atomic.  Every round
                    // whose positions all lie before it (their 4-byte keys verified at d) takes d
                    // as every candidate and skips the hash table: no atomics, no lookup, no
                    // barrier (its positions are never entered, so later rounds see older,
                    // farther occurrences of those keys: still verified candidates).  Long runs of
                    // one period (zeros, a repeated record, an image row) cost one compare per
                    // byte instead of two atomics and a lookup per position -- the parallel form of
                    // zlib not inserting the positions inside a long match (deflate_fast's
                    // max_insert_length).  A run that ends inside the tested round waits 1, 2, 4
                    // .. 16 normal rounds before the next test.  LDS: sh[44] = that candidate (0:
                    // no test), written by the round's last thread; sh[46] = (round + 1) << 16 |
                    // 0xFFFF - first mismatch (atomicMax: no reset between rounds).
                    constexpr bool SKIP = DF_SKIP && RP == 2 * DF_NT;
                    uint32_t skip_d = 0, skip_end = 0, wait = 0, backoff = 1;  // uniform
                    skipped = false;
                    bool pend = false;  // the previous round was a normal one (sh[44] is read)
                    auto round = [&](uint32_t r0, uint32_t rr, RoundState& cur, const RoundState& prev, auto full) {
                        constexpr bool FULL = decltype(full)::value;
                        const uint32_t p0 = r0 + 2 * tt, p1 = p0 + 1;
                        if (SKIP && skip_d) {
                            if (r0 + RP <= skip_end || skip_end >= nb) {  // inside the verified run
                                if (FULL || p0 < nb)
                                    cand32[p0 >> 1] = (FULL || p0 + 4 <= nb ? skip_d : 0u) |
                                                      ((FULL || p1 + 4 <= nb ? skip_d : 0u) << 16);
                                cur = RoundState{NOH, NOH, p0, 0, 0, false, false};
                                skipped = true;
                                return;
                            }
                            skip_d = 0;
                        }
                        uint32_t dlr = 0;  // (issued first: its latency overlaps the data words')
                        if (SKIP && pend) dlr = S.sh[44];
                        const uint32_t i0 = p0 >> 2, sh = p0 & 3;  // sh = 0 or 2
                        const uint32_t wa = S.data32[i0], wb = S.data32[i0 + 1];
                        const uint32_t k0 = __builtin_amdgcn_alignbyte(wb, wa, sh);
                        const uint32_t k1 = __builtin_amdgcn_alignbyte(wb, wa, sh + 1);
                        const uint32_t prod0 = k0 * 0x1E35A7BDu;
                        const uint32_t prod1 = k1 * 0x1E35A7BDu;
                        const bool ok0 = act && (FULL || p0 + 4 <= nb), ok1 = act && (FULL || p1 + 4 <= nb);
                        const uint32_t h0 = ok0 ? prod0 >> (32 - HB) : NOH, h1 = ok1 ? prod1 >> (32 - HB) : NOH;
                        const uint32_t fa0 = (prod0 >> (32 - HB - 16)) & 0xFFFFu, fa1 = (prod1 >> (32 - HB - 16)) & 0xFFFFu;
                        // first occurrence in this round: p1 needs no update when p0 has its hash, p0
                        // none when p0 - 1 (the previous lane's p1, by DPP within rows of 16) has it
                        // (issued before the head updates, which do not wait for the data words: the
                        // wait for the words then finds no atomic in flight)
                        const uint32_t hl = (uint32_t)__builtin_amdgcn_update_dpp((int)NOH, (int)h1, 0x111, 0xF, 0xF, false);
                        const uint32_t rtag = rr << (32 - TAGB);
                        if (ok0 && h0 != hl)
                            atomicMax(&S.U[2 * h0 + 1], rtag | ((0x7FFFu - p0) << FPB) | (fa0 >> (16 - FPB)));
                        if (ok1 && h1 != h0)
                            atomicMax(&S.U[2 * h1 + 1], rtag | ((0x7FFFu - p1) << FPB) | (fa1 >> (16 - FPB)));
                        // latest occurrence, for the previous round's positions: its p0 needs no update
                        // when its p0 + 1 has the hash, p0 + 1 none when p0 + 2 (the next lane's) has it
                        const uint32_t hn = (uint32_t)__builtin_amdgcn_update_dpp((int)NOH, (int)(prev.ok0 ? prev.h0 : NOH), 0x101, 0xF, 0xF, false);
                        if (prev.ok0 && prev.h0 != (prev.ok1 ? prev.h1 : NOH))
                            atomicMax(&S.U[2 * prev.h0], ((prev.p0 + 1) << 16) | prev.f0);
                        if (prev.ok1 && prev.h1 != hn) atomicMax(&S.U[2 * prev.h1], ((prev.p0 + 2) << 16) | prev.f1);
                        bool tested = false;
                        if (SKIP && pend) {
                            pend = false;
                            uint32_t dl = __builtin_amdgcn_readfirstlane(dlr);
                            wait -= wait ? 1u : 0u;
#ifdef DMX_DF_SKIPDBG
                            if (seg == 10 && t == 0) printf("seg %u round %u dl %u wait %u\n", (unsigned)seg, rr, dl, wait);
#endif
                            if (!wait && dl) {
                                tested = true;
                                // Periodic data: the trigger's candidate is a first occurrence in an
                                // earlier round, often a multiple of the period.  The largest k <= 16
                                // (dl % k == 0) whose dl / k repeats the 256 bytes at r0 gives the
                                // tested distance (64 threads per k, one word each; a mismatch tags
                                // sh[48 + k - 2] with the round); the test below then verifies it.
                                {
                                    const uint32_t ki = (uint32_t)t >> 6, k = ki + 2, bq = r0 + 4 * ((uint32_t)t & 63);
                                    if (ki < 15 && dl % k == 0 && bq + 4 <= nb) {
                                        const uint32_t dk = dl / k, ia = (bq - dk) >> 2, sk = (bq - dk) & 3;
                                        if (S.data32[bq >> 2] != __builtin_amdgcn_alignbyte(S.data32[ia + 1], S.data32[ia], sk))
                                            atomicMax(&S.sh[48 + ki], rr + 1);
                                    }
                                }
                                __syncthreads();  // (uniform: dl and wait are the same in every wave)
                                uint32_t dsel = dl;
#pragma unroll
                                for (uint32_t k = 2; k <= 16; k++)
                                    dsel = (dl % k == 0 && S.sh[48 + k - 2] != rr + 1) ? dl / k : dsel;
                                dl = __builtin_amdgcn_readfirstlane(dsel);
                                // words r0 / 4 + t + 1024 j (neighbouring lanes, neighbouring words:
                                // no bank conflicts) against the words dl bytes before them
                                skip_d = dl;
                                const uint32_t sa = (r0 - dl) & 3;  // (r0 is a multiple of 4)
                                uint32_t mm = 0xFFFFFFFFu;
#pragma unroll
                                for (int j = 7; j >= 0; j--) {
                                    const uint32_t bq = r0 + 4 * ((uint32_t)t + DF_NT * j);
                                    if (bq < nb) {
                                        const uint32_t ia = (bq - dl) >> 2;
                                        const uint32_t df = S.data32[bq >> 2] ^
                                                            __builtin_amdgcn_alignbyte(S.data32[ia + 1], S.data32[ia], sa);
                                        mm = df ? bq + ((uint32_t)__builtin_ctz(df) >> 3) : mm;
                                    }
                                }
                                if (mm != 0xFFFFFFFFu) atomicMax(&S.sh[46], ((rr + 1) << 16) | (0xFFFFu - mm));
                            }
                        }
                        __syncthreads();
                        if (SKIP && tested) {
                            // positions p < m - 3 have their key verified at skip_d (m: first mismatch)
                            const uint32_t mt = __builtin_amdgcn_readfirstlane(S.sh[46]);
                            const uint32_t m = (mt >> 16) == rr + 1 ? 0xFFFFu - (mt & 0xFFFFu) : 0xFFFFFFFFu;
                            skip_end = m >= nb ? nb : (m >= 3 ? m - 3 : 0u);
#ifdef DMX_DF_SKIPDBG
                            if (seg == 10 && t == 0) printf("seg %u round %u tested m %u skip_end %u\n", (unsigned)seg, rr, m, skip_end);
#endif
                            if (r0 + RP <= skip_end || skip_end >= nb) {  // this round is inside the run
                                if (act && (FULL || p0 < nb))
                                    cand32[p0 >> 1] = (ok0 ? skip_d : 0u) | ((ok1 ? skip_d : 0u) << 16);
                                cur = RoundState{NOH, NOH, p0, 0, 0, false, false};
                                backoff = 1;
                                skipped = true;
                                return;
                            }
                            skip_d = 0;
                            wait = backoff;
                            backoff = min(2 * backoff, 16u);
                        }
                        uint2 e0 = tab[ok0 ? h0 : 0u], e1 = tab[ok1 ? h1 : 0u];
                        // both halves now: otherwise the compiler sinks the head half of e0 into the
                        // not-first-in-round branch, a second LDS round trip after the first
                        asm volatile("" : "+v"(e0.x), "+v"(e0.y), "+v"(e1.x), "+v"(e1.y));
                        auto pick = [&](uint2 e, uint32_t p, uint32_t fa, bool ok) -> uint32_t {
                            const uint32_t f = e.y, hd = e.x;
                            const uint32_t q = 0x7FFFu - ((f >> FPB) & 0x7FFFu);
                            const bool fr = ((f >> (32 - TAGB)) == rr) & (q < p) &
                                            ((f & ((1u << FPB) - 1)) == (fa >> (16 - FPB)));
                            const bool lt = (hd != 0u) & ((hd & 0xFFFFu) == fa);
                            const uint32_t c = fr ? p - q : (lt ? p + 1u - (hd >> 16) : 0u);
                            return ok ? c : 0u;
                        };
                        const uint32_t c0 = pick(e0, p0, fa0, ok0), c1 = pick(e1, p1, fa1, ok1);
                        if (act && (FULL || p0 < nb)) cand32[p0 >> 1] = c0 | (c1 << 16);
                        cur = RoundState{h0, h1, p0, fa0, fa1, ok0, ok1};
                        if (SKIP) {  // the last wave: (nearly) all its positions have a candidate?
                            if (t >= DF_NT - 64) {
                                // (>= 120 of its 128: collided hash buckets leave a few without)
                                const uint32_t nc = (uint32_t)__popcll(__ballot(c0 != 0u)) + (uint32_t)__popcll(__ballot(c1 != 0u));
                                if (t == DF_NT - 1) S.sh[44] = nc >= 120 ? c1 : 0u;
                            }
                            pend = FULL;
                        }
                        __syncthreads();
                    };
                    using Full = std::integral_constant<bool, true>;
                    using Part = std::integral_constant<bool, false>;
                    const DeflateArgs& Ar = A;  // (shadowed by the round states below)
                    RoundState A = {0, 0, 0, 0, 0, false, false}, B = A;
                    uint32_t r0 = 0, rr = 0;
                    for (; r0 + 2 * RP + 3 <= nb; r0 += 2 * RP, rr += 2) {  // two full rounds
                        round(r0, rr, A, B, Full{});
                        if (rr == 0) DMX_PHASE(Ar.dbg, seg, 12);
                        round(r0 + RP, rr + 1, B, A, Full{});
                        if (rr == 0) DMX_PHASE(Ar.dbg, seg, 13);
                    }
                    for (; r0 < nb; r0 += RP, rr++) {  // the rest (the last may be partial)
                        round(r0, rr, A, B, Part{});
                        const RoundState x = A;
                        A = B;
                        B = x;
                    }
                };
                if (level == 3 && DF_L3_RP != 2 * DF_NT)
                    run_rounds(std::integral_constant<uint32_t, DF_L3_RP>{});
                else
                    run_rounds(std::integral_constant<uint32_t, 2 * DF_NT>{});
                if (DF_SKIP && skipped) __syncthreads();  // skipped rounds end without a barrier
                any_skip = skipped;
            }
            DMX_PHASE(A.dbg, seg, 14);
        }
        if (level == 3) {
            // ---- level 3: deeper search along the candidate chains ----------------------------
            // cand[q] links q to an earlier occurrence of its 4-byte key, so p -> p - cand[p] ->
            // ... walks the occurrences of p's key from the most recent back (a hash chain whose
            // links the match rounds already made).  Every position takes the longest match
            // among the first DF_L3_DEPTH links (the nearest on ties; stop at the longest
            // possible).  Thread t handles positions t + DF_NT k; the results stay in registers
            // until every chain walk is done, so the links read are always the rounds' (the
            // output does not depend on scheduling).  Replaces the reference's O(W^2) backward
            // scan LZ77::getMatchesSlow (deflate.hpp:268-304), whose lengths above 258 turn into
            // literal 0x00 bytes (SURVEY A-2); here matches stay within 258 and the parse chunk.
            constexpr int KP = SEG / DF_NT;  // positions per thread
            uint32_t best[KP / 2];
#pragma unroll
            for (int k = 0; k < KP; k++) {
                const uint32_t p = t + DF_NT * k;
                uint32_t bd = 0;
                const uint32_t d0 = p < nb ? S.cand[p] : 0u;
                if (d0) {
                    const uint32_t hi = min(p / DF_CHUNK * DF_CHUNK + DF_CHUNK, nb);
                    const uint32_t maxl = min(258u, hi - p);
                    // The first link: its length up to DF_L3_LONG bytes; a first link that long
                    // ends the search (periodic data, an image row: every link is that long,
                    // and the parse measures the chosen one in full).  Then a link can only be
                    // longer if the 4 bytes ending at offset bl match as well (zlib's scan_end
                    // test, widened): one word compare per link, the full length only for the
                    // links that pass.
                    auto ml = [&](uint32_t a, uint32_t b, uint32_t m) {
                        return DF_L3_U >= 2 ? matchlen_u(S.data32, a, b, m) : matchlen(S.data32, a, b, m);
                    };
                    auto rd = [&](uint32_t a) {
                        return DF_L3_U >= 1 ? lds_rd32u(S.data32, a) : ld32u(S.data32, a);
                    };
                    uint32_t q = p - d0;
                    // (the first link with aligned words: neighbouring lanes read neighbouring
                    // bytes here, which unaligned 8-byte reads serve slower -- repeat +46 %)
                    uint32_t bl = DF_L3_U >= 3 ? matchlen(S.data32, p, q, min(maxl, DF_L3_LONG))
                                               : ml(p, q, min(maxl, DF_L3_LONG));
                    if (bl >= 3) bd = d0;
                    else bl = 2;  // (a fingerprint collision: no match yet)
                    uint32_t tail = bl >= 3 ? rd(p + bl - 3) : 0u;
                    for (int hop = 1; hop < DF_L3_DEPTH && bl < maxl && bl < DF_L3_LONG; hop++) {
                        const uint32_t dq = S.cand[q];
                        if (!dq) break;
                        q -= dq;
                        if (bl >= 3 && rd(q + bl - 3) != tail) continue;
                        const uint32_t L = ml(p, q, maxl);
                        if (L > bl) {
                            bl = L;
                            bd = p - q;
                            tail = rd(p + bl - 3);
                        }
                    }
                }
                if (k & 1) best[k / 2] |= bd << 16;
                else best[k / 2] = bd;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KP; k++) {
                const uint32_t p = t + DF_NT * k;
                if (p < nb) S.cand[p] = (uint16_t)(k & 1 ? best[k / 2] >> 16 : best[k / 2] & 0xFFFFu);
            }
            __syncthreads();
        }
        if (level >= 2) {
            // match bitmap from the candidates: bit p = "a candidate starts at p"
            for (uint32_t w = t; w < NMAP; w += DF_NT) {
                const uint4* c4 = reinterpret_cast<const uint4*>(S.cand + 32 * w);
                uint32_t m = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint4 v = c4[k];
                    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        m |= ((x[j] & 0xFFFFu) ? 1u : 0u) << (8 * k + 2 * j);
                        m |= ((x[j] >> 16) ? 1u : 0u) << (8 * k + 2 * j + 1);
                    }
                }
                const uint32_t b0 = 32 * w;  // positions past the segment end hold stale entries
                S.mmap[w] = b0 + 32 <= nb ? m : (nb > b0 ? m & ((1u << (nb - b0)) - 1u) : 0u);
            }
            __syncthreads();
        }
        DMX_PHASE(A.dbg, seg, 2);

        // ---- parse walk: one DF_CHUNK-byte chunk per quad of lanes (the four walk in step and
        //      share the match-length compares, matchlen4); jumps over literal runs with the
        //      match bitmap, ORs token starts into tokmap (neighbouring chunks share words) -----
        // DMX_DF_ADAPT: at level 2, a segment without a run (no round taken by the run
        // continuation: short matches, text-like) is parsed in half-size chunks, twice the
        // walkers; a segment with one keeps 258-byte chunks, whose matches reach the maximum
        const uint32_t CH = (DMX_DF_ADAPT && level == 2 && !any_skip) ? (uint32_t)DF_CHUNK / 2 : (uint32_t)DF_CHUNK;
        const uint32_t nwalk = (nb + CH - 1) / CH;
        if (level >= 2 && (uint32_t)t < 4 * nwalk) {
            const uint32_t sub = t & 3;
            const bool lead = sub == 0;
            const uint32_t lo = (t >> 2) * CH;
            const uint32_t hi = min(lo + CH, nb);
            auto bits_range = [](uint32_t a, uint32_t b, uint32_t w) -> uint32_t {  // [a, b) in word w
                const uint32_t e = b - w * 32;
                return (e >= 32 ? 0xFFFFFFFFu : ((1u << e) - 1u)) & (0xFFFFFFFFu << (a & 31));
            };
            auto full_len = [&](uint32_t q) -> uint32_t {  // < 3 only on a fingerprint collision
                return matchlen4(S.data32, q, q - S.cand[q], min(258u, hi - q), sub);
            };
            uint32_t p = lo, w = lo >> 5, mw = S.mmap[w], tok = 0, lastp = lo;  // lastp: last token
            auto mbit = [&](uint32_t q) -> bool {
                return (S.mmap[q >> 5] >> (q & 31)) & 1u;
            };
            while (p < hi) {
                const uint32_t wi = p >> 5;
                if (wi != w) {
                    if (tok && lead) atomicOr(&S.tokmap[w], tok);
                    w = wi;
                    mw = S.mmap[w];
                    tok = 0;
                }
                const uint32_t m = mw & (0xFFFFFFFFu << (p & 31));
                const uint32_t q = m ? w * 32 + __builtin_ctz(m) : 0xFFFFFFFFu;
                if (q >= hi || !m) {  // literals to the end of the word (or chunk)
                    const uint32_t e = min((w + 1) * 32, hi);
                    tok |= bits_range(p, e, w);
                    lastp = e - 1;
                    p = e;
                    continue;
                }
                tok |= bits_range(p, q, w);  // literals before the match
                p = q;
                lastp = p;
                uint32_t L = full_len(p);
                if (L < 3) {  // fingerprint collision, not a match: a literal
                    tok |= 1u << (p & 31);
                    if (lead) S.cand[p] = 0;
                    p++;
                    continue;
                }
                if (level == 3 && L < 258 && p + 1 < hi && mbit(p + 1)) {
                    if (full_len(p + 1) > L) {  // lazy: literal here, the longer match next
                        tok |= 1u << (p & 31);
                        if (lead) S.cand[p] = 0;
                        p++;
                        continue;
                    }
                }
                if (L >= 32) {
                    // long match: prefer the smallest distance giving the same length -- a short
                    // period (1..4) or a divisor c / k of the candidate (periodic data: a table,
                    // an image row, a repeated record).  Equal distances of consecutive matches
                    // are what the lane decoder merges into one periodic copy.
                    const uint32_t c = S.cand[p];
                    const uint32_t ml = min(258u, hi - p);
                    uint32_t best = c;
                    {   // periods 1..4: one 16-byte compare round (lane sub tests 1 + sub), then
                        // full lengths only for the periods that passed, shortest first
                        const uint32_t dd = 1 + sub;
                        bool pass = false;
                        if (dd < c && dd <= p) {
                            const uint32_t ip = p >> 2, sp = p & 3, iq = (p - dd) >> 2, sq = (p - dd) & 3;
                            uint32_t x = 0;
#pragma unroll
                            for (int k = 0; k < 4; k++)
                                x |= __builtin_amdgcn_alignbyte(S.data32[ip + k + 1], S.data32[ip + k], sp) ^
                                     __builtin_amdgcn_alignbyte(S.data32[iq + k + 1], S.data32[iq + k], sq);
                            pass = x == 0;
                        }
                        const int qb = lane_id() & ~3;
                        uint32_t pm = (uint32_t)(__ballot(pass) >> qb) & 0xFu;
                        while (pm) {
                            const uint32_t d1 = 1 + (uint32_t)__builtin_ctz(pm);
                            pm &= pm - 1;
                            if (matchlen4(S.data32, p, p - d1, ml, sub) >= L) {
                                best = d1;
                                break;
                            }
                        }
                    }
                    if (!DF_SKIP && best == c) {  // one probe at c / k, k the largest divisor <= 8 (a
                                                  // probe per k would serialize across lanes that differ in k)
                        uint32_t k = 1;
#pragma unroll
                        for (uint32_t q = 2; q <= 8; q++) k = (c % q == 0) ? q : k;
                        if (k > 1 && matchlen4(S.data32, p, p - c / k, ml, sub) >= L) best = c / k;
                    }
                    if (DF_SKIP && best == c) {
                        // divisors c / k of the candidate, k <= 16 (the run-continuation rounds give
                        // every position of a run the same, possibly far, multiple of the period): lane sub takes the (sub + 1)-th
                        // largest k dividing c; one 16-byte compare round for the four, then full
                        // lengths for those that passed, smallest distance first
                        uint32_t k = 0, seen = 0;
#pragma unroll
                        for (uint32_t q = 16; q >= 2; q--) {
                            const bool dv = c % q == 0;
                            k = (dv && seen == sub) ? q : k;
                            seen += dv ? 1u : 0u;
                        }
                        const uint32_t dk = k ? c / k : 0u;
                        bool pass = false;
                        if (dk > 4) {  // (1..4 were tested above)
                            const uint32_t ip = p >> 2, sp = p & 3, iq = (p - dk) >> 2, sq = (p - dk) & 3;
                            uint32_t x = 0;
#pragma unroll
                            for (int j = 0; j < 4; j++)
                                x |= __builtin_amdgcn_alignbyte(S.data32[ip + j + 1], S.data32[ip + j], sp) ^
                                     __builtin_amdgcn_alignbyte(S.data32[iq + j + 1], S.data32[iq + j], sq);
                            pass = x == 0;
                        }
                        const int qb = lane_id() & ~3;
                        uint32_t pm = (uint32_t)(__ballot(pass) >> qb) & 0xFu;
                        while (pm) {
                            const int f = __builtin_ctz(pm);
                            pm &= pm - 1;
                            const uint32_t d1 = (uint32_t)__shfl((int)dk, qb + f, 64);
                            if (matchlen4(S.data32, p, p - d1, ml, sub) >= L) {
                                best = d1;
                                break;
                            }
                        }
                    }
                    if (lead) S.cand[p] = (uint16_t)best;
                }
                tok |= 1u << (p & 31);
                if (lead) S.cand[p + 1] = (uint16_t)L;
                p += L;
            }
            if (tok && lead) atomicOr(&S.tokmap[w], tok);
            if (lead) S.lasttok[t >> 2] = (uint16_t)lastp;
        }
        __syncthreads();
        DMX_PHASE(A.dbg, seg, 3);

        // ---- chunk-edge fix-up: matches cross the parse-chunk edges --------------------------
        // The walk clips every match at its chunk's end.  Per edge (one quad each): when the
        // last token of the chunk before it is a match clipped at the edge, its full length at
        // the same distance is measured; if it ends inside a match q of the next chunk's parse,
        // q's remainder (a suffix of a verified match: no compare) or 1..2 literals follow, and
        // the next parse resumes unchanged after q.  Committed when that takes fewer tokens.
        // The extension ends before the next chunk's last token (so does q's match), so every
        // edge's rewrite stays inside [last token of chunk c, last token of chunk c + 1) and the
        // edges are independent.
        if (level >= 2) {
            const uint32_t sub = t & 3, c = t >> 2;
            const uint32_t hb = (c + 1) * CH;  // the edge
            if ((uint32_t)t < 4 * (nwalk - 1) && hb < nb) {
                const uint32_t s0 = S.lasttok[c], d0 = S.cand[s0], L0 = S.cand[s0 + 1];
                const uint32_t sn = S.lasttok[c + 1];  // the extension ends before it
                if (d0 != 0 && s0 + L0 == hb && L0 < 258 && sn >= hb + 2) {
                    const uint32_t Lx = matchlen4(S.data32, s0, s0 - d0, min(258u, sn - 1 - s0), sub);
                    const uint32_t e = s0 + Lx;  // < sn
                    uint32_t q = 0;
                    if (Lx > L0) {  // the next chunk's token at or before e (before sn)
                        uint32_t w = e >> 5;
                        uint32_t m = S.tokmap[w] & (0xFFFFFFFFu >> (31 - (e & 31)));
                        while (!m) m = S.tokmap[--w];
                        q = w * 32 + 31 - (uint32_t)__clz(m);
                    }
                    if (Lx > L0 && sub == 0) {
                        const uint32_t dq = S.cand[q], Lq = q == e ? 0u : S.cand[q + 1];
                        const uint32_t r = q == e ? 0u : q + Lq - e;  // q's bytes from e on
                        const uint32_t sync = q == e ? e : q + Lq;
                        uint32_t old = 0;  // tokens now in [s0, sync)
                        for (uint32_t wi = s0 >> 5; wi <= (sync - 1) >> 5; wi++) {
                            const uint32_t a = max(s0, wi * 32) - wi * 32, z = min(sync, wi * 32 + 32) - wi * 32;
                            const uint32_t rm = (z >= 32 ? 0xFFFFFFFFu : ((1u << z) - 1u)) & (0xFFFFFFFFu << a);
                            old += (uint32_t)__popc(S.tokmap[wi] & rm);
                        }
                        const uint32_t nt = 1 + (r >= 3 ? 1u : r);
                        if (nt < old) {
                            // new token starts: s0 (kept), e (and e + 1 for two literals)
                            uint32_t nb0 = 0, nb1 = 0;  // bits of e, e + 1
                            if (r) {
                                atomicOr(&S.tokmap[e >> 5], 1u << (e & 31));
                                if (r == 2) atomicOr(&S.tokmap[(e + 1) >> 5], 1u << ((e + 1) & 31));
                            }
                            S.cand[s0 + 1] = (uint16_t)Lx;
                            if (r >= 3) {
                                S.cand[e] = (uint16_t)dq;
                                S.cand[e + 1] = (uint16_t)r;
                            } else if (r) {
                                S.cand[e] = 0;
                                if (r == 2) S.cand[e + 1] = 0;
                            }
                            for (uint32_t wi = s0 >> 5; wi <= (sync - 1) >> 5; wi++) {
                                const uint32_t a = max(s0, wi * 32) - wi * 32, z = min(sync, wi * 32 + 32) - wi * 32;
                                const uint32_t rm = (z >= 32 ? 0xFFFFFFFFu : ((1u << z) - 1u)) & (0xFFFFFFFFu << a);
                                nb0 = (s0 >> 5) == wi ? 1u << (s0 & 31) : 0u;
                                nb1 = (r && (e >> 5) == wi ? 1u << (e & 31) : 0u) |
                                      (r == 2 && ((e + 1) >> 5) == wi ? 1u << ((e + 1) & 31) : 0u);
                                atomicAnd(&S.tokmap[wi], ~rm | nb0 | nb1);
                            }
                        }
                    }
                }
            }
            __syncthreads();
        }

        // ---- token ranges (TokRange): per-word token counts, block scan into the match
        //      bitmap (dead after the parse), binary search for the thread's first token ------
        TokRange tr;
        uint32_t tr_total;  // tokens of the segment
        {
            const uint32_t c = t < NMAP ? (uint32_t)__popc(S.tokmap[t]) : 0u;
            uint32_t tot;
            const uint32_t ex = block_excl_scan(c, S.scan, &tot);
            if (t < NMAP) S.mmap[t] = ex;
            __syncthreads();
            tr_total = tot;
            const uint32_t K = (tot + DF_NT - 1) / DF_NT;
            const uint32_t first = min((uint32_t)t * K, tot);
            tr.n = min(first + K, tot) - first;
            uint32_t lo = 0, hi = NMAP;  // largest word lo with pre[lo] <= first
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (S.mmap[mid] <= first) lo = mid;
                else hi = mid;
            }
            tr.w = lo;
            // drop the word's first r tokens: the r-th set bit by a 5-step popcount search
            const uint32_t m = S.tokmap[lo];
            uint32_t b = 0, k = tr.n ? first - S.mmap[lo] : 0u;
#pragma unroll
            for (uint32_t sh = 16; sh >= 1; sh >>= 1) {
                const uint32_t c = (uint32_t)__popc((m >> b) & ((1u << sh) - 1u));
                const bool up = k >= c;
                b += up ? sh : 0u;
                k -= up ? c : 0u;
            }
            tr.m = m & (0xFFFFFFFFu << b);
        }
        DMX_PHASE(A.dbg, seg, 15);
        // ---- token words for k_deflate_emit, in position order: literal runs of up to three
        //      bytes per word, one word per match (count, block scan of the counts, write).  A
        //      segment without a match (every position a token: incompressible data) writes none:
        //      the emission kernel reads its literals from the input -----
        const bool all_lit = tr_total == nb;
        if (all_lit) {
            if (t == 0) A.ntok[seg] = EM_ALL_LITERALS;
            if (DMX_DF_HIST)  // the literal histogram, four bytes per word
                for (uint32_t i = t; 4 * i < nb; i += DF_NT) {
                    const uint32_t x = S.data32[i];
#pragma unroll
                    for (uint32_t b = 0; b < 4; b++)
                        if (4 * i + b < nb) atomicAdd(&S.hist[(x >> (8 * b)) & 0xFFu], 1u);
                }
        } else {
            auto walk = [&](auto emit) {
                uint32_t w = tr.w, m = tr.m, lit = 0, nl = 0;
                for (uint32_t i = 0; i < tr.n; i++) {
                    const uint32_t p = next_tok(S.tokmap, w, m);
                    const uint32_t d = S.cand[p];
                    if (d) {
                        if (nl) emit(lit | (nl << 24));
                        nl = 0;
                        lit = 0;
                        emit(0x80000000u | ((uint32_t)(S.cand[p + 1] - 3) << 16) | (d - 1));
                    } else {
                        lit |= (uint32_t)data_byte(S.data32, p) << (8 * nl);
                        if (++nl == 3) {
                            emit(lit | (3u << 24));
                            nl = 0;
                            lit = 0;
                        }
                    }
                }
                if (nl) emit(lit | (nl << 24));
            };
            uint32_t nw = 0;
            walk([&](uint32_t) { nw++; });
            uint32_t wtot;
            const uint32_t woff = block_excl_scan(nw, S.scan, &wtot);
            uint32_t* const dst = A.tok + seg * (uint64_t)A.tok_stride + woff;
            uint32_t j = 0;
            walk([&](uint32_t v) {
                dst[j++] = v;
                if (DMX_DF_HIST) {  // the symbol counts the emission kernel codes with
                    if (v >> 31) {
                        atomicAdd(&S.hist[len_sym(((v >> 16) & 0xFFu) + 3)], 1u);
                        atomicAdd(&S.hist[288 + dist_sym((v & 0x7FFFu) + 1)], 1u);
                    } else {
                        const uint32_t cnt = (v >> 24) & 3u;
#pragma unroll
                        for (uint32_t b = 0; b < 3; b++)
                            if (b < cnt) atomicAdd(&S.hist[(v >> (8 * b)) & 0xFFu], 1u);
                    }
                }
            });
            if (t == 0) A.ntok[seg] = wtot;
        }
        DMX_PHASE(A.dbg, seg, 11);
        __syncthreads();  // every read of the segment's bytes is done
        if (DMX_DF_HIST && t < (int)kDeflateHistWords)
            A.tok[seg * (uint64_t)A.tok_stride + A.tok_stride - kDeflateHistWords + t] = S.hist[2 * t] | (S.hist[2 * t + 1] << 16);
        staged = df_prefetch_next<SEG>(A, seg, S);
        DMX_PHASE(A.dbg, seg, 10);
    }
}

// The 32 KiB kernel is limited to one workgroup per CU by its LDS (~146 KiB), so the compiler may
// use up to 128 registers; the 16 KiB one fits two workgroups per CU (80 KiB each) only at <= 64
// registers per lane, which amdgpu_waves_per_eu(8) asks for.
// Persistent workgroups (as many as fit the GPU at once): workgroup b compresses segments
// b, b + G, b + 2G, ... and loads each next segment while it works on the current one.
template <int SEG, bool L3>
__device__ __forceinline__ void deflate_segments(const DeflateArgs& A, DfSmem<SEG>& S) {
    bool staged = false;  // S.data32 already holds the segment's bytes
    for (uint64_t seg = blockIdx.x; seg < A.nseg; seg += gridDim.x) {
        deflate_segment<SEG, L3>(A, S, seg, staged);
        __syncthreads();  // the next segment reuses the LDS (and its prefetch has landed)
    }
}
template <int SEG, bool L3>
__global__ __launch_bounds__(DF_NT) void k_deflate_segments(DeflateArgs A) {
    __shared__ DfSmem<SEG> S;
    deflate_segments<SEG, L3>(A, S);
}
template <bool L3>
__global__ __launch_bounds__(DF_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_deflate_segments16(DeflateArgs A) {
    __shared__ DfSmem<16384> S;
    deflate_segments<16384, L3>(A, S);
}

// ---------------------------------------------------------------------------------------
// k_deflate_emit: the entropy stage, ONE WAVEFRONT PER SEGMENT.  k_deflate_segments leaves
// each level-2/3 segment's tokens in HBM as 32-bit words in position order:
//     match        1 | L - 3 (8) << 16 | d - 1 (15)
//     literal run  0 | count (2) << 24 | up to three bytes (24), first byte lowest
// (level 1: the input's own words, four literals each; level 0: none).  A wave takes one
// segment: histogram (LDS atomics into its own table), length-limited lit/len and distance
// codes (em_build_codes), the RLE of the two code-length sequences and the precode, the block
// type by exact size (dynamic / fixed / stored, as the reference's compare deflate.hpp:739-746),
// then the bit packing: blocks of 256 token words, four consecutive words per lane, one wave
// scan of their bit counts, the patterns ORed into an LDS staging window that goes to the
// segment's HBM slot in whole words.  Every step is wave-synchronous (no workgroup barrier):
// the serial parts of a segment (the code build, the header) overlap other segments' work in
// the other waves of the CU instead of idling fifteen waves of a 1024-thread workgroup.
// ---------------------------------------------------------------------------------------
constexpr int EM_NW = 4;          // waves (segments) per 256-thread workgroup
constexpr int EM_FLUSH = 256;     // staged whole words that trigger a flush to HBM
constexpr int EM_STG = 576;       // staging words: EM_FLUSH + one block (256 x 36 bits) + slack
// EmWave: the symbol counts share their LDS with the bit-staging window (1), and the emission
// kernel asks for DMX_EM_OCC waves per SIMD (0: the compiler's choice)
#ifndef DMX_EM_UNION
#define DMX_EM_UNION 1
#endif
#ifndef DMX_EM_OCC
#define DMX_EM_OCC 6
#endif
constexpr int EM_LIT = 288, EM_SYM = 320;  // lit/len symbols at [0, 288), distance at [288, 320)

struct EmWave {
#if DMX_EM_UNION
    // the symbol counts die with the code build; the bit-staging window starts after it
    union {
        uint32_t freq[EM_SYM];
        uint32_t stg[EM_STG];
    };
#else
    uint32_t freq[EM_SYM];
#endif
    uint32_t code[EM_SYM];   // (len << 16) | bit-reversed code
    uint8_t len[EM_SYM];
    uint16_t rk[EM_SYM];     // per symbol slot: half-class | rank in it, then rank in its length;
                             // per header position: run length (run starts), then run bit offset
    uint32_t prefreq[20];
    uint32_t precode[20];
    uint8_t prelen[24];
    uint32_t hcnt[6][20];    // per chunk of 64 symbols: members of half-class k (k < 20)
    uint32_t lcnt[6][16];    // per chunk: members of code length l
    uint32_t kpre[2][20];    // per alphabet: members of the half-classes below k
    uint32_t start[2][16];   // per alphabet: first rank of code length l
    uint32_t next[2][16];    // per alphabet: first canonical code of length l
#if !DMX_EM_UNION
    uint32_t stg[EM_STG];
#endif
};

struct EmCodes {
    uint32_t dyn_tok, fix_tok;  // token bits under the dynamic / the fixed code (EOB included)
    uint32_t nlit, ndist;       // HLIT + 257, HDIST + 1
};

// symbol slot c of a lane: lit/len symbol 64 c + lane (c < 5) or distance symbol lane (c = 5)
__device__ __forceinline__ uint32_t em_slot(int c, int lane) { return c < 5 ? 64 * c + lane : EM_LIT + lane; }
__device__ __forceinline__ bool em_valid(int c, int lane) { return c < 5 ? 64 * c + lane < 286 : lane < 30; }

// One-wave form of the block-parallel code build the 1024-thread kernel used (same lengths,
// same codes): initial lengths round(log2 F/f) clamped to the limit, order (initial length,
// frequency half of the class, symbol) by ballots per 64-symbol chunk, Kraft repair / slack fill
// on the class sizes (fit_classes), lengths by rank ranges, canonical codes (RFC 1951 3.2.2;
// reference FlatHuffmanTree::construct common.hpp:104-145).  Per-symbol state lives in LDS
// (W.rk), not in registers.  Stands in for generateCodeLengths (common.hpp:322-404); the costs
// feed the size compare of deflate.hpp:739-746.
__device__ EmCodes em_build_codes(EmWave& W) {
    const int lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t Fl = 0, nzl = 0, hil = 0;
    for (int c = 0; c < 5; c++) {
        const uint32_t f = em_valid(c, lane) ? W.freq[em_slot(c, lane)] : 0u;
        Fl += f;
        const uint64_t b = __ballot(f != 0);
        nzl += (uint32_t)__popcll(b);
        if (b) hil = 64 * c + 64 - (uint32_t)__clzll(b);
    }
    Fl = wave_sum(Fl);
    const uint32_t f5 = lane < 30 ? W.freq[EM_LIT + lane] : 0u;
    const uint32_t Fd = wave_sum(f5);
    const uint64_t bd = __ballot(f5 != 0);
    const uint32_t nzd = (uint32_t)__popcll(bd), hid = bd ? 64 - (uint32_t)__clzll(bd) : 0u;
    // half-classes, their per-chunk counts (lane k holds the count of half-class k), ranks
    for (int c = 0; c < 6; c++) {
        const uint32_t f = em_valid(c, lane) ? W.freq[em_slot(c, lane)] : 0u;
        const uint32_t F = c < 5 ? Fl : Fd;
        const uint32_t L0 = init_len(f, F, c < 5 ? DF_LIT_MAXBITS : DF_DIST_MAXBITS);
        const uint32_t k0 = L0 ? 2 * L0 + (((uint64_t)f << L0) <= F ? 1u : 0u) : 0u;
        uint32_t mine = 0, w0 = 0;
#pragma unroll
        for (int k = 2; k <= 2 * DF_LIT_MAXBITS + 1; k++) {
            const uint64_t b = __ballot(k0 == (uint32_t)k);
            mine = lane == k ? (uint32_t)__popcll(b) : mine;
            w0 = k0 == (uint32_t)k ? (uint32_t)__popcll(b & lt) : w0;
        }
        if (lane < 20) W.hcnt[c][lane] = mine;
        W.rk[64 * c + lane] = (uint16_t)(k0 | (w0 << 5));
    }
    wave_sync();
    // class sizes per alphabet (lanes 0..19: lit/len, 32..51: distance), start ranks of the
    // half-classes (exclusive scan over k), then fit_classes and the class starts / next codes
    {
        const int a = lane >= 32 ? 1 : 0, k = lane & 31;
        uint32_t v = 0;
        if (k < 20) {
            if (a) v = W.hcnt[5][k];
            else v = W.hcnt[0][k] + W.hcnt[1][k] + W.hcnt[2][k] + W.hcnt[3][k] + W.hcnt[4][k];
        }
        uint32_t inc = v;  // inclusive scan inside each half (rows of 32 lanes)
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
            const uint32_t u = __shfl_up(inc, d, 64);
            if (k >= d) inc += u;
        }
        if (k < 20) W.kpre[a][k] = inc - v;
        uint32_t cnt[17];
        cnt[0] = cnt[16] = 0;
        const uint32_t nz = a ? nzd : nzl;
#pragma unroll
        for (int L = 1; L <= 15; L++) {
            const uint32_t x = (2 * L + 1 < 20) ? (uint32_t)__shfl(v, (a << 5) + 2 * L, 64) +
                                                      (uint32_t)__shfl(v, (a << 5) + 2 * L + 1, 64)
                                                : 0u;
            cnt[L] = nz > 1 ? x : (L == 1 ? 2u : 0u);
        }
        if (nz > 1) fit_classes(cnt, a ? DF_DIST_MAXBITS : DF_LIT_MAXBITS);
        if (k == 0) {
            uint32_t st = 0, code = 0;
#pragma unroll
            for (int L = 1; L <= 15; L++) {
                W.start[a][L] = st;
                st += cnt[L];
                code = (code + cnt[L - 1]) << 1;
                W.next[a][L] = code;
            }
        }
    }
    wave_sync();
    // code lengths by rank; per-chunk ranks within each length
    for (int c = 0; c < 6; c++) {
        const int a = c == 5 ? 1 : 0;
        const bool sym = em_valid(c, lane);
        const uint32_t nz = a ? nzd : nzl;
        uint32_t L = 0;
        if (sym) {
            const uint32_t s = c < 5 ? 64 * c + lane : (uint32_t)lane;
            if (nz > 1) {
                if (W.freq[em_slot(c, lane)]) {
                    const uint32_t r = W.rk[64 * c + lane], k0 = r & 31;
                    uint32_t q = (r >> 5) + W.kpre[a][k0];
                    for (int c2 = 0; c2 < c && !a; c2++) q += W.hcnt[c2][k0];
#pragma unroll
                    for (int l = 1; l <= 15; l++) L += q >= W.start[a][l] ? 1u : 0u;
                }
            } else {  // zero or one used symbol: two codes of length 1 (a complete code)
                const uint32_t u = a ? hid : hil;
                L = (s == (u ? u - 1 : 0u) || s == (u <= 1 ? 1u : 0u)) ? 1u : 0u;
            }
            W.len[em_slot(c, lane)] = (uint8_t)L;
        }
        uint32_t mine = 0, wl = 0;
#pragma unroll
        for (int k = 1; k <= DF_LIT_MAXBITS; k++) {
            const uint64_t b = __ballot(L == (uint32_t)k);
            wl = L == (uint32_t)k ? (uint32_t)__popcll(b & lt) : wl;
            mine = lane == k ? (uint32_t)__popcll(b) : mine;
        }
        if (lane < 16) W.lcnt[c][lane] = mine;
        W.rk[64 * c + lane] = (uint16_t)wl;
    }
    wave_sync();
    uint32_t dyn = 0, fix = 0, hl = 0, hd = 0;
    for (int c = 0; c < 6; c++) {
        const int a = c == 5 ? 1 : 0;
        const bool sym = em_valid(c, lane);
        const uint32_t L = sym ? W.len[em_slot(c, lane)] : 0u;
        if (sym) {
            const uint32_t s = c < 5 ? 64 * c + lane : (uint32_t)lane;
            uint32_t code = 0;
            if (L) {
                uint32_t cc = W.next[a][L] + W.rk[64 * c + lane];
                for (int c2 = 0; c2 < c && !a; c2++) cc += W.lcnt[c2][L];
                code = (L << 16) | bitrev(cc, L);
            }
            W.code[em_slot(c, lane)] = code;
            const uint32_t f = W.freq[em_slot(c, lane)];
            const uint32_t ex = a ? dist_extra(s) : (s > 256 ? len_extra(s) : 0u);
            dyn += f * (L + ex);
            fix += f * ((a ? 5u : fixed_lit_len(s)) + ex);
        }
        const uint64_t used = __ballot(L != 0);
        if (used) {
            const uint32_t h = 64 - (uint32_t)__clzll(used);
            if (a) hd = h;
            else hl = 64 * c + h;
        }
    }
    wave_sync();
    EmCodes r;
    r.dyn_tok = wave_sum(dyn);
    r.fix_tok = wave_sum(fix);
    r.nlit = max(257u, hl);
    r.ndist = max(1u, hd);
    return r;
}

// OR a pattern of n <= 36 bits into the staging window at bit pos
__device__ __forceinline__ void em_put(uint32_t* stg, uint32_t pos, uint64_t pat, uint32_t n) {
    if (!n) return;
    const uint32_t wi = pos >> 5, sh = pos & 31;
    const uint64_t lo = pat << sh;
    atomicOr(&stg[wi], (uint32_t)lo);
    if (sh + n > 32) atomicOr(&stg[wi + 1], (uint32_t)(lo >> 32));
    if (sh + n > 64) atomicOr(&stg[wi + 2], (uint32_t)(pat >> (64 - sh)));
}

// bit pattern of one token word under the codes in W.code (n <= 36)
__device__ __forceinline__ uint64_t em_pattern(const EmWave& W, uint32_t v, uint32_t cnt, uint32_t& n, bool raw) {
    uint64_t pat = 0;
    n = 0;
    if (!raw && (v >> 31)) {
        const uint32_t L = ((v >> 16) & 0xFFu) + 3, d = (v & 0x7FFFu) + 1;
        const uint32_t ls = len_sym(L), ds = dist_sym(d);
        const uint32_t lc = W.code[ls], dc = W.code[EM_LIT + ds];
        pat = lc & 0xFFFFu;
        n = lc >> 16;
        pat |= (uint64_t)(L - len_base(ls)) << n;
        n += len_extra(ls);
        pat |= (uint64_t)(dc & 0xFFFFu) << n;
        n += dc >> 16;
        pat |= (uint64_t)(d - dist_base(ds)) << n;
        n += dist_extra(ds);
        return pat;
    }
#pragma unroll
    for (uint32_t i = 0; i < 4u; i++) {
        if (i < cnt) {
            const uint32_t c = W.code[(v >> (8 * i)) & 0xFFu];
            pat |= (uint64_t)(c & 0xFFFFu) << n;
            n += c >> 16;
        }
    }
    return pat;
}

// staging -> HBM: the first `nw` words of the window go to dst; the partial word moves to the
// window's start, the rest is zeroed (only words up to nw + 1 were ever written)
__device__ __forceinline__ void em_flush(uint32_t* stg, uint32_t* dst, uint32_t nw) {
    const int lane = lane_id();
    // (not unrolled: eight unrolled stores held eight 64-bit addresses, the kernel's register peak)
#pragma unroll 2
    for (uint32_t i = lane; i < nw; i += 64) dst[i] = stg[i];
    wave_sync();
    const uint32_t part = stg[nw];
    wave_sync();
#pragma unroll 2
    for (uint32_t i = lane; i <= nw + 1; i += 64) stg[i] = i == 0 ? part : 0u;
    wave_sync();
}

// DMX_PHASES: one stamp per wave (its lane 0) into the segment's slots 4..9
#define EM_PHASE(dbg, seg, slot)                                                          \
    do {                                                                                  \
        if ((dbg) && lane_id() == 0) (dbg)[(seg) * kPhaseSlots + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// The token source of one front-kernel segment: the whole block, or one 32 KiB half of a
// 64 KiB block (config C4's block size).  Level 1 reads the input's words (four
// literals each; the part's base is 4-aligned when the input is: parts are multiples of 4),
// levels 2-3 the front kernel's words; a part the front kernel found no match in is all
// literals: its input's words too.
struct EmSrc {
    const uint32_t* inw;    // 4-aligned base at or below the part's first input byte
    const uint32_t* tok;    // front-kernel words (raw: unused)
    uint64_t in_words_end;  // readable words from inw
    uint32_t mis;           // the part's first byte - inw
    uint32_t nb;            // input bytes of the part
    uint32_t ntok;          // token words (raw: input words)
    bool raw;
    __device__ uint32_t raw_word(uint32_t k) const {  // input bytes 4k .. 4k + 3 of the part
        const uint32_t x = 4 * k + mis;
        const uint32_t a = inw[x >> 2];
        const uint32_t b = (x >> 2) + 1 < in_words_end ? inw[(x >> 2) + 1] : 0u;
        return mis ? __builtin_amdgcn_alignbyte(b, a, x & 3) : a;
    }
    __device__ void load4(uint32_t blk, uint32_t (&v)[4]) const {
        const uint32_t i0 = blk * 256 + 4 * lane_id();
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = 0;
        if (raw) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (i0 + j < ntok) v[j] = raw_word(i0 + j);
        } else if (i0 + 3 < ntok) {
            const uint4 q = *reinterpret_cast<const uint4*>(tok + i0);  // tok_stride % 4 == 0
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (i0 + j < ntok) v[j] = tok[i0 + j];
        }
    }
    __device__ uint32_t count_of(uint32_t v, uint32_t idx) const {  // literals in the word
        if (raw) return min(4u, nb - 4 * idx);
        return (v >> 31) ? 0u : (v >> 24) & 3u;
    }
};
template <bool RAW>
__device__ EmSrc em_src(const DeflateArgs& A, uint64_t fseg, uint64_t base, uint32_t nb) {
    EmSrc s;
    const uint8_t* const inb = A.in + base;
    s.mis = (uint32_t)(reinterpret_cast<uintptr_t>(inb) & 3);
    s.inw = reinterpret_cast<const uint32_t*>(inb - s.mis);
    s.in_words_end = (A.n - base + s.mis + 3) / 4;
    s.nb = nb;
    s.raw = RAW || A.ntok[fseg] == EM_ALL_LITERALS;
    s.ntok = s.raw ? (nb + 3) / 4 : A.ntok[fseg];
    s.tok = s.raw ? nullptr : A.tok + fseg * (uint64_t)A.tok_stride;
    return s;
}

// stored-block header byte q (0..4): [BFINAL|00] LEN NLEN (deflate.hpp:387-399, padded on the
// global bit position: every stored block here starts byte-aligned)
__device__ __forceinline__ uint32_t em_stored_hdr(uint32_t q, bool fin, uint32_t len) {
    return q == 0 ? (fin ? 1u : 0u) : q == 1 ? len & 0xFFu : q == 2 ? (len >> 8) & 0xFFu
         : q == 3 ? ~len & 0xFFu : (~len >> 8) & 0xFFu;
}

// One block of SEG input bytes.  SEG = 65536 (C4's 64 KiB blocks): the front kernel matched the
// two 32 KiB halves as independent segments (its LDS holds one 32 KiB image; the halves are
// front segments 2s and 2s + 1), and this wave codes both halves' token words as ONE block --
// one histogram, one code, one header -- so the block is a 64 KiB DEFLATE block whose second
// half simply never refers into the first (valid: a reference may, but need not, reach back).
template <int SEG, bool RAW>
__device__ void em_segment(const DeflateArgs& A, EmWave& W, uint64_t seg) {
    constexpr uint32_t NH = SEG > 32768 ? 2u : 1u;  // front segments per block
    constexpr uint32_t HB = (uint32_t)SEG / NH;
    const int lane = lane_id();
    EM_PHASE(A.dbg, seg, 4);
    const uint64_t base = seg * (uint64_t)SEG;
    const uint32_t nb = (uint32_t)min((uint64_t)SEG, A.n - base);
    const uint32_t np = (nb + HB - 1) / HB;  // parts of this block (the last block may be short)
    const bool is_final = (seg + 1 == A.nseg) && A.final_last;
    uint32_t* const slot = reinterpret_cast<uint32_t*>(A.slots + seg * (uint64_t)A.slot_bytes);
    auto part = [&](uint32_t h) { return em_src<RAW>(A, seg * NH + h, base + (uint64_t)h * HB, min(HB, nb - h * HB)); };
    // a stored form longer than 65535 bytes (LEN is 16 bits) is two stored blocks of 32 KiB
    const uint32_t nsto = nb > 65535u ? 2u : 1u;
    const uint32_t n1 = nsto == 2 ? 32768u : nb;
    const uint64_t stored_bytes = 5ull * nsto + nb + (is_final ? 0 : 5);

    if (A.level != 0) {
        // ---- histogram ------------------------------------------------------------------
        if (DMX_DF_HIST && !RAW && NH == 1) {  // the front kernel's counts
            const uint32_t* const hs = A.tok + seg * (uint64_t)A.tok_stride + A.tok_stride - kDeflateHistWords;
            for (int i = lane; i < (int)kDeflateHistWords; i += 64) {
                const uint32_t x = hs[i];
                W.freq[2 * i] = x & 0xFFFFu;
                W.freq[2 * i + 1] = x >> 16;
            }
        } else {
            for (int i = lane; i < EM_SYM; i += 64) W.freq[i] = 0;
            wave_sync();
            for (uint32_t h = 0; h < np; h++) {
                const EmSrc S = part(h);
                const uint32_t nblk = (S.ntok + 255) / 256;
                for (uint32_t blk = 0; blk < nblk; blk++) {
                    uint32_t v[4];
                    S.load4(blk, v);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t idx = blk * 256 + 4 * lane + j;
                        if (idx >= S.ntok) continue;
                        if (!S.raw && (v[j] >> 31)) {
                            atomicAdd(&W.freq[len_sym(((v[j] >> 16) & 0xFFu) + 3)], 1u);
                            atomicAdd(&W.freq[EM_LIT + dist_sym((v[j] & 0x7FFFu) + 1)], 1u);
                        } else {
                            const uint32_t cnt = S.count_of(v[j], idx);
#pragma unroll
                            for (uint32_t i = 0; i < 4u; i++)
                                if (i < cnt) atomicAdd(&W.freq[(v[j] >> (8 * i)) & 0xFFu], 1u);
                        }
                    }
                }
            }
        }
        wave_sync();
        if (lane == 0) atomicAdd(&W.freq[256], 1u);  // end-of-block
        wave_sync();
        EM_PHASE(A.dbg, seg, 5);
        const EmCodes ec = em_build_codes(W);
        EM_PHASE(A.dbg, seg, 6);
        // ---- dynamic header: RLE runs over (len[0..nlit), len[288..288+ndist)) -------------
        const uint32_t nlit = ec.nlit, ndist = ec.ndist, nall = nlit + ndist;
        auto seqv = [&](uint32_t i) -> uint32_t { return i < nlit ? W.len[i] : W.len[EM_LIT + i - nlit]; };
        uint64_t rm[5];  // run starts, one ballot per chunk of 64 positions
        if (lane < 20) W.prefreq[lane] = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            const uint32_t i = 64 * c + lane;
            bool start = false;
            if (i < nall) start = i == 0 || i == nlit || seqv(i - 1) != seqv(i);
            rm[c] = __ballot(start);
        }
        wave_sync();
        for (int c = 0; c < 5; c++) {
            uint32_t rl = 0;
            if ((rm[c] >> lane) & 1) {
                const uint32_t i = 64 * c + lane;
                uint32_t j = nall;
                const uint64_t m = lane < 63 ? rm[c] & (~0ull << (lane + 1)) : 0ull;
                if (m) j = 64 * c + (uint32_t)__builtin_ctzll(m);
                else
                    for (int c2 = 4; c2 > c; c2--)
                        if (rm[c2]) j = 64 * c2 + (uint32_t)__builtin_ctzll(rm[c2]);
                rl = min(j, nall) - i;
                const uint32_t v = seqv(i);
                const RunPlan p = plan_run(v, rl);
                if (p.n18) atomicAdd(&W.prefreq[18], p.n18);
                if (p.n17) atomicAdd(&W.prefreq[17], p.n17);
                if (p.n16) atomicAdd(&W.prefreq[16], p.n16);
                if (p.nlit) atomicAdd(&W.prefreq[v], p.nlit);
            }
            W.rk[64 * c + lane] = (uint16_t)rl;
        }
        wave_sync();
        wave_build_lengths64(W.prefreq, 19, 7, W.prelen);
        wave_sync();
        wave_assign_codes(W.prelen, 19, W.precode);
        wave_sync();
        const uint32_t pv = lane < 19 ? W.prelen[kPerm[lane]] : 0u;
        const uint64_t nzp = __ballot(pv != 0u);
        const uint32_t hclen = max(4u, nzp ? 64u - (uint32_t)__clzll(nzp) : 0u);
        uint32_t rtot = 0;  // run bit offsets (exclusive scan in position order) -> W.rk
        for (int c = 0; c < 5; c++) {
            const uint32_t rl = W.rk[64 * c + lane];
            uint32_t b = 0;
            if (rl) {
                const uint32_t v = seqv(64 * c + lane);
                const RunPlan p = plan_run(v, rl);
                b = p.n18 * (W.prelen[18] + 7) + p.n17 * (W.prelen[17] + 3) + p.n16 * (W.prelen[16] + 2) +
                    p.nlit * W.prelen[v];
            }
            const uint32_t inc = wave_incl_scan(b);
            W.rk[64 * c + lane] = (uint16_t)(rl ? rtot + inc - b : 0xFFFFu);
            rtot += __shfl(inc, 63, 64);
        }
        wave_sync();
        const uint32_t hdr_bits = 14 + 3 * hclen + rtot;
        EM_PHASE(A.dbg, seg, 7);

        // ---- block type by exact size (reference deflate.hpp:739-746 picks the smallest) ----
        const uint64_t dyn_bits = 3ull + hdr_bits + ec.dyn_tok;
        const uint64_t fix_bits = 3ull + ec.fix_tok;
        const bool use_dyn = dyn_bits <= fix_bits;
        const uint64_t bits = use_dyn ? dyn_bits : fix_bits;
        const uint64_t hbytes = is_final ? (bits + 7) / 8 : (bits + 3 + 7) / 8 + 4;
        if (hbytes < stored_bytes) {
            if (!use_dyn) {
                for (int s = lane; s < EM_SYM; s += 64)
                    W.code[s] = s < EM_LIT ? (s < 286 ? (fixed_lit_len(s) << 16) | fixed_lit_code(s) : 0u)
                                           : (s - EM_LIT < 30 ? (5u << 16) | bitrev(s - EM_LIT, 5) : 0u);
            }
#pragma unroll 3
            for (int i = lane; i < EM_STG; i += 64) W.stg[i] = 0;
            wave_sync();
            // ---- header bits ------------------------------------------------------------
            if (lane == 0) {
                uint64_t h = (is_final ? 1u : 0u) | ((use_dyn ? 2u : 1u) << 1);
                if (use_dyn) h |= ((uint64_t)(nlit - 257) << 3) | ((uint64_t)(ndist - 1) << 8) | ((uint64_t)(hclen - 4) << 13);
                em_put(W.stg, 0, h, use_dyn ? 17 : 3);
            }
            if (use_dyn) {
                if (lane < (int)hclen) em_put(W.stg, 17 + 3 * lane, pv, 3);
                const uint32_t rb = 17 + 3 * hclen;
                for (int c = 0; c < 5; c++) {
                    const uint32_t ro = W.rk[64 * c + lane];
                    if (ro == 0xFFFFu) continue;
                    const uint32_t i = 64 * c + lane;
                    const uint32_t v = seqv(i);
                    uint32_t j = nall;  // the run's end: the next start
                    const uint64_t m = lane < 63 ? rm[c] & (~0ull << (lane + 1)) : 0ull;
                    if (m) j = 64 * c + (uint32_t)__builtin_ctzll(m);
                    else
                        for (int c2 = 4; c2 > c; c2--)
                            if (rm[c2]) j = 64 * c2 + (uint32_t)__builtin_ctzll(rm[c2]);
                    const RunPlan p = plan_run(v, min(j, nall) - i);
                    uint32_t pos = rb + ro;
                    auto put = [&](uint32_t sym, uint32_t extra, uint32_t xb) {
                        const uint32_t pc = W.precode[sym];
                        const uint32_t l = pc >> 16;
                        em_put(W.stg, pos, (uint64_t)(pc & 0xFFFFu) | ((uint64_t)extra << l), l + xb);
                        pos += l + xb;
                    };
                    if (v == 0) {
                        for (uint32_t q = 0; q < p.n18; q++) put(18, (q + 1 == p.n18 ? p.last18 : 138) - 11, 7);
                        if (p.n17) put(17, p.r17 - 3, 3);
                        for (uint32_t q = 0; q < p.nlit; q++) put(0, 0, 0);
                    } else {
                        put(v, 0, 0);
                        for (uint32_t q = 0; q < p.n16; q++) put(16, (q + 1 == p.n16 ? p.last16 : 6) - 3, 2);
                        for (uint32_t q = 1; q < p.nlit; q++) put(v, 0, 0);
                    }
                }
            }
            wave_sync();
            // ---- tokens -------------------------------------------------------------------
            uint32_t cur = 3 + (use_dyn ? hdr_bits : 0u);  // bit position in the window
            uint32_t* dst = slot;                          // next HBM word of the slot
            for (uint32_t h = 0; h < np; h++) {
                const EmSrc S = part(h);
                const uint32_t nblk = (S.ntok + 255) / 256;
                for (uint32_t blk = 0; blk < nblk; blk++) {
                    uint32_t v[4], nbit[4];
                    uint64_t pat[4];
                    S.load4(blk, v);
                    uint32_t mine = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t idx = blk * 256 + 4 * lane + j;
                        nbit[j] = 0;
                        pat[j] = 0;
                        if (idx < S.ntok) pat[j] = em_pattern(W, v[j], S.count_of(v[j], idx), nbit[j], S.raw);
                        mine += nbit[j];
                    }
                    const uint32_t inc = wave_incl_scan(mine);
                    uint32_t pos = cur + inc - mine;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        em_put(W.stg, pos, pat[j], nbit[j]);
                        pos += nbit[j];
                    }
                    cur += __shfl(inc, 63, 64);
                    wave_sync();
                    if (cur >= 32u * EM_FLUSH) {
                        const uint32_t nw = cur >> 5;
                        em_flush(W.stg, dst, nw);
                        dst += nw;
                        cur &= 31;
                    }
                }
            }
            EM_PHASE(A.dbg, seg, 8);
            // ---- end of block, then (non-final) the empty stored block 000|pad|0000|FFFF ----
            const uint32_t eob = W.code[256];
            if (lane == 0) em_put(W.stg, cur, eob & 0xFFFFu, eob >> 16);
            const uint32_t end_bits = cur + (eob >> 16);
            const uint32_t tail = is_final ? (end_bits + 7) / 8 : (end_bits + 3 + 7) / 8 + 4;  // bytes in the window
            wave_sync();
            if (lane == 0 && !is_final) {
                atomicOr(&W.stg[(tail - 2) >> 2], 0xFFu << (((tail - 2) & 3) * 8));
                atomicOr(&W.stg[(tail - 1) >> 2], 0xFFu << (((tail - 1) & 3) * 8));
            }
            wave_sync();
            const uint32_t nw = (tail + 3) / 4;
#pragma unroll 2
            for (uint32_t i = lane; i < nw; i += 64) dst[i] = W.stg[i];
            if (lane == 0)
                A.sizes[seg] = (uint32_t)((reinterpret_cast<uint8_t*>(dst) - reinterpret_cast<uint8_t*>(slot)) + tail);
            EM_PHASE(A.dbg, seg, 9);
            return;
        }
    }
    // ---- stored: [BFINAL|00][LEN][NLEN][data] (two such blocks above 65535 bytes), then the
    // empty stored block unless final ------------------------------------------------------
    const uint32_t total = (uint32_t)stored_bytes;
    const uint8_t* const inb = A.in + base;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(inb) & 3);
    const uint32_t* const inw = reinterpret_cast<const uint32_t*>(inb - mis);
    const uint64_t in_words_end = (A.n - base + mis + 3) / 4;  // readable words from inw
    const uint32_t d2 = 10 + n1;  // first output byte of the second block's data (nsto == 2)
    // 16 output bytes per lane and step, four steps in flight (the copy is latency-bound):
    // output bytes [16 k, 16 k + 16) inside a block's data are input bytes shifted by that
    // block's header bytes (5, or 10 in the second block), five input words funnelled by the
    // segment's constant misalignment; headers and the tail go word by word
    const uint32_t n16 = (total + 15) / 16;
    uint4* const slot4 = reinterpret_cast<uint4*>(slot);
    auto data_shift = [&](uint32_t a, uint32_t b) -> uint32_t {  // output bytes [a, b) all data: the shift
        if (a >= 5 && b <= 5 + n1) return 5u;
        if (nsto == 2 && a >= d2 && b <= 10 + nb) return 10u;
        return 0u;
    };
    auto word_at = [&](uint32_t k) -> uint32_t {  // output word k = bytes 4k .. 4k + 3
        uint32_t w = 0;
        if (const uint32_t sh = data_shift(4 * k, 4 * k + 4)) {
            const uint32_t x = 4 * k - sh + mis;  // aligned-base byte of the first
            const uint32_t a = inw[x >> 2];
            const uint32_t b = (x >> 2) + 1 < in_words_end ? inw[(x >> 2) + 1] : 0u;
            w = __builtin_amdgcn_alignbyte(b, a, x & 3);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t pos = 4 * k + j;
                uint32_t byte;
                if (pos < 5) byte = em_stored_hdr(pos, is_final && nsto == 1, n1);
                else if (pos < 5 + n1) byte = inb[pos - 5];
                else if (nsto == 2 && pos < d2) byte = em_stored_hdr(pos - 5 - n1, is_final, nb - n1);
                else if (nsto == 2 && pos < 10 + nb) byte = inb[pos - 10];
                else byte = (!is_final && pos >= 5 * nsto + nb + 3 && pos < total) ? 0xFFu : 0u;
                w |= byte << (8 * j);
            }
        }
        return w;
    };
#pragma unroll 4
    for (uint32_t k4 = lane; k4 < n16; k4 += 64) {
        uint4 o;
        if (const uint32_t sh = data_shift(16 * k4, 16 * k4 + 16)) {
            const uint32_t x = 16 * k4 - sh + mis, i0 = x >> 2, s = x & 3;
            const uint32_t a0 = inw[i0], a1 = inw[i0 + 1], a2 = inw[i0 + 2], a3 = inw[i0 + 3];
            const uint32_t a4 = i0 + 4 < in_words_end ? inw[i0 + 4] : 0u;
            o.x = __builtin_amdgcn_alignbyte(a1, a0, s);
            o.y = __builtin_amdgcn_alignbyte(a2, a1, s);
            o.z = __builtin_amdgcn_alignbyte(a3, a2, s);
            o.w = __builtin_amdgcn_alignbyte(a4, a3, s);
        } else {
            o.x = word_at(4 * k4);
            o.y = word_at(4 * k4 + 1);
            o.z = word_at(4 * k4 + 2);
            o.w = word_at(4 * k4 + 3);
        }
        slot4[k4] = o;
    }
    if (lane == 0) A.sizes[seg] = total;
}

// RAW: level 1 (the input's bytes are the tokens) and level 0; else the front kernel's words
template <int SEG, bool RAW>
__global__ __launch_bounds__(64 * EM_NW)
#if DMX_EM_OCC
__attribute__((amdgpu_waves_per_eu(DMX_EM_OCC)))
#endif
void k_deflate_emit(DeflateArgs A) {
    __shared__ EmWave Ws[EM_NW];
    const uint64_t seg = (uint64_t)blockIdx.x * EM_NW + (threadIdx.x >> 6);
    if (seg >= A.nseg) return;
    em_segment<SEG, RAW>(A, Ws[threadIdx.x >> 6], seg);
}

// exclusive scan of segment sizes -> offsets (single workgroup of 1024 threads).  Thread t owns
// the contiguous run [t per, (t + 1) per) and moves it in batches of 32 sizes: eight 16-byte
// loads issued together (one memory latency per batch), registers summed, a block scan of the
// run totals, then the offsets of each batch written back as 16-byte stores.  A 1 GiB shard
// (32768 sizes) is one batch per thread.
// Exclusive scan of n 32-bit values into 64-bit offsets (+ the total), over blocks of
// SCAN_BLK values, 32 per thread: k_scan_part sums each block, k_scan_apply scans its block
// from the sum of the blocks before it.  (Round 4 scanned with one 1024-thread workgroup: ~20 us
// for the 32768 segment sizes of 1 GiB, the bandwidth of one CU.)
constexpr uint32_t SCAN_NT = 256, SCAN_PER = 32, SCAN_BLK = SCAN_NT * SCAN_PER;
__device__ __forceinline__ void scan_load32(const uint32_t* v, uint64_t i, uint64_t n, bool vec, uint32_t (&x)[32]) {
    if (vec && i + 32 <= n) {
        const uint4* s4 = reinterpret_cast<const uint4*>(v + i);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint4 q = s4[k];
            x[4 * k] = q.x;
            x[4 * k + 1] = q.y;
            x[4 * k + 2] = q.z;
            x[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 32; k++) x[k] = i + k < n ? v[i + k] : 0u;
    }
}
// 64-bit inclusive scan over the workgroup's threads; *all gets the workgroup's sum
__device__ __forceinline__ uint64_t scan_block64(uint64_t s, uint64_t* part, uint64_t* all) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint64_t inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)inc, d, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(inc >> 32), d, 64);
        if (lane >= d) inc += ((uint64_t)hi << 32) | lo;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < (int)(SCAN_NT / 64); w++) {
        const uint64_t v = part[w];
        before += w < wave ? v : 0ull;
        tot += v;
    }
    *all = tot;
    return before + inc;
}
__global__ __launch_bounds__(SCAN_NT) void k_scan_part(const uint32_t* v, uint64_t n, uint64_t* partial) {
    __shared__ uint64_t part[SCAN_NT / 64];
    const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLK + (uint64_t)threadIdx.x * SCAN_PER;
    const bool vec = (reinterpret_cast<uintptr_t>(v) & 15) == 0;
    uint32_t x[32];
    scan_load32(v, i, n, vec, x);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) s += x[k];
    uint64_t all;
    (void)scan_block64(s, part, &all);
    if (threadIdx.x == 0) partial[blockIdx.x] = all;
}
__global__ __launch_bounds__(SCAN_NT) void k_scan_apply(const uint32_t* v, uint64_t n, const uint64_t* partial,
                                                        uint64_t* offs, uint64_t* total) {
    __shared__ uint64_t part[SCAN_NT / 64];
    __shared__ uint64_t base_s;
    const int t = threadIdx.x;
    // the blocks before this one
    uint64_t pb = 0;
    for (uint32_t b = t; b < blockIdx.x; b += SCAN_NT) pb += partial[b];
    uint64_t bsum;
    (void)scan_block64(pb, part, &bsum);
    if (t == 0) base_s = bsum;
    __syncthreads();
    const uint64_t base = base_s;
    const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLK + (uint64_t)t * SCAN_PER;
    const bool vec = ((reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(offs)) & 15) == 0;
    uint32_t x[32];
    scan_load32(v, i, n, vec, x);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) s += x[k];
    uint64_t all;
    uint64_t run = base + scan_block64(s, part, &all) - s;
    uint64_t o[32];
#pragma unroll
    for (int k = 0; k < 32; k++) {
        o[k] = run;
        run += x[k];
    }
    if (vec && i + 32 <= n) {
        ulonglong2* d2 = reinterpret_cast<ulonglong2*>(offs + i);
#pragma unroll
        for (int k = 0; k < 16; k++) d2[k] = make_ulonglong2(o[2 * k], o[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < 32; k++)
            if (i + k < n) offs[i + k] = o[k];
    }
    if (blockIdx.x == gridDim.x - 1 && t == 0) *total = base + all;
}

// copy each segment slot to its place in the contiguous stream
// one wave per segment, four per workgroup (a workgroup per segment was dispatch-bound on
// small segments: 32768 workgroups for ~480 B each on the repeat corpus)
__global__ __launch_bounds__(256) void k_compact(const uint8_t* slots, uint32_t slot_bytes,
                                                  const uint32_t* sizes, const uint64_t* offs,
                                                  uint64_t nseg, uint8_t* out, uint64_t cap) {
    const uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (s >= nseg) return;
    const uint32_t sz = sizes[s];
    const uint64_t o = offs[s];
    const uint8_t* src = slots + s * (uint64_t)slot_bytes;
    if (o + sz > cap) return;
    uint8_t* dst = out + o;
    // align the destination to 4 bytes, then move words built with alignbyte
    const uint32_t head = (uint32_t)((4 - ((uintptr_t)dst & 3)) & 3);
    const uint32_t hb = min(head, sz);
    if (lane < hb) dst[lane] = src[lane];
    if (sz <= hb) return;
    const uint32_t rem = sz - hb;
    const uint32_t nw = rem / 4;
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst + hb);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(src);  // slot is 256-B aligned
    for (uint32_t k = lane; k < nw; k += 64) {
        const uint32_t p = hb + 4 * k;
        dw[k] = __builtin_amdgcn_alignbyte(sw[(p >> 2) + 1], sw[p >> 2], p & 3);
    }
    for (uint32_t i = hb + nw * 4 + lane; i < sz; i += 64) dst[i] = src[i];
}

hipError_t launch_deflate(const DeflateArgs& A, uint32_t seg_bytes, hipStream_t st,
                          hipEvent_t ev_main0, hipEvent_t ev_main1) {
    // persistent grid: the workgroups that fit at once (CUs x workgroups per CU)
    int dev = 0, ncu = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (seg_bytes >= 32768)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_deflate_segments<32768, false>, DF_NT, 0);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_deflate_segments16<false>, DF_NT, 0);
    const uint64_t fit = (uint64_t)max(ncu, 1) * (uint64_t)max(per, 1);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(A.nseg, fit);  // host min(int, int) would truncate
    if (ev_main0) (void)hipEventRecord(ev_main0, st);
    if (grid && A.level >= 2) {  // match finding + parse -> token words (levels 0-1 have none)
        const bool l3 = A.level >= 3;
        if (seg_bytes == 65536) {  // 64 KiB blocks: the front kernel matches their 32 KiB halves
            DeflateArgs H = A;
            H.nseg = (A.n + 32767) / 32768;
            H.dbg = nullptr;
            const uint32_t hg = (uint32_t)std::min<uint64_t>(H.nseg, fit);
            if (l3) hipLaunchKernelGGL((k_deflate_segments<32768, true>), dim3(hg), dim3(DF_NT), 0, st, H);
            else hipLaunchKernelGGL((k_deflate_segments<32768, false>), dim3(hg), dim3(DF_NT), 0, st, H);
        } else if (seg_bytes == 32768) {
            if (l3) hipLaunchKernelGGL((k_deflate_segments<32768, true>), dim3(grid), dim3(DF_NT), 0, st, A);
            else hipLaunchKernelGGL((k_deflate_segments<32768, false>), dim3(grid), dim3(DF_NT), 0, st, A);
        } else {
            if (l3) hipLaunchKernelGGL(k_deflate_segments16<true>, dim3(grid), dim3(DF_NT), 0, st, A);
            else hipLaunchKernelGGL(k_deflate_segments16<false>, dim3(grid), dim3(DF_NT), 0, st, A);
        }
    }
    if (A.nseg) {  // entropy coding and bit packing, one wavefront per segment
        const uint32_t eg = (uint32_t)((A.nseg + EM_NW - 1) / EM_NW);
        const bool raw = A.level < 2;
        if (seg_bytes == 65536) {
            if (raw) hipLaunchKernelGGL((k_deflate_emit<65536, true>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
            else hipLaunchKernelGGL((k_deflate_emit<65536, false>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
        } else if (seg_bytes == 32768) {
            if (raw) hipLaunchKernelGGL((k_deflate_emit<32768, true>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
            else hipLaunchKernelGGL((k_deflate_emit<32768, false>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
        } else {
            if (raw) hipLaunchKernelGGL((k_deflate_emit<16384, true>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
            else hipLaunchKernelGGL((k_deflate_emit<16384, false>), dim3(eg), dim3(64 * EM_NW), 0, st, A);
        }
    }
    if (ev_main1) (void)hipEventRecord(ev_main1, st);
    {
        const hipError_t e = launch_scan_u32(A.sizes, A.offsets, A.nseg, A.total, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_compact, dim3((uint32_t)((A.nseg + 3) / 4)), dim3(256), 0, st, A.slots, A.slot_bytes,
                       A.sizes, A.offsets, A.nseg, A.out, A.cap);
    return hipGetLastError();
}

// the block sums go to offs[n + 1 ..] (offs holds scan_words(n) entries; offs[n] may be total)
uint64_t scan_words(uint64_t n) { return n + 2 + (n + SCAN_BLK - 1) / SCAN_BLK; }
hipError_t launch_scan_u32(const uint32_t* v, uint64_t* offs, uint64_t n, uint64_t* total,
                           hipStream_t st) {
    const uint64_t nb = n ? (n + SCAN_BLK - 1) / SCAN_BLK : 1;
    uint64_t* partial = offs + n + 1;
    if (nb > 1) hipLaunchKernelGGL(k_scan_part, dim3((uint32_t)nb), dim3(SCAN_NT), 0, st, v, n, partial);
    hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nb), dim3(SCAN_NT), 0, st, v, n, partial, offs, total);
    return hipGetLastError();
}

}  // namespace dmx
