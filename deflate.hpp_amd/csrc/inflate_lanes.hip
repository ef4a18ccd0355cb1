// inflate_lanes.hip -- two-phase inflate of segment-structured streams (gfx950).
//
// Phase A, k_inflate_lanes: ONE LANE PER CANDIDATE SEGMENT.  Huffman decoding is serial within
// a segment, but a 1 GiB stream holds ~32K independent segments (libdmx's deflate, or any
// encoder's full-flush points), so 32 segments decode side by side in one wavefront and the
// whole stream is in flight at once.  LDS layout (per segment 1152 B of tables + 128 B shared
// area; 32 segments per one-wave workgroup = 40 KiB, four workgroups per CU): see LN_REGION.
// Phases of a workgroup:
//   1. each lane reads its block header (BTYPE; stored segments are handled right there);
//   2. the wave builds every dynamic segment's precode table in turn (ln_coop_table: ballot
//      counts, canonical order, one table entry per lane);
//   3. each lane decodes its code-length sequence once into bytes (branch-free steps);
//   4. the wave builds every segment's 9-bit lit/len and 6-bit distance tables in turn;
//   5. each lane decodes its tokens: a 64-bit window per symbol from a per-lane LDS ring of
//      the stream (no refill branch), table lookups, select-based token logic.  The decoded
//      tokens go to HBM as 32-bit words:
//     match        1 | L(16) | d-1(15)          consecutive matches with the same distance are
//                                               merged: one periodic copy of their summed length
//     literal run  0 | count(7) = 1..3 | bytes(24)
//     stored       0 | 0 | len(24), then the data's byte offset from the candidate start
// Lanes accept exactly the layout libdmx's deflate emits: one stored / fixed / dynamic block
// (lit/len codes <= 9 bits, distance codes <= 6 bits, complete codes, no A-11/A-12 header
// quirks, output <= 32 KiB, no reference before the segment start) ended by the empty stored
// block "00 00 FF FF" or by BFINAL.  Anything else is flagged SEGF_EXOTIC and redone by the
// exact wave decoder (k_inflate_segments mode 3), so results never depend on this path's
// coverage.  Decode semantics on the accepted layout are the reference's
// (decompressHuffmanBlock inflate.hpp:226-275, readDynamicTreeCodes :166-206, realDecompress
// :277-322), including "distance beyond the output so far copies nothing" at the stream start.
//
// Phase B, k_inflate_resolve: one workgroup per segment rebuilds the output in a 32 KiB LDS
// window from the token list; its first wavefront takes 64 tokens per step (wave prefix sum of
// token lengths): literal runs and short matches whose source lies before the step go in
// parallel (4 bytes per iteration when d >= 4), long or self-dependent matches are copied by the
// whole wave in token order (periodic copy out[o + i] = out[o - d + (i mod d)], as the
// reference's byte-serial copy inflate.hpp:268-270); then all waves put the window at j * slot
// with 16-byte stores (a long periodic copy at the segment's end goes straight to HBM).
#include "../../include/dmx.h"
#include "dmx_device.h"
#include "dmx_internal.h"
#include "inflate_common.h"

namespace dmx {

// LDS of one workgroup (one wavefront, LN_LANES segments): per segment a region of
//     [   0, 1024)  lit/len lookup table, 512 x u16, indexed by the next 9 stream bits
//                   (while the header is decoded: the code lengths, one byte per symbol, at
//                   [LN_LENS, 1024): lit/len 0..287, distance 288..319)
//     [1024, 1152)  distance lookup table, 64 x u16 (while the precode table of this segment
//                   is built: its symbols in canonical order)
// and a shared area of LN_LANES x 128 B: each segment's precode table (128 x u8) while the
// headers are decoded, then the canonical symbol order of the table being built.
constexpr uint32_t LN_REGION = 1152;
constexpr uint32_t LN_DIST = 1024;
constexpr uint32_t LN_LENS = 704;
constexpr uint32_t LN_PRE_BYTES = 128;
constexpr uint32_t LN_OUT_CAP = 32768;
// stream quads staged in LDS for a segment's code-length sequence: >= 15 bytes of offset + 553
// (316 symbols x 14 bits at most) + 8 bytes of read-ahead, below the code-length bytes
constexpr uint32_t LN_HDR_QUADS = 40;
// gfx950 LDS takes unaligned 2-, 4- and 8-byte accesses
typedef uint64_t u64_unaligned __attribute__((aligned(1)));
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
typedef uint16_t u16_unaligned __attribute__((aligned(1)));
static_assert(LN_HDR_QUADS * 16 <= LN_LENS, "header quads overlap the code lengths");
#ifndef DMX_LN_LANES
#define DMX_LN_LANES 32
#endif
// segments per 64-thread workgroup: 32 x 1280 B = 40 KiB of LDS, four workgroups per CU, one
// decoding wave per SIMD holding 32 segments.  The branch-free token step is VALU-issue-bound,
// so one wave of 32 segments beats two of 16 (1 GiB text inflate 12.3 -> 10.9 ms); the
// table builds take the other half of the wave's lanes.
constexpr uint32_t LN_LANES = DMX_LN_LANES;
// token step: a literal followed by a literal decodes both (the step's second table lookup is the
// distance code after a length, else the next lit/len symbol)
#ifndef DMX_LN_PAIR
#define DMX_LN_PAIR 1
#endif
// lane tables: the code-length words read ahead of their use (1) or at it (0)
#ifndef DMX_LN_PREF
#define DMX_LN_PREF 1
#endif
// precode tables: one per lane, all segments at once (1), or built by the whole wave one segment
// after the other (0, ln_coop_table)
#ifndef DMX_LN_PRETAB
#define DMX_LN_PRETAB 1
#endif
// resolve workgroup: RS_NT threads around one window.  Wave 0 runs the token steps, the
// workgroup fills periodic copies of >= RS_BIG bytes (repeat, zeros, image rows: segments of at
// most RS_FOLLOW token words) and copies the window out.  A 32 KiB window allows five workgroups
// per CU: with one wave each, those copies ran at 1.25 waves per SIMD, latency-bound.
#ifndef DMX_RS_NT
#define DMX_RS_NT 256
#endif
#ifndef DMX_RS_BIG
#define DMX_RS_BIG 2048
#endif
#ifndef DMX_RS_FOLLOW
#define DMX_RS_FOLLOW 1024
#endif
constexpr uint32_t RS_FOLLOW = DMX_RS_FOLLOW;
#ifndef DMX_RS_SPLIT
#define DMX_RS_SPLIT 1
#endif
// (NT = 64) the segment's last token, a periodic copy, written straight to HBM (1) or through
// the window (0; measured faster: repeat inflate 0.629 vs 0.655 ms, zeros 0.468 vs 0.495 ms)
#ifndef DMX_LN_DIRECT
#define DMX_LN_DIRECT 0
#endif
constexpr uint32_t RS_NT = DMX_RS_NT;
constexpr uint32_t RS_BIG = DMX_RS_BIG;
static_assert(RS_NT % 64 == 0 && RS_NT <= 1024, "resolve workgroup");
constexpr bool kRsSplit = DMX_RS_SPLIT && RS_NT > 64;
#ifndef DMX_RS_TICKET_WG
#define DMX_RS_TICKET_WG 5
#endif
constexpr uint32_t RS_TICKET_WG = DMX_RS_TICKET_WG;  // one-wave resolve workgroups per CU

__constant__ const uint8_t kLnPerm[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5,
                                          11, 4,  12, 3, 13, 2, 14, 1, 15};

struct LaneArgs {
    uint32_t* tok;          // token words
    const uint64_t* tokoff; // ncand + 1 word offsets (exclusive scan of the capacities)
    uint32_t* ntok;         // ncand token counts
    uint32_t* caps;         // ncand capacities (words)
    uint32_t* split;        // 64 KiB segments: ncand first-word indices of the second 32 KiB
                            // half (~0: not split; 0 for a stored segment).  32 KiB segments:
                            // [0] a count, [1] a ticket, then the candidates whose token lists
                            // the one-wave resolve takes (ncand + 2 words)
};

// lit/len table entry: literal / end-of-block  0 | cl(4) << 11 | sym(9)
//                      length               1 | cl(4) << 11 | extra(3) << 8 | base - 3 (8)
// symbols 286/287 (fixed code only) are entered as literals >= 257 -> flagged on use.
__device__ __forceinline__ uint32_t ln_lit_entry(uint32_t s, uint32_t l) {
    if (s >= 257 && s <= 285) return 0x8000u | (l << 11) | (len_extra(s) << 8) | (len_base(s) - 3);
    return (l << 11) | s;
}

// Canonical decode table of one code, built by the whole wavefront (RFC 1951 3.2.2; the
// reference builds a bit-trie, FlatHuffmanTree::construct common.hpp:104-145).  lens(s) gives
// the code length of symbol s < nsym (0 = unused); table[x] for every B-bit index x (the next B
// stream bits, LSB first) decodes the code that is a prefix of x.  Steps: per-length counts by
// ballots, canonical first codes, symbols in canonical order into `order`, then each lane fills
// entries x = lane + 64 k: the code length is the first l with (rev(x) >> (B - l)) below that
// length's limit (canonical codes are monotone, so the test is a count, no search), the symbol
// order[base[l] + code].  Returns false unless the code is complete with all lengths <= B.
template <int B, class Lens, class Order, class Put>
__device__ __forceinline__ bool ln_coop_table(uint32_t nsym, Lens lens, Order order, Put put) {
    const uint32_t lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t cnt[B + 1];
#pragma unroll
    for (int l = 0; l <= B; l++) cnt[l] = 0;
    bool bad = false;
    for (uint32_t c = 0; c < nsym; c += 64) {
        const uint32_t s = c + lane;
        const uint32_t L = s < nsym ? lens(s) : 0u;
        bad |= __ballot(L > (uint32_t)B) != 0;
#pragma unroll
        for (int l = 1; l <= B; l++) cnt[l] += (uint32_t)__popcll(__ballot(L == (uint32_t)l));
    }
    uint32_t kraft = 0;
#pragma unroll
    for (int l = 1; l <= B; l++) kraft += cnt[l] << (B - l);
    if (bad || kraft != (1u << B)) return false;
    uint32_t limit[B + 1], base[B + 1], run[B + 1];
    uint32_t first = 0, off = 0;
#pragma unroll
    for (int l = 1; l <= B; l++) {
        first = (first + cnt[l - 1]) << 1;  // cnt[0] = 0
        limit[l] = first + cnt[l];
        base[l] = off - first;  // order index = base + code (mod 2^32)
        run[l] = off;
        off += cnt[l];
    }
    for (uint32_t c = 0; c < nsym; c += 64) {
        const uint32_t s = c + lane;
        const uint32_t L = s < nsym ? lens(s) : 0u;
#pragma unroll
        for (int l = 1; l <= B; l++) {
            const uint64_t b = __ballot(L == (uint32_t)l);
            if (L == (uint32_t)l) order(run[l] + (uint32_t)__popcll(b & lt), s, 1);
            run[l] += (uint32_t)__popcll(b);
        }
    }
    wave_sync();
    static_assert(B >= 6, "one table entry per lane at least");
#pragma unroll
    for (uint32_t k = 0; k < (1u << B) / 64; k++) {
        const uint32_t x = lane + 64 * k;
        const uint32_t v = bitrev(x, B);
        uint32_t idx = 0, len = 0;
#pragma unroll
        for (int l = B; l >= 1; l--) {
            const uint32_t p = v >> (B - l);
            if (p < limit[l]) {
                idx = base[l] + p;
                len = (uint32_t)l;
            }
        }
        put(x, order(idx, 0, 0), len);
    }
    wave_sync();
    return true;
}

// Per-lane canonical tables (one lane per segment, all segments of the wave at once).  Nine 9-bit
// counters or next codes per lane in two registers: code lengths 1..6 in lo, 7..9 in hi.
struct Pk9 {
    uint64_t lo;
    uint32_t hi;
};
__device__ __forceinline__ uint32_t pk_get(const Pk9& p, uint32_t L) {  // L in 1..9
    return L <= 6 ? (uint32_t)(p.lo >> (9 * (L - 1))) & 511u : (p.hi >> (9 * (L - 7))) & 511u;
}
__device__ __forceinline__ void pk_add(Pk9& p, uint32_t L) {  // L in 0..9 (0: nothing)
    p.lo += (L - 1u) < 6u ? 1ull << (9 * (L - 1)) : 0ull;
    p.hi += L >= 7 ? 1u << (9 * (L - 7)) : 0u;
}
// The table T[0, 2^B) of a code with per-length counts `cnt` (lengths <= B), symbols s < nsym of
// lengths nib(s) (4-bit nibbles, packed 8 per word: word(k) holds symbols 8k .. 8k + 7); entries
// ent(s, L) whose length field is (e >> lsh) & lmask.  RFC 1951 3.2.2 canonical codes: the next
// code of each length, symbols in order.  Each symbol's entry goes to its bit-reversed code
// (a "seed", below 2^L); the table is then completed level by level: for b = 1 .. B-1 every entry
// in [0, 2^b) of length <= b is copied to + 2^b (a longer code's seed stays, and its own positions
// come from its seed).  Entries not yet written hold `mark` (a length above B).  Index rotation
// by lane keeps the lanes' accesses (regions 1152 B apart) off a common bank.  B >= 6.  Returns false
// unless the code is complete.
template <int B, int NL, class Word, class Ent>
__device__ __forceinline__ bool ln_lane_table(uint16_t* T, const Pk9& cnt, uint32_t nsym, Word word, Ent ent,
                                              uint32_t lsh, uint32_t lmask, uint32_t mark) {
    const uint32_t lane = lane_id();
    uint32_t kraft = 0, code = 0;
    Pk9 nc = {0ull, 0u};
#pragma unroll
    for (uint32_t l = 1; l <= (uint32_t)B; l++) {
        const uint32_t c = pk_get(cnt, l);
        kraft += c << (B - l);
        code = (code + (l > 1 ? pk_get(cnt, l - 1) : 0u)) << 1;  // first code of length l
        if (l <= 6) nc.lo |= (uint64_t)code << (9 * (l - 1));
        else nc.hi |= code << (9 * (l - 7));
    }
    if (kraft != (1u << B)) return false;
    constexpr uint32_t NW = (1u << B) / 2;  // table words
    uint64_t* const T64w = reinterpret_cast<uint64_t*>(T);
    const uint64_t m4 = (uint64_t)(mark | (mark << 16)) * 0x0000000100000001ull;
#pragma unroll 4
    for (uint32_t w = 0; w < NW / 2; w++) T64w[(w + lane) & (NW / 2 - 1)] = m4;
    // symbols below NL (a multiple of 8, < nsym): entry (L << lsh) | sym, no bound test
    // (DMX_LN_PREF: each word read one iteration ahead, its LDS latency behind the 8 symbols)
#if DMX_LN_PREF
    uint32_t xn = word(0);
#endif
    for (uint32_t k = 0; 8 * k < (uint32_t)NL; k++) {
#if DMX_LN_PREF
        const uint32_t x = xn;
        xn = word(k + 1);  // (k + 1 <= NL / 8: the next loop's first word)
#else
        const uint32_t x = word(k);
#endif
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t sym = 8 * k + i, L = (x >> (4 * i)) & 15u;
            if (L != 0u) {
                const uint32_t c = pk_get(nc, L);
                T[__builtin_bitreverse32(c) >> (32 - L)] = (uint16_t)((L << lsh) | sym);
            }
            pk_add(nc, L);
        }
    }
    for (uint32_t k = NL / 8; 8 * k < nsym; k++) {
#if DMX_LN_PREF
        const uint32_t x = k == NL / 8 && NL > 0 ? xn : word(k);
#else
        const uint32_t x = word(k);
#endif
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t sym = 8 * k + i, L = (x >> (4 * i)) & 15u;
            if (L != 0u && sym < nsym) {
                const uint32_t c = pk_get(nc, L);
                T[__builtin_bitreverse32(c) >> (32 - L)] = (uint16_t)ent(sym, L);
            }
            pk_add(nc, L);
        }
    }
    auto put = [&](uint32_t q, uint32_t e, uint32_t b) {
        if (((e >> lsh) & lmask) <= b) T[q] = (uint16_t)e;
    };
    // levels 1 and 2 entry by entry; from level 3 on (n >= 8) the reads of a batch go first (8
    // entries as two 8-byte reads, 4-entry aligned, rotated by 4 * lane), then the writes
    // (reads in [0, n), writes in [n, 2n): no overlap)
    put(2, T[0], 1);
    put(3, T[1], 1);
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) put(4 + i, T[i], 2);
    const uint64_t* const T64 = reinterpret_cast<const uint64_t*>(T);
#pragma unroll
    for (uint32_t b = 3; b < (uint32_t)B; b++) {
        const uint32_t n = 1u << b;
        for (uint32_t i = 0; i < n; i += 8) {
            const uint32_t q0 = (i + 4 * lane) & (n - 1), q1 = (q0 + 4) & (n - 1);
            const uint64_t v0 = T64[q0 >> 2], v1 = T64[q1 >> 2];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                put(q0 + n + k, (uint32_t)(v0 >> (16 * k)) & 0xFFFFu, b);
                put(q1 + n + k, (uint32_t)(v1 >> (16 * k)) & 0xFFFFu, b);
            }
        }
    }
    return true;
}

// The precode table of one segment per lane: T[0, 128) as u8 entries sym | len << 5 for the
// 19 precode lengths pl (3 bits each, by symbol), by the same canonical seeds and level doubling
// as ln_lane_table (per-length counts and next codes packed in registers; from level 3 on the
// doubling moves 8 entries per 8-byte word, the entries to copy picked by a per-byte compare of
// their length fields).  0xFF marks an entry not yet written.  False unless the code is complete.
__device__ __forceinline__ bool ln_lane_pretab(uint8_t* T, uint64_t pl) {
    const uint32_t lane = lane_id();
    uint64_t cnt = 0;  // per-length counts, 5 bits each, length L at 5 (L - 1)
#pragma unroll
    for (uint32_t s = 0; s < 19; s++) {
        const uint32_t L = (uint32_t)(pl >> (3 * s)) & 7u;
        cnt += L ? 1ull << (5 * (L - 1)) : 0ull;
    }
    uint32_t kraft = 0, code = 0, prev = 0;
    uint64_t nc = 0;  // next code per length, 7 bits each
#pragma unroll
    for (uint32_t l = 1; l <= 7; l++) {
        const uint32_t c = (uint32_t)(cnt >> (5 * (l - 1))) & 31u;
        kraft += c << (7 - l);
        code = (code + prev) << 1;
        nc |= (uint64_t)code << (7 * (l - 1));
        prev = c;
    }
    if (kraft != 128u) return false;
    uint64_t* const T64 = reinterpret_cast<uint64_t*>(T);
#pragma unroll
    for (uint32_t w = 0; w < 16; w++) T64[(w + lane) & 15] = ~0ull;
#pragma unroll
    for (uint32_t s = 0; s < 19; s++) {
        const uint32_t L = (uint32_t)(pl >> (3 * s)) & 7u;
        if (L) {
            const uint32_t c = (uint32_t)(nc >> (7 * (L - 1))) & 127u;
            T[__builtin_bitreverse32(c) >> (32 - L)] = (uint8_t)(s | (L << 5));
        }
        nc += L ? 1ull << (7 * (L - 1)) : 0ull;
    }
    auto put = [&](uint32_t q, uint32_t e, uint32_t b) {
        if ((e >> 5) <= b) T[q] = (uint8_t)e;
    };
    put(2, T[0], 1);
    put(3, T[1], 1);
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) put(4 + i, T[i], 2);
    constexpr uint64_t ONES = 0x0101010101010101ull;
#pragma unroll
    for (uint32_t b = 3; b < 7; b++) {
        const uint32_t nw = 1u << (b - 3);  // words of level b
#pragma unroll
        for (uint32_t i = 0; i < nw; i++) {
            const uint32_t q = (i + lane) & (nw - 1);
            const uint64_t src = T64[q], dst = T64[q + nw];
            const uint64_t lens = (src >> 5) & (7 * ONES);
            const uint64_t gt = ((lens + (7 - b) * ONES) >> 3) & ONES;  // length > b
            const uint64_t m = (gt ^ ONES) * 0xFFu;                      // bytes to copy
            T64[q + nw] = (src & m) | (dst & ~m);
        }
    }
    return true;
}

// CAP: the largest segment output (32 KiB; 64 KiB for config C4's blocks); NL: segments per
// wavefront (32).  With CAP > 32 KiB the lane also finds the split of its segment into two
// halves that k_inflate_resolve_half rebuilds in 32 KiB windows (see HALF below).  A lane
// decodes about one symbol per 1000 cycles whatever the segment size, so a 64 KiB segment
// takes twice a 32 KiB one's time and a stream has half as many of them: the lane pass of
// 64 KiB blocks is at best half as fast as that of 32 KiB segments.
template <uint32_t CAP, uint32_t NL>
__global__ __launch_bounds__(64) void k_inflate_lanes(InflateArgs A, LaneArgs B) {
    constexpr uint32_t LN_LANES = NL;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LN_LANES * (LN_REGION + LN_PRE_BYTES)];
    const uint32_t lane = threadIdx.x;
    const uint64_t j = (uint64_t)blockIdx.x * LN_LANES + lane;
    // lanes 0 .. LN_LANES-1 decode one segment each; the whole wave builds the tables
    const bool seg_lane = lane < LN_LANES && j < cand_count(A);
    uint8_t* const R = lds + min(lane, LN_LANES - 1) * LN_REGION;
    uint8_t* const SH = lds + LN_LANES * LN_REGION;  // shared area
    uint8_t* const PRE = SH + min(lane, LN_LANES - 1) * LN_PRE_BYTES;
    auto lut16 = [&](uint32_t b) -> uint32_t { return *reinterpret_cast<const uint16_t*>(R + b); };

    // code-length bytes of every segment start at zero (zero runs are then just skipped)
    for (uint32_t i = lane; i < LN_LANES * (1024 - LN_LENS) / 4; i += 64) {
        const uint32_t sgm = i / ((1024 - LN_LENS) / 4), w = i % ((1024 - LN_LENS) / 4);
        reinterpret_cast<uint32_t*>(lds + sgm * LN_REGION + LN_LENS)[w] = 0u;
    }
    wave_sync();

    const uintptr_t base4 = reinterpret_cast<uintptr_t>(A.in_words);
    const uintptr_t base16 = base4 & ~(uintptr_t)15;
    const uint64_t off0 = (uint64_t)(base4 - base16) + A.misalign;  // stream byte 0
    LaneIn br;
    const uint64_t start = seg_lane ? A.cands[j] : 0;
    uint64_t cb = (off0 + start) & ~(uint64_t)15;  // stream byte of relative position 0
    if (cb >= 16 && cb >= off0 + A.n) cb -= 16;  // a candidate at the stream end: keep a quad in bounds
    br.blk = (GUint4*)(base16 + cb);
    br.E = (uint32_t)min(off0 + A.n - cb, (uint64_t)1 << 26);
    br.nblk = (br.E + 15) / 16;
    uint64_t* const dbg = (A.dbg && seg_lane) ? A.dbg + j * kPhaseSlots : nullptr;  // DMX_PHASES aid
    uint32_t n_iter = 0, n_top = 0;
    if (dbg) dbg[0] = __builtin_amdgcn_s_memtime();
    uint32_t flags = seg_lane ? 0u : SEGF_EXOTIC;
    uint32_t outpos = 0;
    bool fin = false;
    uint64_t end_byte = 0;
    uint32_t* const tk = seg_lane ? B.tok + B.tokoff[j] : B.tok;
    const uint32_t tcap = seg_lane ? B.caps[j] : 0u;
    if (seg_lane) {
        br.seek((uint32_t)(off0 + start - cb));
        // consume the loads above now: a later first use would wait with vmcnt(0), draining
        // the stream prefetch in flight at that point
        if (tcap == 0 || (reinterpret_cast<uintptr_t>(tk) & 15)) flags |= SEGF_EXOTIC;
    }

    // token output: pending token (merges), 4-word queue, 16-byte stores
    uint32_t ntok = 0, qn = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    // CAP > 32 KiB: the word index where output byte HALF begins (no token straddles it and no
    // word merges across it), and whether a match past HALF reaches back before it; a segment
    // with a split and no such match resolves as two independent 32 KiB halves
    constexpr uint32_t HALF = 32768;
    constexpr bool SPLIT = CAP > HALF;
    uint32_t split = ~0u;
    bool xhalf = false;
    uint32_t pk = 0, pa = 0, pd = 0;  // pending: kind (1 literal run, 2 match), bytes / L, count / d
    auto push = [&](uint32_t w) {
        q0 = q1;  // shift register (no indexed writes: stays in VGPRs)
        q1 = q2;
        q2 = q3;
        q3 = w;
        if (++qn == 4) {
            if (ntok + 4 <= tcap) *reinterpret_cast<uint4*>(tk + ntok) = make_uint4(q0, q1, q2, q3);
            ntok += 4;
            qn = 0;
        }
    };
    auto flushp = [&]() {
        if (pk == 1) push((pd << 24) | pa);
        else if (pk == 2) push(0x80000000u | (pa << 15) | (pd - 1));
        pk = 0;
    };

    // ---- block header: BFINAL, BTYPE, stored segments, dynamic-header fields ---------------
    uint32_t bfinal = 0, btype = 0, hlit = 288, hdist = 32;
    uint64_t pl = 0;  // dynamic: 19 x 3-bit precode lengths, by symbol
    if (seg_lane && !flags) {
        br.ensure(3);
        bfinal = br.bits(1);
        btype = br.bits(2);
        if (btype == 0) {
            // stored block (libdmx emits these for incompressible segments) or an empty segment
            br.align();
            br.ensure(32);
            const uint32_t len = br.bits(16), nlen = br.bits(16);
            const uint32_t b0 = br.bitpos() >> 3;  // byte of the data (relative)
            if (!bfinal && len == 0 && nlen == 0xFFFF) {
                end_byte = b0 + cb - off0;  // empty segment: the candidate is itself a marker
            } else if (b0 + len > br.E || len > CAP) {
                flags |= SEGF_EXOTIC;
            } else {
                split = 0;  // (a stored segment is copied whole by the half resolve's first item)
                push(len);
                push((uint32_t)(b0 + cb - off0 - start));
                outpos = len;
                br.seek(b0 + len);
                if (bfinal) {
                    fin = true;
                    end_byte = b0 + len + cb - off0;
                } else {
                    br.ensure(3);
                    const uint32_t f2 = br.bits(1), t2 = br.bits(2);
                    br.align();
                    br.ensure(32);
                    const uint32_t l2 = br.bits(16), n2 = br.bits(16);
                    if (t2 == 0 && l2 != 0 && n2 == (~l2 & 0xFFFFu)) {
                        // a second stored block: the stored form of a 64 KiB segment (LEN is 16
                        // bits, so libdmx writes two blocks of 32 KiB), then BFINAL or the marker
                        const uint32_t c2 = br.bitpos() >> 3;
                        if (c2 + l2 > br.E || outpos + l2 > CAP) {
                            flags |= SEGF_EXOTIC;
                        } else {
                            push(l2);
                            push((uint32_t)(c2 + cb - off0 - start));
                            outpos += l2;
                            br.seek(c2 + l2);
                            if (f2) {
                                fin = true;
                                end_byte = c2 + l2 + cb - off0;
                            } else {
                                br.ensure(3);
                                const uint32_t f3 = br.bits(1), t3 = br.bits(2);
                                br.align();
                                br.ensure(32);
                                const uint32_t l3 = br.bits(16), n3 = br.bits(16);
                                if (f3 || t3 != 0 || l3 != 0 || n3 != 0xFFFF) flags |= SEGF_EXOTIC;
                                end_byte = (br.bitpos() >> 3) + cb - off0;
                            }
                        }
                    } else {
                        if (f2 || t2 != 0 || l2 != 0 || n2 != 0xFFFF) flags |= SEGF_EXOTIC;
                        end_byte = (br.bitpos() >> 3) + cb - off0;
                    }
                }
            }
        } else if (btype == 3) {
            flags |= SEGF_EXOTIC;  // reference: empty block, then more blocks -- not this layout
        } else if (btype == 2) {
            br.ensure(14);
            hlit = br.bits(5) + 257;
            hdist = br.bits(5) + 1;
            const uint32_t hclen = br.bits(4) + 4;
            for (uint32_t i = 0; i < hclen; i++) {
                br.ensure(3);
                pl |= (uint64_t)br.bits(3) << (3 * kLnPerm[i]);
            }
            if (hlit > 286 || hdist > 30) flags |= SEGF_EXOTIC;
        }
    }
    const bool huff = seg_lane && !flags && (btype == 1 || btype == 2);
    const uint32_t dyn_mask = (uint32_t)__ballot(huff && btype == 2);
    // ---- precode tables of the dynamic segments, built by the wave (7-bit, u8 entries) -------
    uint32_t bad_mask = 0;
#if DMX_LN_PRETAB
    // one table per lane, all segments at once
    if (huff && btype == 2 && !ln_lane_pretab(PRE, pl)) flags |= SEGF_EXOTIC;
    wave_sync();
#else
    for (uint32_t m = dyn_mask; m; m &= m - 1) {
        const uint32_t s = (uint32_t)__builtin_ctz(m);
        const uint64_t pls = ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(pl >> 32), s) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pl, s);
        uint8_t* const ord = lds + s * LN_REGION + LN_DIST;  // canonical order scratch
        uint8_t* const tab = SH + s * LN_PRE_BYTES;
        const bool ok = ln_coop_table<7>(
            19u, [&](uint32_t sym) { return (uint32_t)(pls >> (3 * sym)) & 7u; },
            [&](uint32_t i, uint32_t sym, int wr) -> uint32_t {
                if (wr) { ord[i] = (uint8_t)sym; return 0u; }
                return ord[i];
            },
            [&](uint32_t x, uint32_t sym, uint32_t len) { tab[x] = (uint8_t)(sym | (len << 5)); });
        if (!ok) bad_mask |= 1u << s;
    }
#endif
    if (seg_lane && ((bad_mask >> lane) & 1u)) flags |= SEGF_EXOTIC;
    if (dbg) dbg[1] = __builtin_amdgcn_s_memtime();

    // ---- code lengths of the dynamic segments, decoded once into bytes (lane-serial) ------------
    // The sequences come from LDS: the next LN_HDR_QUADS stream quads of every segment go into
    // its lit/len table area (built only after this), loaded by the whole wave at once -- one
    // memory latency for all 32 segments, where the register ring's top-ups stalled the wave
    // once per lane running low (a 300-byte header of a high-ratio segment: 4x the decode time).
    const uint32_t hq0 = br.wi >> 2;  // stream quad of the area's first byte
    if (dyn_mask) {
        const uint64_t b64 = reinterpret_cast<uint64_t>(br.blk);
        const uint32_t blo = (uint32_t)b64, bhi = (uint32_t)(b64 >> 32);
        const uint32_t k = min(lane, LN_HDR_QUADS - 1);  // lanes >= LN_HDR_QUADS: not stored
        u32x4 t[LN_LANES];
#pragma unroll
        for (uint32_t s = 0; s < LN_LANES; s++) {  // unconditional: every lane's blk is valid
            const uint64_t b = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)bhi, s) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)blo, s);
            const uint32_t q = min((uint32_t)__builtin_amdgcn_readlane((int)hq0, s) + k,
                                   (uint32_t)__builtin_amdgcn_readlane((int)br.nblk, s) - 1u);
            t[s] = reinterpret_cast<GUint4*>(b)[q];
        }
        if (lane < LN_HDR_QUADS) {
#pragma unroll
            for (uint32_t s = 0; s < LN_LANES; s++)
                *reinterpret_cast<u32x4*>(lds + s * LN_REGION + 16 * lane) = t[s];
        }
        wave_sync();
    }
    if (seg_lane && !flags && btype == 2) {
        uint8_t* const LL = R + LN_LENS;  // lit/len lengths [0, 288), distance [288, 320)
        const uint32_t* const H = reinterpret_cast<const uint32_t*>(R);  // stream words from 4 hq0
        const uint32_t hw0 = 4 * hq0;
        uint32_t i = 0, prev = 0;
        bool prevok = false;
        const uint32_t total = hlit + hdist;
        uint32_t nxt = H[br.wi - hw0];  // the word at br.wi, read one step ahead
        // one precode symbol per step, outcome by selects (short-circuit && would branch)
        while (!flags && i < total) {
            {   // >= 14 bits buffered: a precode code (<= 7 bits) and its repeat bits (<= 7).
                // Bytes past the stream end are not masked: a header that reads them ends past
                // it, and the segment is then flagged (endbit > 8 E below) and decoded exactly.
                const bool need = br.nb < 14;
                br.bb |= need ? (uint64_t)nxt << br.nb : 0ull;
                br.nb += need ? 32u : 0u;
                br.wi += need ? 1u : 0u;
                nxt = H[min(br.wi - hw0, 4 * LN_HDR_QUADS - 1)];
            }
            const uint32_t e = PRE[(uint32_t)(br.bb & 127)];
            const uint32_t len = e >> 5, sym = e & 31;
            const bool lit = sym < 16;
            // repeat codes 16 / 17 / 18: extra bits 2 / 3 / 7, base count 3 / 3 / 11 (nibbles)
            const uint32_t rk = 4 * (sym - 16);
            const uint32_t ex = lit ? 0u : (0x732u >> rk) & 15u;
            const uint32_t xv = (uint32_t)(br.bb >> len) & ((1u << ex) - 1u);
            br.consume(len + ex);
            const uint32_t run = lit ? 1u : ((0xB33u >> rk) & 15u) + xv;
            const uint32_t val = lit ? sym : (sym == 16 ? prev : 0u);
            const bool inl = i < hlit;
            const bool bad = ((sym == 16) & (!prevok | (i == hlit))) |  // A-12 / sequence-start repeat
                             (inl & (i + run > hlit)) | (i + run > total) |  // A-11
                             (val > (inl ? 9u : 6u));                      // beyond the lane tables
            prevok = lit | ((sym == 16) & prevok);
            prev = lit ? sym : prev;
            const uint32_t at = inl ? i : 288 + (i - hlit);
            const uint32_t nw = ((val != 0u) & !bad) ? run : 0u;  // <= 6 bytes (a 16 repeats <= 6)
            if (nw) {  // one unaligned 8-byte store: val x nw, then zeros over positions not yet
                       // decoded (zero runs are skipped, the lengths start zeroed); at + 7 stays
                       // inside the region (distance lengths end at 320 + 7 < 1152 - LN_LENS)
                const uint64_t rep = (uint64_t)val * 0x0101010101010101ull;
                *reinterpret_cast<u64_unaligned*>(LL + at) = rep & ((1ull << (8 * nw)) - 1ull);
            }
            i += run;
            flags |= bad ? (uint32_t)SEGF_EXOTIC : 0u;
        }
    }
    if (dbg) dbg[2] = __builtin_amdgcn_s_memtime();

    // ---- lit/len (9-bit) and distance (6-bit) tables, one lane per segment (ln_lane_table) -----
    // The code lengths are first packed to nibbles (symbols 0..255 into the lane's 128 B of the
    // shared area, 256..287 and the distance lengths into its distance-table area), because the
    // lit/len table overwrites their bytes [LN_LENS, 1024); the distance table is built last.
    if (huff && !flags) {
        const bool fixed = btype == 1;
        uint32_t* const PK = reinterpret_cast<uint32_t*>(SH + lane * LN_PRE_BYTES);  // words 0..31
        uint32_t* const PD = reinterpret_cast<uint32_t*>(R + LN_DIST);             // words 32..39
        const uint32_t* const LW = reinterpret_cast<const uint32_t*>(R + LN_LENS);
        Pk9 cl = {0ull, 0u}, cd = {0ull, 0u};
#if DMX_LN_PREF
#pragma unroll 8
#endif
        for (uint32_t k = 0; k < 40; k++) {
            // fixed code (RFC 1951 3.2.6): 8 (0..143), 9 (144..255), 7 (256..279), 8 (280..287), 5
            const uint32_t fw = k < 18 ? 0x88888888u : k < 32 ? 0x99999999u : k < 35 ? 0x77777777u
                              : k < 36 ? 0x88888888u : 0x55555555u;
            const uint32_t lo = LW[2 * k], hi = LW[2 * k + 1];  // 8 length bytes (each <= 9)
            auto nib4 = [](uint32_t x) {
                return (x & 0xFu) | ((x >> 4) & 0xF0u) | ((x >> 8) & 0xF00u) | ((x >> 12) & 0xF000u);
            };
            const uint32_t x = fixed ? fw : nib4(lo) | (nib4(hi) << 16);
            if (k < 32) PK[(k + lane) & 31] = x;  // rotated by lane (bank spread), read back alike
            else PD[k - 32] = x;
#pragma unroll
            for (uint32_t i = 0; i < 8; i++) {
                if (k < 36) pk_add(cl, (x >> (4 * i)) & 15u);
                else pk_add(cd, (x >> (4 * i)) & 15u);
            }
        }
        const uint32_t dw0 = PD[4], dw1 = PD[5], dw2 = PD[6], dw3 = PD[7];
        uint16_t* const lt = reinterpret_cast<uint16_t*>(R);
        uint16_t* const dt = reinterpret_cast<uint16_t*>(R + LN_DIST);
        bool ok = ln_lane_table<9, 256>(
            lt, cl, 288u, [&](uint32_t k) { return k < 32 ? PK[(k + lane) & 31] : PD[k - 32]; },
            [](uint32_t sym, uint32_t len) { return ln_lit_entry(sym, len); }, 11, 15, 0x7800u);
        ok = ok && ln_lane_table<6, 0>(
            dt, cd, 32u, [&](uint32_t k) { return k == 0 ? dw0 : k == 1 ? dw1 : k == 2 ? dw2 : dw3; },
            [](uint32_t sym, uint32_t len) { return 0x8000u | (len << 8) | sym; }, 8, 7, 0x8700u);
        if (!ok) flags |= SEGF_EXOTIC;
    }
    wave_sync();
    if (dbg) dbg[3] = __builtin_amdgcn_s_memtime();

    uint32_t endbit = seg_lane ? br.bitpos() : 0u;
    if (huff && !flags) {
        // ---- tokens until end-of-block -------------------------------------------------------
        // The stream comes through a ring of 8 quads (128 B) per lane in the shared LDS area:
        // each step reads the 64 bits at the bit position (two ds_read_b64 + funnel shifts), so
        // every symbol -- a literal, or a length and distance with their extra bits (<= 33
        // bits) -- decodes from one window with no refill branch.  Every LN_PERIOD steps the
        // lane loads the next quad of its stream into a staging register and writes the quad
        // staged two periods earlier into the ring (loads complete off the critical path); a
        // quad goes into the ring only once the one it replaces is consumed.  LN_PERIOD steps
        // consume <= 99 bits < one quad, so the ring stays >= 5 quads ahead.  The token logic
        // is written with selects so the lanes of a wave, each on its own segment, execute
        // one short path per step.
        constexpr uint32_t LN_PERIOD = 3;
        u32x4* const ring = reinterpret_cast<u32x4*>(SH + lane * LN_PRE_BYTES);
        const uint64_t* const ring2 = reinterpret_cast<const uint64_t*>(ring);
        uint32_t bp = br.bitpos();
        {
            const uint32_t q0 = bp >> 7;
            u32x4 t[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) t[k] = br.blk[min(q0 + k, br.nblk - 1)];
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) ring[(q0 + k) & 7] = t[k];
        }
        uint32_t nextq = (bp >> 7) + 8, tq0 = 0, tq1 = 0;
        u32x4 S0 = {0, 0, 0, 0}, S1 = {0, 0, 0, 0};
        bool v0 = false, v1 = false;
        // one symbol; returns false once the lane's block has ended (EOB or a flag)
        const uint32_t E8 = 8 * br.E;
        const uint32_t xref_fl = (j != 0 || (A.flags & DMX_IFLAG_PIECE)) ? (uint32_t)SEGF_XREF : 0u;
        // The 64-bit window at bp lives in registers; each step reads the next 64 bits (from
        // two word pairs addressed by the old bp, so the LDS latency overlaps the table lookups)
        // and funnels them in after consuming the symbol.
        auto window_at = [&](uint32_t pos, uint64_t q0, uint64_t q1) -> uint64_t {  // q0, q1: pairs
            const bool odd = (pos >> 5) & 1;                                       // holding pos
            const uint32_t w0 = odd ? (uint32_t)(q0 >> 32) : (uint32_t)q0;
            const uint32_t w1 = odd ? (uint32_t)q1 : (uint32_t)(q0 >> 32);
            const uint32_t w2 = odd ? (uint32_t)(q1 >> 32) : (uint32_t)q1;
            const uint32_t sh = pos & 31;
            return ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh) << 32) | __builtin_amdgcn_alignbit(w1, w0, sh);
        };
        uint64_t win;
        {
            const uint32_t pr = bp >> 6;
            win = window_at(bp, ring2[pr & 15], ring2[(pr + 1) & 15]);
        }
        auto step = [&]() -> bool {
#ifdef DMX_LN_COUNT
            n_iter++;  // diagnostic build: steps per lane (DMX_PHASES slot 8)
#endif
            const uint32_t pr = bp >> 6;
            const uint64_t nq0 = ring2[(pr + 1) & 15], nq1 = ring2[(pr + 2) & 15];
            // lit/len symbol, then the distance decoded from the same window (used for lengths)
            const uint32_t e = lut16(2 * ((uint32_t)win & 511u));
            const uint32_t cl = (e >> 11) & 15;
            const bool isl = (e & 0x8000u) != 0;
            const uint32_t ex = isl ? (e >> 8) & 7 : 0u;
            const uint32_t L = (e & 255) + 3 + ((uint32_t)(win >> cl) & ((1u << ex) - 1u));
            const uint32_t n1 = cl + ex;
            const uint64_t dwin = win >> n1;
#if DMX_LN_PAIR
            // the second lookup from the same window: the distance code after a length, else the
            // next lit/len symbol -- a literal after a literal is consumed in the same step
            // (literal pairs at the cost of one step)
            const uint32_t de = lut16(isl ? LN_DIST + 2 * ((uint32_t)dwin & 63u) : 2 * ((uint32_t)dwin & 511u));
#else
            const uint32_t de = lut16(LN_DIST + 2 * ((uint32_t)dwin & 63u));
#endif
            const uint32_t dcl = (de >> 8) & 7, ds = de & 31;
            const uint32_t dx = dist_extra(ds);
            const uint32_t d = dist_base(ds) + ((uint32_t)(dwin >> dcl) & ((1u << dx) - 1u));
            const uint32_t sym = e & 511;
#if DMX_LN_PAIR
            const uint32_t sym2 = de & 511, cl2 = (de >> 11) & 15;
            const bool lit2 = !isl & (sym < 256) & ((de & 0x8000u) == 0u) & (sym2 < 256) &
                              (outpos + 2 <= CAP) & (!SPLIT | (outpos + 1 != HALF));
            const uint32_t c = n1 + (isl ? dcl + dx : (lit2 ? cl2 : 0u));  // 1 .. 33 bits
#else
            const uint32_t c = n1 + (isl ? dcl + dx : 0u);  // 1 .. 33 bits
#endif
            const uint64_t ext = window_at(bp + 64, nq0, nq1);
            win = (win >> c) | ((ext << 1) << (63 - c));
            bp += c;
            // outcome by selects: literal, match (or the stream-start copy of nothing), end of
            // block, or a flag (distance symbol 30/31 = the reference's distance 0; length
            // symbols 286/287 = its length 0; a segment past 32 KiB; a reference before the
            // segment start, or at the stream start an over-read -- the one step that produces
            // nothing, so the loop stays bounded)
            // (bitwise & / | on the conditions: short-circuit && would become branches)
            const bool lit = !isl & (sym < 256);
            const bool far = d > outpos;
            const uint32_t EXO = SEGF_EXOTIC;
            const uint32_t f_far = xref_fl | (((xref_fl == 0u) & (bp > E8)) ? EXO : 0u);
            const uint32_t f_m = (ds >= 30) ? EXO : (far ? f_far : ((outpos + L > CAP) ? EXO : 0u));
            const uint32_t f_o = lit ? ((outpos >= CAP) ? EXO : 0u) : ((sym != 256) ? EXO : 0u);
            const uint32_t fl = isl ? f_m : f_o;
            const bool ok = fl == 0u;
            const bool mt = isl & !far & ok;
            const bool lt = lit & ok;
            const bool prod = lt | mt;
#if DMX_LN_PAIR
            // nl literal bytes lb (1 or 2); a pending run of 2 takes the first of a pair and a
            // new run starts with the second (lsplit)
            const bool lt2 = lt & lit2;
            const uint32_t nl = lt2 ? 2u : 1u;
            const uint32_t lb = lt2 ? sym | (sym2 << 8) : sym;
            const bool at_half = SPLIT & (outpos == HALF);  // no word merges across HALF
            const bool lcont = lt & (pk == 1u) & (pd + nl <= 3u) & !at_half;
            const bool lsplit = lt2 & (pk == 1u) & (pd == 2u) & !at_half;
            const bool mcont = mt & (pk == 2u) & (pd == d) & (pa + L <= 0xFFFFu) & !at_half;
            if (SPLIT) {
                split = (at_half & prod & (split == ~0u)) ? ntok + qn + (pk != 0u ? 1u : 0u) : split;
                xhalf |= mt & (outpos >= HALF) & (d > outpos - HALF);
            }
            const bool cont = lcont | mcont;
            const bool emit = prod & !cont & (pk != 0u);
            const uint32_t ew = lsplit ? (3u << 24) | pa | (sym << 16)
                              : pk == 1u ? (pd << 24) | pa : 0x80000000u | (pa << 15) | (pd - 1u);
            const uint32_t a_cont = lcont ? (pa | (lb << (8 * pd))) : (pa + L);
            const uint32_t a_new = lsplit ? sym2 : lt ? lb : L;
            const uint32_t d_cont = lcont ? pd + nl : pd;
            const uint32_t d_new = lsplit ? 1u : lt ? nl : d;
            const uint32_t npa = cont ? a_cont : a_new;
            const uint32_t npd = cont ? d_cont : d_new;
            pa = prod ? npa : pa;
            pd = prod ? npd : pd;
            pk = prod ? (lt ? 1u : 2u) : pk;
            outpos += prod ? (lt ? nl : L) : 0u;
#else
            const bool lcont = lt & (pk == 1u) & (pd < 3u);
            const bool mcont = mt & (pk == 2u) & (pd == d) & (pa + L <= 0xFFFFu);
            const bool cont = lcont | mcont;
            const bool emit = prod & !cont & (pk != 0u);
            const uint32_t ew = pk == 1u ? (pd << 24) | pa : 0x80000000u | (pa << 15) | (pd - 1u);
            const uint32_t a_cont = lcont ? (pa | (sym << (8 * pd))) : (pa + L);
            const uint32_t a_new = lt ? sym : L;
            const uint32_t d_cont = lcont ? pd + 1u : pd;
            const uint32_t d_new = lt ? 1u : d;
            const uint32_t npa = cont ? a_cont : a_new;
            const uint32_t npd = cont ? d_cont : d_new;
            pa = prod ? npa : pa;
            pd = prod ? npd : pd;
            pk = prod ? (lt ? 1u : 2u) : pk;
            outpos += prod ? (lt ? 1u : L) : 0u;
#endif
            // queue of 4 token words (shift register), one 16-byte store per 4 words
            q0 = emit ? q1 : q0;
            q1 = emit ? q2 : q1;
            q2 = emit ? q3 : q2;
            q3 = emit ? ew : q3;
            qn += emit ? 1u : 0u;
            if (qn == 4) {
                if (ntok + 4 <= tcap) *reinterpret_cast<uint4*>(tk + ntok) = make_uint4(q0, q1, q2, q3);
                ntok += 4;
                qn = 0;
            }
            flags |= fl;
            return ok & (isl | lit);
        };
        // two periods per trip, each with its own staging register (a select between them
        // would make every load's latency part of the step that follows it)
        auto stage = [&](u32x4& S, bool& v, uint32_t& tq) {
            if (v) ring[tq & 7] = S;  // staged two periods ago
            const bool adv = nextq < (bp >> 7) + 8;  // its slot's quad is consumed
            S = br.blk[min(nextq, br.nblk - 1)];
            v = adv;
            tq = nextq;
            nextq += adv ? 1u : 0u;
        };
        static_assert(LN_PERIOD == 3, "steps per period below");
        for (;;) {
#ifdef DMX_LN_COUNT
            const uint64_t ts0 = __builtin_amdgcn_s_memtime();
            stage(S0, v0, tq0);
            n_top += (uint32_t)(__builtin_amdgcn_s_memtime() - ts0);  // cycles in stage (slot 9)
#else
            stage(S0, v0, tq0);
#endif
            if (!step() || !step() || !step()) break;
#ifdef DMX_LN_COUNT
            const uint64_t ts1 = __builtin_amdgcn_s_memtime();
            stage(S1, v1, tq1);
            n_top += (uint32_t)(__builtin_amdgcn_s_memtime() - ts1);
#else
            stage(S1, v1, tq1);
#endif
            if (!step() || !step() || !step()) break;
        }
        endbit = bp;
        if (dbg) dbg[4] = __builtin_amdgcn_s_memtime();
        // ---- what follows the block: BFINAL, or the empty stored block of a segment end ------
        if (!flags) {
            if (bfinal) {
                fin = true;
                end_byte = ((bp + 7) >> 3) + cb - off0;
            } else {  // 000, pad to the byte, LEN = 0000, NLEN = FFFF: from a window at bp
                const uint32_t wi = bp >> 5, pr = wi >> 1;
                const uint64_t pa0 = ring2[pr & 15], pa1 = ring2[(pr + 1) & 15];
                const bool odd = wi & 1;
                const uint32_t w0 = odd ? (uint32_t)(pa0 >> 32) : (uint32_t)pa0;
                const uint32_t w1 = odd ? (uint32_t)pa1 : (uint32_t)(pa0 >> 32);
                const uint32_t w2 = odd ? (uint32_t)(pa1 >> 32) : (uint32_t)pa1;
                const uint32_t sh = bp & 31;
                const uint64_t win = ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh) << 32) |
                                     __builtin_amdgcn_alignbit(w1, w0, sh);
                const uint32_t pad = (8u - ((bp + 3) & 7u)) & 7u;
                const uint32_t hdr = (uint32_t)win & 7u, ln = (uint32_t)(win >> (3 + pad));
                if (hdr != 0 || ln != 0xFFFF0000u) flags |= SEGF_EXOTIC;
                endbit = bp + 3 + pad + 32;
                end_byte = (endbit >> 3) + cb - off0;
            }
        }
    }
    if (!seg_lane) return;
    if (endbit > 8 * br.E) flags |= SEGF_EXOTIC;
    flushp();
    if (qn) {  // the queue's last partial group: the newest qn words, q[4 - qn .. 3]
        if (ntok + qn <= tcap) {
            if (qn == 3) {
                tk[ntok] = q1;
                tk[ntok + 1] = q2;
                tk[ntok + 2] = q3;
            } else if (qn == 2) {
                tk[ntok] = q2;
                tk[ntok + 1] = q3;
            } else {
                tk[ntok] = q3;
            }
        }
        ntok += qn;
    }
    if (ntok > tcap) flags |= SEGF_EXOTIC;
    SegRecord r;
    r.end_byte = end_byte;
    r.offset = j * (uint64_t)A.slot;
    r.out_size = flags ? 0u : outpos;
    r.flags = flags | (fin ? SEGF_FINAL : 0u);
    A.recs[j] = r;
    B.ntok[j] = ntok;
    // 32 KiB segments: a long token list goes on the one-wave resolve's list (the rest: the
    // workgroup resolve, launched over every candidate)
    if (!SPLIT && kRsSplit && !(r.flags & ~SEGF_FINAL) && ntok > RS_FOLLOW) B.split[2 + atomicAdd(B.split, 1u)] = (uint32_t)j;
    // the split holds only if the output crossed HALF at a token boundary, or never reached it
    if (SPLIT) B.split[j] = (flags || xhalf || (outpos > HALF && split == ~0u)) ? ~0u : (outpos <= HALF ? ntok : split);
    if (dbg) {  // (slots 5..7 belong to k_inflate_resolve)
        dbg[8] = n_iter;
        dbg[9] = n_top;
        dbg[10] = ntok;
        dbg[11] = outpos;
    }
}

// token-list capacity per candidate: min(one word per compressed bit, cap / 2 + 2) + 16,
// rounded to whole 16-byte groups.  A segment of at most 32 KiB needs at most 16 Ki + 1 words:
// a literal-run word holds up to 3 bytes and two consecutive ones hold >= 4 (a short run is
// followed by a match), a match word >= 3 bytes, so words <= bytes / 2 + 1.
// A dense candidate spans more than `heavy` compressed bytes and does not start with a stored
// block (BTYPE 00: the lanes pass a stored segment on as one token, the resolve copies it).
__device__ __forceinline__ bool ln_dense(const uint8_t* in, uint64_t start, uint64_t n, uint64_t span,
                                        uint32_t heavy) {
    return span > heavy && start < n && ((in[start] >> 1) & 3u) != 0u;
}

// With heavy != 0 and at most `limit` heavy candidates in the stream (hl[1], counted by
// k_heavy_count), a dense candidate (ln_dense) gets capacity 0 (the
// lane declines it: SEGF_EXOTIC) and is appended to the list hl[2..] (hl[0] = its length)
// for the workgroup decoder (mode 6): a lane decodes ~1 symbol per 1000 cycles, so one dense
// segment sets the time of a wave.
// (rsl: the one-wave resolve's count and ticket, zeroed here for the lanes that follow)
__global__ void k_lane_caps(const uint8_t* in, const uint64_t* cands, uint64_t ncand, uint64_t n, uint32_t* caps,
                            uint32_t heavy, uint32_t limit, uint32_t* hl, uint32_t ocap, const uint64_t* ncand_dev,
                            uint32_t* rsl) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rsl && j < 2) rsl[j] = 0;
    if (j >= ncand) return;
    if (ncand_dev && j >= *ncand_dev) {  // (async: past the device-side count)
        caps[j] = 0;
        return;
    }
    if (ncand_dev && *ncand_dev < ncand) ncand = *ncand_dev;
    const uint64_t nxt = j + 1 < ncand ? cands[j + 1] : n;
    const uint64_t span = nxt - cands[j];
    if (heavy && ln_dense(in, cands[j], n, span, heavy) && hl[1] <= limit) {
        caps[j] = 0;
        hl[2 + atomicAdd(hl, 1u)] = (uint32_t)j;
        return;
    }
    const uint64_t bits = 8 * span;
    const uint64_t c = min(bits, (uint64_t)ocap / 2 + 2) + 16;
    caps[j] = (uint32_t)((c + 3) & ~3ull);
}

// Wave-cooperative copies inside the 32 KiB window.  The body of a copy goes as 16-byte aligned
// stores, each lane building its quad from five source words with alignbyte.
// the 16 bytes at window byte s (the fifth word is needed only when s is not word-aligned, and
// is clamped into the window for the aligned case)
template <uint32_t CAP>
__device__ __forceinline__ uint4 ln_quad_at(const uint8_t* win, uint32_t s) {
    constexpr uint32_t LN_WIN_WORDS = CAP / 4;
    const uint32_t* const W = reinterpret_cast<const uint32_t*>(win);
    const uint32_t i = s >> 2, sh = s & 3;
    const uint32_t w0 = W[i], w1 = W[i + 1], w2 = W[i + 2], w3 = W[i + 3];
    const uint32_t w4 = W[min(i + 4, LN_WIN_WORDS - 1)];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// ln_copy_plain moves n bytes from s to o with s + n <= o (source wholly before the destination,
// so every lane copies independently): unaligned head and tail bytes one per lane, the body as
// aligned quads (one quad per lane and wave-step: these copies are mostly short).
template <uint32_t CAP>
__device__ __forceinline__ void ln_copy_plain(uint8_t* win, uint32_t o, uint32_t s, uint32_t n) {
    constexpr uint32_t LN_WIN_WORDS = CAP / 4;
    const uint32_t lane = lane_id();
    const uint32_t* const W = reinterpret_cast<const uint32_t*>(win);
    const uint32_t end = o + n;
    const uint32_t a0 = min((o + 15) & ~15u, end);  // first 16-byte aligned body byte
    const uint32_t a1 = max(a0, end & ~15u);        // first tail byte
    if (lane < a0 - o) win[o + lane] = win[s + lane];
    else if (lane >= 16 && lane - 16 < end - a1) win[a1 + lane - 16] = win[s + (a1 - o) + lane - 16];
    const uint32_t nq = (a1 - a0) >> 4;
    const uint32_t sb = s + (a0 - o), sh = sb & 3;
    for (uint32_t k = lane; k < nq; k += 64) {
        const uint32_t i = (sb >> 2) + 4 * k;
        // the fifth word is needed only when sh != 0, and then i + 4 < LN_WIN_WORDS (the source
        // ends before the destination): the clamp only keeps the sh == 0 read in the window
        const uint32_t w0 = W[i], w1 = W[i + 1], w2 = W[i + 2], w3 = W[i + 3];
        const uint32_t w4 = W[min(i + 4, LN_WIN_WORDS - 1)];
        *reinterpret_cast<uint4*>(win + a0 + 16 * k) =
            make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                       __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
    }
}

// ln_fill_mod: out[o + i] = out[o + (i mod Q)] for i in [P, L), where Q is a multiple of the match
// distance (so this continues the periodic copy) and the prefix [o, o + Q + 16) is final
// (P >= Q + 16): every source quad lies in that prefix, so the rest of the match is one pass of
// independent quad copies.  Lane phases advance by 1024 mod Q per wave-step (one division per
// lane, at the start).
template <uint32_t CAP>
__device__ __forceinline__ uint32_t ln_fill_mod(uint8_t* win, uint32_t o, uint32_t P, uint32_t L, uint32_t Q,
                                                uint8_t* out) {
    const uint32_t lane = lane_id();
    const uint32_t beg = o + P, end = o + L;
    const uint32_t a0 = min((beg + 15) & ~15u, end);
    const uint32_t a1 = max(a0, end & ~15u);
    if (lane < a0 - beg) win[beg + lane] = win[o + (P + lane) % Q];
    else if (lane >= 16 && lane - 16 < end - a1) out[a1 + lane - 16] = win[o + (a1 - o + lane - 16) % Q];
    const uint32_t nq = (a1 - a0) >> 4;
    if (nq <= lane) return a0;
    const uint32_t R = 1024u % Q;
    auto adv = [&](uint32_t r) { r += R; return r >= Q ? r - Q : r; };
    uint32_t r = (a0 - o + 16 * lane) % Q;  // phase of quad k = lane
    uint4* const D = reinterpret_cast<uint4*>(out + a0);
    uint32_t k = lane;
    for (; k + 192 < nq; k += 256) {
        const uint32_t r1 = adv(r), r2 = adv(r1), r3 = adv(r2);
        const uint4 v0 = ln_quad_at<CAP>(win, o + r), v1 = ln_quad_at<CAP>(win, o + r1);
        const uint4 v2 = ln_quad_at<CAP>(win, o + r2), v3 = ln_quad_at<CAP>(win, o + r3);
        D[k] = v0;
        D[k + 64] = v1;
        D[k + 128] = v2;
        D[k + 192] = v3;
        r = adv(r3);
    }
    for (; k < nq; k += 64) {
        D[k] = ln_quad_at<CAP>(win, o + r);
        r = adv(r);
    }
    return a0;
}

// 8 bytes of the window at byte a (a < CAP); near the window's end the read is moved
// back inside it and shifted (only bytes below the end are used)
template <uint32_t CAP>
__device__ __forceinline__ uint64_t ln_rd8(const uint8_t* win, uint32_t a) {
    const uint32_t c = min(a, CAP - 8);
    return *reinterpret_cast<const u64_unaligned*>(win + c) >> (8 * (a - c));
}
// the low r (1..7) bytes of x at q
__device__ __forceinline__ void ln_store_tail(uint8_t* q, uint64_t x, uint32_t r) {
    if (r & 4) {
        *reinterpret_cast<u32_unaligned*>(q) = (uint32_t)x;
        q += 4;
        x >>= 32;
    }
    if (r & 2) {
        *reinterpret_cast<u16_unaligned*>(q) = (uint16_t)x;
        q += 2;
        x >>= 16;
    }
    if (r & 1) *q = (uint8_t)x;
}

// periodic copy out[o + i] = out[o - d + (i mod d)], i < L (the reference's byte-serial
// overlapping copy, inflate.hpp:268-270): the first period (or, for d < 64, the largest
// multiple of d that fits one byte per lane) is built directly; the prefix is doubled (a plain
// copy of itself, P stays a multiple of d) until it holds a multiple Q >= 16 of d plus 16 bytes
// and the rest is more than 3 prefixes long, then ln_fill_mod writes the rest in one pass.
// `out`: where that pass writes the bytes from its first 16-byte boundary on -- the window, or
// for the segment's last token (nothing reads those bytes back) the segment's output in HBM.
// Returns the window byte from which the output went to `out` (L + o when all of it is in the
// window).
template <uint32_t CAP>
__device__ __forceinline__ uint32_t ln_copy_wave(uint8_t* win, uint32_t o, uint32_t L, uint32_t d, uint8_t* out) {
    if (d >= L) {
        ln_copy_plain<CAP>(win, o, o - d, L);
        return o + L;
    }
    uint32_t P;
    if (d >= 64) {
        ln_copy_plain<CAP>(win, o, o - d, d);
        P = d;
    } else {
        const uint32_t lane = lane_id();
        P = d * (64 / d);  // 33..64 bytes, a multiple of d
        if (lane < min(P, L)) win[o + lane] = win[o - d + lane % d];
    }
    // smallest multiple of d >= 16 (d < 16: d * ceil(16 / d), no division)
    const uint32_t c16 = d >= 16 ? d : d * (d == 1 ? 16u : d == 2 ? 8u : d == 3 ? 6u : d <= 5 ? 4u : d <= 7 ? 3u : 2u);
    // doubling while the rest is short (at most two more rounds: no divisions), or until the
    // prefix holds c16 + 16 bytes
    while (P < L && (P < c16 + 16 || L <= 4 * P)) {
        wave_sync();
        const uint32_t n = min(P, L - P);
        ln_copy_plain<CAP>(win, o + P, o, n);
        P += n;
    }
    if (P < L) {
        wave_sync();
        return ln_fill_mod<CAP>(win, o, P, L, P - c16, out);
    }
    return o + L;
}

// smallest multiple of d >= 16 (d < 16: d * ceil(16 / d), no division)
__device__ __forceinline__ uint32_t ln_c16(uint32_t d) {
    return d >= 16 ? d : d * (d == 1 ? 16u : d == 2 ? 8u : d == 3 ? 6u : d <= 5 ? 4u : d <= 7 ? 3u : 2u);
}
// the prefix length ln_copy_wave builds before its fill pass (L if none): the first period (or
// for d < 64 the largest multiple of d that fits one byte per lane), doubled while the rest is
// short (at most two more rounds: no divisions) or until it holds c16 + 16 bytes
__device__ __forceinline__ uint32_t ln_prefix_len(uint32_t L, uint32_t d) {
    uint32_t P = d >= 64 ? d : d * (64 / d);
    const uint32_t c16 = ln_c16(d);
    while (P < L && (P < c16 + 16 || L <= 4 * P)) P += min(P, L - P);
    return min(P, L);
}
// builds [o, o + P) of the periodic copy (the wave; the caller syncs before reading it)
template <uint32_t CAP>
__device__ __forceinline__ void ln_build_prefix(uint8_t* win, uint32_t o, uint32_t L, uint32_t d, uint32_t Pend) {
    uint32_t P;
    if (d >= 64) {
        ln_copy_plain<CAP>(win, o, o - d, d);
        P = d;
    } else {
        const uint32_t lane = lane_id();
        P = d * (64 / d);  // 33..64 bytes, a multiple of d
        if (lane < min(P, L)) win[o + lane] = win[o - d + lane % d];
    }
    while (P < Pend) {
        wave_sync();
        const uint32_t n = min(P, Pend - P);
        ln_copy_plain<CAP>(win, o + P, o, n);
        P += n;
    }
}

// A periodic copy of L >= RS_BIG bytes at o with distance d < L: wave 0 builds its prefix
// [o, o + P) and the bytes up to the next 16-byte boundary a0 (the caller syncs the workgroup),
// then ln_fill_wg has every thread of the workgroup write [a0, o + L) from that prefix (period
// Q = P - c16, a multiple Q >= 16 of d; the prefix holds Q + 16 bytes).
template <uint32_t CAP>
__device__ __forceinline__ void ln_fill_head(uint8_t* win, uint32_t o, uint32_t L, uint32_t d, uint32_t P) {
    ln_build_prefix<CAP>(win, o, L, d, P);
    wave_sync();
    const uint32_t beg = o + P, a0 = (beg + 15) & ~15u, Q = P - ln_c16(d);
    if (lane_id() < a0 - beg) win[beg + lane_id()] = win[o + (P + lane_id()) % Q];
}
template <uint32_t CAP, uint32_t NT>
__device__ __forceinline__ void ln_fill_wg(uint8_t* win, uint32_t o, uint32_t L, uint32_t d, uint32_t P) {
    const uint32_t t = threadIdx.x;
    const uint32_t Q = P - ln_c16(d), end = o + L, a0 = (o + P + 15) & ~15u, a1 = end & ~15u;
    const uint32_t nq = (a1 - a0) >> 4;
    const uint32_t R = (16 * NT) % Q;
    auto adv = [&](uint32_t r) { r += R; return r >= Q ? r - Q : r; };
    uint32_t r = (a0 - o + 16 * t) % Q;
    uint4* const D = reinterpret_cast<uint4*>(win + a0);
    uint32_t k = t;
    for (; k + 3 * NT < nq; k += 4 * NT) {
        const uint32_t r1 = adv(r), r2 = adv(r1), r3 = adv(r2);
        const uint4 v0 = ln_quad_at<CAP>(win, o + r), v1 = ln_quad_at<CAP>(win, o + r1);
        const uint4 v2 = ln_quad_at<CAP>(win, o + r2), v3 = ln_quad_at<CAP>(win, o + r3);
        D[k] = v0;
        D[k + NT] = v1;
        D[k + 2 * NT] = v2;
        D[k + 3 * NT] = v3;
        r = adv(r3);
    }
    for (; k < nq; k += NT) {
        D[k] = ln_quad_at<CAP>(win, o + r);
        r = adv(r);
    }
    if (t < end - a1) win[a1 + t] = win[o + (a1 - o + t) % Q];
}

// One segment of k_inflate_resolve: `sf` = its record's {out_size, flags}, n token words at tk.
// All NT threads call it.  NT = 64: one wave does everything.  NT > 64 (token lists of at most
// RS_FOLLOW words): wave 0 steps through the token words and writes the window; the other waves
// step through the words and their scan too and join the fills of long periodic copies (they
// reach the same copies in the same order: workgroup barriers in uniform control flow), the
// stored copies and the copy-out.
template <uint32_t CAP, uint32_t NT>
__device__ __forceinline__ void ln_resolve_one(const InflateArgs& A, uint64_t j, uint2 sf, uint32_t n,
                                               const uint32_t* tk, uint8_t* win, uint32_t half_off = 0) {
    constexpr bool GRP = NT > 64;
    const uint32_t lane = GRP ? lane_id() : threadIdx.x;
    const uint32_t t = threadIdx.x;  // (= lane when NT = 64)
    const bool wz = !GRP || t < 64;  // the stepping wave
    if (sf.y & ~SEGF_FINAL) return;
    const uint64_t dst0 = j * (uint64_t)A.slot + half_off;
    if (dst0 >= A.cap) return;
    const uint32_t size = sf.x;
    const uint32_t nb = (uint32_t)min((uint64_t)size, A.cap - dst0);
    uint8_t* const dst = A.out + dst0;
    if (n == 0) return;
    // the first step's token words are loaded together with word 0 (one memory latency)
    uint32_t wa = tk[min(lane, n - 1)];
    const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)wa);  // lane 0 holds word 0
    if ((w0 >> 24) == 0) {  // stored segment: straight from the stream, 16-byte stores
        // one (len, offset) word pair per stored block: one block, or two (a 64 KiB segment)
        const uint8_t* const sbase = reinterpret_cast<const uint8_t*>(A.in_words) + A.misalign + A.cands[j];
        uint32_t done = 0;
        for (uint32_t p = 0; 2 * p + 1 < n && done < nb; p++) {
            const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)wa, 2 * p);
            const uint8_t* const src = sbase + (uint32_t)__builtin_amdgcn_readlane((int)wa, 2 * p + 1);
            const uint32_t m = min(len, nb - done);
            uint8_t* const d = dst + done;
            if ((((uintptr_t)d) & 15) == 0) {
                // word-aligned source base; the words read stay inside the stream (its last word
                // holds the last data byte) except the fifth at sh == 0, which is not used then
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3);
                const uint32_t* sw = reinterpret_cast<const uint32_t*>(src - sh);
                uint4* d4 = reinterpret_cast<uint4*>(d);
                for (uint32_t i = t; i < m / 16; i += NT) {
                    const uint32_t w0 = sw[4 * i], w1 = sw[4 * i + 1], w2 = sw[4 * i + 2], w3 = sw[4 * i + 3];
                    const uint32_t w4 = sh ? sw[4 * i + 4] : 0u;
                    d4[i] = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                       __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
                }
                for (uint32_t i = (m & ~15u) + t; i < m; i += NT) d[i] = src[i];
            } else {
                for (uint32_t i = t; i < m; i += NT) d[i] = src[i];
            }
            done += m;
        }
        return;
    }
    uint64_t* const dbg = (A.dbg && t == 0) ? A.dbg + j * kPhaseSlots : nullptr;
    if (dbg) dbg[5] = __builtin_amdgcn_s_memtime();
    uint32_t pos = 0, n_cx = 0;
    // the window holds the output below lim; the rest went straight to dst (see ln_copy_wave)
    uint32_t lim = nb;
    const bool direct = nb == size && (((uintptr_t)dst) & 15) == 0;
    uint64_t c_simple = 0, c_cx = 0, tstep0 = dbg ? __builtin_amdgcn_s_memtime() : 0;  // DMX_PHASES
    // One step = 64 token words, loaded one step ahead: the memory latency of the next step's
    // load passes while this step's copies run (unconditional, index clamped, so the wait before
    // the use is for the older load only; four steps ahead measured the same on text).
    auto tstep = [&](uint32_t t0, uint32_t wraw) {
        const uint32_t w = t0 + lane < n ? wraw : 0u;
        const bool ism = (w >> 31) != 0;
        const uint32_t L = ism ? (w >> 15) & 0xFFFFu : (w >> 24) & 0x7Fu;
        const uint32_t d = (w & 0x7FFFu) + 1;
        const uint32_t inc = wave_incl_scan(L);
        const uint32_t off = pos + inc - L;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (wz && !ism) {  // literal run of 1..3 bytes: exact-size stores
            if (L & 2) {
                *reinterpret_cast<u16_unaligned*>(win + off) = (uint16_t)w;
                if (L & 1) win[off + 2] = (uint8_t)(w >> 16);
            } else if (L) {
                win[off] = (uint8_t)w;
            }
        }
        // short matches whose source lies before this step: each lane copies its own
        const bool simple = ism && L <= 32 && off + min(L, d) <= pos + d;
        if (wz && simple) {
            if (d >= L) {  // the whole source is final: read it at once (one LDS latency, not one
                           // per word), store exactly L bytes (neighbouring tokens store beside it)
                uint64_t v[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) v[k] = 8 * k < L ? ln_rd8<CAP>(win, off - d + 8 * k) : 0ull;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    const uint32_t b = 8 * k;
                    if (b + 8 <= L) *reinterpret_cast<u64_unaligned*>(win + off + b) = v[k];
                    else if (b < L) ln_store_tail(win + off + b, v[k], L - b);
                }
            } else if (d >= 4) {
                for (uint32_t i = 0; i < L; i += 4) {
                    const uint32_t v = ld32u(reinterpret_cast<const uint32_t*>(win), off + i - d);
                    win[off + i] = (uint8_t)v;
                    if (i + 1 < L) win[off + i + 1] = (uint8_t)(v >> 8);
                    if (i + 2 < L) win[off + i + 2] = (uint8_t)(v >> 16);
                    if (i + 3 < L) win[off + i + 3] = (uint8_t)(v >> 24);
                }
            } else {
                for (uint32_t i = 0; i < L; i++) win[off + i] = win[off + i - d];
            }
        }
        wave_sync();
        uint64_t m = __ballot(ism && !simple);
        uint64_t tcx0 = 0;
        if (dbg) {
            tcx0 = __builtin_amdgcn_s_memtime();
            c_simple += tcx0 - tstep0;
        }
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t ok = (uint32_t)__builtin_amdgcn_readlane((int)off, k);
            const uint32_t Lk = (uint32_t)__builtin_amdgcn_readlane((int)L, k);
            const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)d, k);
            if constexpr (GRP) {
                const uint32_t P = dk < Lk && Lk >= RS_BIG ? ln_prefix_len(Lk, dk) : Lk;
                if (P + 64 <= Lk) {  // the workgroup fills it
                    if (wz) ln_fill_head<CAP>(win, ok, Lk, dk, P);
                    __syncthreads();
                    ln_fill_wg<CAP, NT>(win, ok, Lk, dk, P);
                    __syncthreads();
                } else if (wz) {
                    ln_copy_wave<CAP>(win, ok, Lk, dk, win);
                    wave_sync();
                }
            } else {
                const bool last = DMX_LN_DIRECT && direct && t0 + (uint32_t)k + 1 == n && ok + Lk == nb;
                const uint32_t e = ln_copy_wave<CAP>(win, ok, Lk, dk, last ? dst : win);
                if (last) lim = e;
                wave_sync();
            }
            n_cx++;
        }
        if (dbg) {
            tstep0 = __builtin_amdgcn_s_memtime();
            c_cx += tstep0 - tcx0;
        }
        pos += tot;
    };
    auto ldw = [&](uint32_t t) { return tk[min(t + lane, n - 1)]; };
    for (uint32_t t0 = 0; t0 < n; t0 += 64) {
        const uint32_t w = wa;
        wa = ldw(t0 + 64);
        tstep(t0, w);
    }
    if (dbg) {
        dbg[6] = __builtin_amdgcn_s_memtime();
        dbg[12] = n_cx;
        dbg[13] = c_simple;
        dbg[14] = c_cx;
    }
    if (GRP) __syncthreads();
    if ((((uintptr_t)dst) & 15) == 0) {
        const uint32_t nv = lim / 16;  // (lim < nb: a 16-byte boundary)
        const uint4* s4 = reinterpret_cast<const uint4*>(win);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        uint32_t i = t;
        for (; i + 3 * NT < nv; i += 4 * NT) {  // four 16-byte LDS reads in flight per lane
            const uint4 v0 = s4[i], v1 = s4[i + NT], v2 = s4[i + 2 * NT], v3 = s4[i + 3 * NT];
            d4[i] = v0;
            d4[i + NT] = v1;
            d4[i + 2 * NT] = v2;
            d4[i + 3 * NT] = v3;
        }
        for (; i < nv; i += NT) d4[i] = s4[i];
        for (uint32_t i = nv * 16 + t; i < lim; i += NT) dst[i] = win[i];
    } else {
        for (uint32_t i = t; i < nb; i += NT) dst[i] = win[i];
    }
    if (dbg) dbg[7] = __builtin_amdgcn_s_memtime();
}

// one workgroup per segment (a persistent grid with ticket-drawn segments and the next record
// prefetched measured 5-20% slower on repeat and zeros, equal on text).  Two launches split the
// segments by token count: NT = RS_NT takes lists of at most RS_FOLLOW words (and stored
// segments), NT = 64 the longer ones -- one-wave workgroups step text faster (a 256-thread
// workgroup whose other waves leave at once still measured 5 % slower on 1 GiB of text).
template <uint32_t NT>
__device__ __forceinline__ bool rs_mine(uint32_t n) {
    return !kRsSplit || ((n <= RS_FOLLOW) == (NT > 64));
}
template <uint32_t CAP, uint32_t NT>
__global__ __launch_bounds__(NT) void k_inflate_resolve(InflateArgs A, LaneArgs B) {
    __shared__ __attribute__((aligned(16))) uint8_t win[CAP];  // 32 KiB: five per CU; 64 KiB: two
    const uint64_t j = blockIdx.x;
    if constexpr (CAP == LN_OUT_CAP && NT == 64 && kRsSplit) {
        // the long token lists listed by the lanes, drawn by ticket (a grid over every candidate
        // kept a 32 KiB window per empty workgroup: ~15 us on 1 GiB of repeat, which has none)
        // (the first item is the workgroup's own index: no ticket traffic when the list is
        // short or empty -- 1280 tickets drawn on one word took ~15 us)
        const uint32_t cnt = B.split[0];
        for (uint32_t i = blockIdx.x;;) {
            if (i >= cnt) break;
            const uint32_t jj = B.split[2 + i];
            const SegRecord* const rp = &A.recs[jj];
            ln_resolve_one<CAP, NT>(A, jj, make_uint2(rp->out_size, rp->flags), B.ntok[jj], B.tok + B.tokoff[jj], win);
            if (threadIdx.x == 0) i = gridDim.x + atomicAdd(B.split + 1, 1u);
            i = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
        }
        return;
    }
    // (j < A.ncand: the record, count and offset loads go out together, before the tests -- the
    // compiler otherwise sinks each below the test before it, a chain of scalar-load latencies)
    const SegRecord* const rp = &A.recs[j];
    const uint32_t n = B.ntok[j];
    const uint2 sf = make_uint2(rp->out_size, rp->flags);
    const uint64_t to = B.tokoff[j];
    const uint64_t cc = cand_count(A);
    asm volatile("" ::"s"(n), "s"(sf.x), "s"(sf.y), "s"(to), "s"(cc));
    if (j >= cc) return;
    if (CAP > LN_OUT_CAP && B.split[j] != ~0u) return;  // rebuilt by k_inflate_resolve_half
    if (!rs_mine<NT>(n)) return;
    ln_resolve_one<CAP, NT>(A, j, sf, n, B.tok + to, win);
}

// 64 KiB segments whose two 32 KiB halves are independent (every libdmx 64 KiB block: its halves
// were matched separately): two items per segment, each rebuilt in a 32 KiB window -- five
// windows per CU instead of two 64 KiB ones.  Item 2j + h: half h, token words [0, split) or
// [split, n), written at j * slot + 32768 h; a stored segment is copied whole by item 2j.
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_inflate_resolve_half(InflateArgs A, LaneArgs B) {
    __shared__ __attribute__((aligned(16))) uint8_t win[LN_OUT_CAP];
    const uint64_t j = blockIdx.x >> 1;
    const uint32_t h = blockIdx.x & 1;
    if (j >= cand_count(A)) return;
    const uint32_t sp = B.split[j];
    if (sp == ~0u) return;
    const SegRecord* const rp = &A.recs[j];
    const uint32_t size = rp->out_size, n = B.ntok[j];
    const uint32_t* const tk = B.tok + B.tokoff[j];
    if (sp == 0) {  // stored (or empty): one item copies it
        if (h == 0 && rs_mine<NT>(n)) ln_resolve_one<LN_OUT_CAP, NT>(A, j, make_uint2(size, rp->flags), n, tk, win);
        return;
    }
    if (h == 0) {
        if (rs_mine<NT>(sp)) ln_resolve_one<LN_OUT_CAP, NT>(A, j, make_uint2(min(size, LN_OUT_CAP), rp->flags), sp, tk, win);
    } else if (size > LN_OUT_CAP && rs_mine<NT>(n - sp)) {
        ln_resolve_one<LN_OUT_CAP, NT>(A, j, make_uint2(size - LN_OUT_CAP, rp->flags), n - sp, tk + sp, win, LN_OUT_CAP);
    }
}

// number of dense candidates (*cnt zeroed by the caller)
__global__ void k_heavy_count(const uint8_t* in, const uint64_t* cands, uint64_t ncand, uint64_t n, uint32_t heavy,
                              uint32_t* cnt) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ncand) return;
    const uint64_t nxt = j + 1 < ncand ? cands[j + 1] : n;
    const uint64_t b = __ballot(ln_dense(in, cands[j], n, nxt - cands[j], heavy));
    if (lane_id() == 0 && b) atomicAdd(cnt, (uint32_t)__popcll(b));  // lane 0 holds the wave's first j
}

// Chain repair (dmx_host.cpp, rare): segment chain[k] was written at chain[k] * slot of src;
// it goes to dst + offs[k] (sizes[k] bytes).  One workgroup per segment, 16-byte copies when
// both sides are aligned.
__global__ __launch_bounds__(256) void k_place_segments(const uint8_t* src, uint32_t slot, const uint64_t* chain,
                                                         const uint64_t* offs, const uint32_t* sizes,
                                                         uint64_t nch, uint8_t* dst) {
    const uint64_t k = blockIdx.x;
    if (k >= nch) return;
    const uint8_t* s = src + chain[k] * (uint64_t)slot;
    uint8_t* d = dst + offs[k];
    const uint32_t n = sizes[k];
    if ((((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(s);
        uint4* d4 = reinterpret_cast<uint4*>(d);
        for (uint32_t i = threadIdx.x; i < n / 16; i += 256) d4[i] = s4[i];
        for (uint32_t i = (n & ~15u) + threadIdx.x; i < n; i += 256) d[i] = s[i];
    } else {
        for (uint32_t i = threadIdx.x; i < n; i += 256) d[i] = s[i];
    }
}

hipError_t launch_place_segments(const uint8_t* src, uint32_t slot, const uint64_t* chain, const uint64_t* offs,
                                 const uint32_t* sizes, uint64_t nch, uint8_t* dst, hipStream_t st) {
    if (nch) hipLaunchKernelGGL(k_place_segments, dim3((uint32_t)nch), dim3(256), 0, st, src, slot, chain, offs, sizes,
                                nch, dst);
    return hipGetLastError();
}

hipError_t launch_inflate_lanes(const InflateArgs& A, uint32_t* tok, uint64_t* tokoff,
                                uint32_t* ntok, uint32_t* caps, uint32_t heavy, uint32_t limit,
                                uint32_t* hl, uint32_t* split, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, st);
    const uint32_t g = (uint32_t)((A.ncand + 255) / 256);
    const uint8_t* const in = reinterpret_cast<const uint8_t*>(A.in_words) + A.misalign;  // stream byte 0
    if (heavy) {
        const hipError_t e = hipMemsetAsync(hl, 0, 8, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_heavy_count, dim3(g), dim3(256), 0, st, in, A.cands, A.ncand, A.n, heavy, hl + 1);
    }
    const bool big = A.slot > LN_OUT_CAP;  // 64 KiB segments (config C4's blocks)
    hipLaunchKernelGGL(k_lane_caps, dim3(g), dim3(256), 0, st, in, A.cands, A.ncand, A.n, caps, heavy, limit, hl,
                       big ? 2 * LN_OUT_CAP : LN_OUT_CAP, A.ncand_dev, !big && kRsSplit ? split : nullptr);
    hipError_t e = launch_scan_u32(caps, tokoff, A.ncand, tokoff + A.ncand, st);
    if (e != hipSuccess) return e;
    LaneArgs B{tok, tokoff, ntok, caps, split};
    if (big) {
        // (32 segments per wave here too: 16 per wave measured slower at 1 GiB of mixed data,
        // 17.5 against ~14.5 ms for the lanes, though it puts a wave on every SIMD)
        constexpr uint32_t NL = LN_LANES;
        const dim3 lg((uint32_t)((A.ncand + NL - 1) / NL));
        hipLaunchKernelGGL((k_inflate_lanes<2 * LN_OUT_CAP, NL>), lg, dim3(64), 0, st, A, B);
        hipLaunchKernelGGL(k_inflate_resolve_half<RS_NT>, dim3((uint32_t)(2 * A.ncand)), dim3(RS_NT), 0, st, A, B);
        hipLaunchKernelGGL((k_inflate_resolve<2 * LN_OUT_CAP, RS_NT>), dim3((uint32_t)A.ncand), dim3(RS_NT), 0, st, A, B);
        if (kRsSplit) {
            hipLaunchKernelGGL(k_inflate_resolve_half<64>, dim3((uint32_t)(2 * A.ncand)), dim3(64), 0, st, A, B);
            hipLaunchKernelGGL((k_inflate_resolve<2 * LN_OUT_CAP, 64>), dim3((uint32_t)A.ncand), dim3(64), 0, st, A, B);
        }
    } else {
        const dim3 lg((uint32_t)((A.ncand + LN_LANES - 1) / LN_LANES));
        hipLaunchKernelGGL((k_inflate_lanes<LN_OUT_CAP, LN_LANES>), lg, dim3(64), 0, st, A, B);
        hipLaunchKernelGGL((k_inflate_resolve<LN_OUT_CAP, RS_NT>), dim3((uint32_t)A.ncand), dim3(RS_NT), 0, st, A, B);
        if (kRsSplit) {
            static int ncu = 0;
            if (!ncu) {
                int dev = 0;
                (void)hipGetDevice(&dev);
                if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
                    ncu = 256;
            }
            const uint32_t g = (uint32_t)std::min<uint64_t>(A.ncand, (uint64_t)RS_TICKET_WG * (uint64_t)ncu);
            if (g) hipLaunchKernelGGL((k_inflate_resolve<LN_OUT_CAP, 64>), dim3(g), dim3(64), 0, st, A, B);
        }
    }
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

}  // namespace dmx
