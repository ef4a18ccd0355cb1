// deflate_kernels.hip -- MI355X (gfx950) DEFLATE encoder kernels.
//
// One 256-thread workgroup compresses one independent segment (16 or 32 KiB) entirely out of
// LDS, the way the reference compresses one 32 KiB chunk with a fresh LZ77 state
// (realCompress, /root/reference/include/deflate.hpp:680-752):
//
//   load (16 B/lane coalesced)  -> LDS byte image of the segment
//   match candidates            -> LDS hash table (u32 head, atomicMax), rounds of 1024
//                                  positions; cand[p] = distance to the latest earlier
//                                  occurrence of the 4-byte prefix   (replaces LZ77::getMatches
//                                  deflate.hpp:310-383 / getMatchesSlow :268-304)
//   tokenize walk               -> 256-byte chunk per lane, greedy (level 2) or one-step lazy
//                                  (level 3) parse; matches never cross a chunk edge, so chunks
//                                  parse independently; LDS histogram   (constructDynamicHuffmanTree
//                                  :402-418)
//   code lengths                -> block-parallel length-limited Huffman
//                                  (FlatHuffmanTree::generateCodeLengths common.hpp:322-404)
//   canonical codes             -> (FlatHuffmanTree::construct common.hpp:104-145)
//   dynamic header              -> parallel RLE of the two code-length sequences, precode
//                                  (writeDynamicHuffmanTree deflate.hpp:544-626)
//   bit pack                    -> per-lane bit counts, block scan, per-lane 64-bit
//                                  accumulators OR-ed into an LDS word image  (compressBuffer
//                                  deflate.hpp:630-674, Bitstream :80-159)
//   store                       -> dynamic / fixed / stored, whichever is smallest
//                                  (deflate.hpp:739-746), then an empty stored block so every
//                                  segment ends byte-aligned (segments concatenate bytewise).
//
// A second kernel scans the per-segment sizes and a third compacts the segment slots.
#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

constexpr int DF_NT = 256;     // threads per workgroup
constexpr int DF_CHUNK = 256;  // bytes per tokenizer lane

template <int SEG>
struct DfSmem {
    static constexpr int HB = (SEG >= 32768) ? 13 : 12;
    static constexpr int NWALK = SEG / DF_CHUNK;
    static constexpr int UW0 = 1 << HB;
    static constexpr int UW1 = SEG / 4 + 64;
    static constexpr int UW = UW0 > UW1 ? UW0 : UW1;
    uint32_t data32[SEG / 4 + 16];
    uint16_t cand[SEG + 8];
    uint32_t U[UW];  // hash head during matching, output bit image afterwards
    uint32_t litfreq[288];
    uint32_t distfreq[32];
    uint32_t prefreq[32];
    uint32_t litcode[288];  // (len << 16) | bit-reversed code
    uint32_t distcode[32];
    uint32_t precode[32];
    uint8_t litlen[288];
    uint8_t distlen[32];
    uint8_t prelen[32];
    uint16_t order[320];
    uint32_t scan[2 * DF_NT];
    uint32_t sh[48];
};

// ---------------------------------------------------------------------------------------
// block primitives
// ---------------------------------------------------------------------------------------

// exclusive block scan of one value per thread; returns the prefix, *total gets the sum
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    const int t = threadIdx.x, w = t >> 6;
    uint32_t inc = wave_incl_scan(v);
    if ((t & 63) == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < DF_NT / 64; i++) {
        uint32_t s = scratch[i];
        if (i < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// Length-limited code lengths for freq[0..nsym), written to lens[].  Block-parallel:
//  1. L = round(log2(F/f)) clamped to [1, maxbits]  (rank symbols by (f desc, sym asc))
//  2. Kraft repair: while sum 2^-L > 1 lengthen the least frequent codes, longest class first
//  3. slack fill: per class of equal length (shortest first) shorten the most frequent codes
//     while the Kraft budget allows; repeat until the code is complete.
// Zero or one used symbol -> two codes of length 1 (complete code, as zlib emits).
// Stands in for FlatHuffmanTree::generateCodeLengths (common.hpp:322-404), which is a serial
// priority-queue Huffman; this one stays within ~1% of optimal.
__device__ void build_lengths(const uint32_t* freq, int nsym, int maxbits, uint8_t* lens,
                              uint16_t* order, uint32_t* sh) {
    const int t = threadIdx.x;
    if (t == 0) { sh[0] = 0; sh[1] = 0; sh[2] = 0; }
    __syncthreads();
    for (int s = t; s < nsym; s += DF_NT) {
        uint32_t f = freq[s];
        if (f) { atomicAdd(&sh[0], f); atomicAdd(&sh[1], 1u); }
    }
    __syncthreads();
    const uint32_t F = sh[0], nz = sh[1];
    const uint32_t U = 1u << maxbits;
    if (nz <= 1) {
        for (int s = t; s < nsym; s += DF_NT) lens[s] = 0;
        __syncthreads();
        if (t == 0) {
            int used = -1;
            for (int s = 0; s < nsym; s++)
                if (freq[s]) { used = s; break; }
            if (used < 0) { lens[0] = 1; lens[1] = 1; }
            else { lens[used] = 1; lens[used == 0 ? 1 : 0] = 1; }
        }
        __syncthreads();
        return;
    }
    for (int s = t; s < nsym; s += DF_NT) {
        uint32_t f = freq[s];
        uint32_t L = 0;
        if (f) {
            uint32_t L0 = 31 - __clz(F / f);
            uint64_t a = (uint64_t)f << (L0 + 1);
            L = L0 + ((a * a <= 2ull * F * F) ? 1u : 0u);
            L = max(1u, min((uint32_t)maxbits, L));
            atomicAdd(&sh[2], U >> L);
            uint32_t rank = 0;
            for (int s2 = 0; s2 < nsym; s2++) {
                uint32_t f2 = freq[s2];
                rank += (f2 > f) || (f2 == f && s2 < s);
            }
            order[rank] = (uint16_t)s;
        }
        lens[s] = (uint8_t)L;
    }
    __syncthreads();
    if (t < 64) {
        const int lane = t;
        const uint32_t S = (nz + 63) / 64;  // <= 5
        uint32_t sym[5], len[5];
        bool val[5];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            uint32_t r = lane * S + i;
            val[i] = (uint32_t)i < S && r < nz;
            sym[i] = val[i] ? order[r] : 0;
            len[i] = val[i] ? lens[sym[i]] : 0;
        }
        uint32_t K = sh[2];
        // Kraft repair (over-full after rounding / clamping)
        while (K > U) {
            for (int L = maxbits - 1; L >= 1 && K > U; L--) {
                const uint32_t gain = U >> (L + 1);
                const uint32_t need = (K - U + gain - 1) / gain;
                uint32_t cnt = 0;
#pragma unroll
                for (int i = 0; i < 5; i++) cnt += (val[i] && len[i] == (uint32_t)L);
                uint32_t inc = wave_incl_scan(cnt);
                uint32_t total = __shfl(inc, 63, 64);
                uint32_t after = total - inc;  // class members with a higher rank
                uint32_t k = min(need, total);
                uint32_t local = 0;
#pragma unroll
                for (int i = 4; i >= 0; i--) {
                    if (val[i] && len[i] == (uint32_t)L) {
                        if (after + local < k) len[i] = L + 1;
                        local++;
                    }
                }
                K -= k * gain;
            }
        }
        // slack fill
        uint32_t R = U - K;
        for (int pass = 0; pass < 64 && R; pass++) {
            bool changed = false;
            for (int L = 2; L <= maxbits; L++) {
                const uint32_t c = U >> L;
                uint32_t cnt = 0;
#pragma unroll
                for (int i = 0; i < 5; i++) cnt += (val[i] && len[i] == (uint32_t)L);
                uint32_t inc = wave_incl_scan(cnt);
                uint32_t total = __shfl(inc, 63, 64);
                uint32_t before = inc - cnt;
                uint32_t k = min(total, R / c);
                if (k) { changed = true; R -= k * c; }
                uint32_t local = 0;
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    if (val[i] && len[i] == (uint32_t)L) {
                        if (before + local < k) len[i] = L - 1;
                        local++;
                    }
                }
            }
            if (!changed) break;
        }
#pragma unroll
        for (int i = 0; i < 5; i++)
            if (val[i]) lens[sym[i]] = (uint8_t)len[i];
    }
    __syncthreads();
}

// Canonical codes (RFC 1951 3.2.2; reference FlatHuffmanTree::construct common.hpp:104-145),
// stored bit-reversed for the LSB-first bit packer: codes[s] = (len << 16) | rev(code).
__device__ void assign_codes(const uint8_t* lens, int nsym, uint32_t* codes, uint32_t* sh) {
    const int t = threadIdx.x;
    if (t < 32) sh[t] = 0;
    __syncthreads();
    for (int s = t; s < nsym; s += DF_NT)
        if (lens[s]) atomicAdd(&sh[lens[s]], 1u);
    __syncthreads();
    if (t == 0) {
        uint32_t code = 0;
        for (int b = 1; b <= 15; b++) {
            code = (code + (b > 1 ? sh[b - 1] : 0)) << 1;
            sh[16 + b] = code;
        }
    }
    __syncthreads();
    for (int s = t; s < nsym; s += DF_NT) {
        uint32_t L = lens[s];
        uint32_t v = 0;
        if (L) {
            uint32_t rank = 0;
            for (int s2 = 0; s2 < s; s2++) rank += (lens[s2] == L);
            v = (L << 16) | bitrev(sh[16 + L] + rank, L);
        }
        codes[s] = v;
    }
    __syncthreads();
}

// LSB-first bit writer that ORs 32-bit words into an LDS image (image pre-zeroed).
struct BitOr {
    uint32_t* out;
    uint64_t acc;
    uint32_t nacc, wi;
    __device__ void init(uint32_t* o, uint32_t bitpos) {
        out = o;
        wi = bitpos >> 5;
        nacc = bitpos & 31;
        acc = 0;
    }
    __device__ void put(uint32_t bits, uint32_t n) {  // n <= 32
        acc |= (uint64_t)bits << nacc;
        nacc += n;
        if (nacc >= 32) {
            atomicOr(&out[wi], (uint32_t)acc);
            wi++;
            acc >>= 32;
            nacc -= 32;
        }
    }
    __device__ void flush() {
        if (nacc) atomicOr(&out[wi], (uint32_t)acc);
    }
};

__device__ __forceinline__ uint32_t matchlen(const uint32_t* w, uint32_t p, uint32_t q,
                                             uint32_t maxl) {
    uint32_t L = 0;
    while (L < maxl) {
        uint32_t x = ld32u(w, p + L) ^ ld32u(w, q + L);
        if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
        L += 4;
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
// the segment kernel
// ---------------------------------------------------------------------------------------

// stored block: [BFINAL|00][LEN][NLEN][data] (+ empty stored block unless final)
template <int SEG>
__device__ void emit_stored(DfSmem<SEG>& S, uint32_t nb, bool is_final, uint8_t* slot,
                            uint32_t* size_out) {
    const int t = threadIdx.x;
    __syncthreads();
    const uint32_t total = 5 + nb + (is_final ? 0 : 5);
    const uint32_t nw = (total + 3) / 4;
    // word k holds output bytes 4k..4k+3 = data bytes 4k-5 .. 4k-2
    for (uint32_t k = t; k < nw; k += DF_NT) {
        uint32_t v;
        if (k == 0) {
            v = (is_final ? 1u : 0u) | ((nb & 0xFF) << 8) | (((nb >> 8) & 0xFF) << 16) |
                ((~nb & 0xFF) << 24);
        } else if (k == 1) {
            v = ((~nb >> 8) & 0xFF) | ((uint32_t)data_byte(S.data32, 0) << 8) |
                ((uint32_t)data_byte(S.data32, 1) << 16) | ((uint32_t)data_byte(S.data32, 2) << 24);
        } else {
            v = ld32u(S.data32, 4 * k - 5);
        }
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t pos = 4 * k + b;
            uint32_t byte = (v >> (8 * b)) & 0xFF;
            if (pos >= 5 + nb) byte = (!is_final && pos >= 5 + nb + 3) ? 0xFF : 0;
            w |= byte << (8 * b);
        }
        S.U[k] = w;
    }
    __syncthreads();
    const uint32_t nv = (total + 15) / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(S.U);
    uint4* d4 = reinterpret_cast<uint4*>(slot);
    for (uint32_t i = t; i < nv; i += DF_NT) d4[i] = s4[i];
    if (t == 0) *size_out = total;
}

// Huffman (dynamic or fixed) block for the tokenized segment; returns false when a stored
// block would be smaller (the caller then emits it), true after writing the slot.
template <int SEG>
__device__ bool emit_huffman(DfSmem<SEG>& S, uint32_t nb, bool is_final, uint8_t* slot,
                             uint32_t* size_out) {
    constexpr int NWALK = DfSmem<SEG>::NWALK;
    const int t = threadIdx.x;

    // ---- code lengths + canonical codes -------------------------------------------------
    build_lengths(S.litfreq, 286, 15, S.litlen, S.order, S.sh);
    build_lengths(S.distfreq, 30, 15, S.distlen, S.order, S.sh);
    assign_codes(S.litlen, 286, S.litcode, S.sh);
    assign_codes(S.distlen, 30, S.distcode, S.sh);

    // ---- token cost under the dynamic and the fixed code; HLIT / HDIST ------------------
    if (t < 8) S.sh[32 + t] = 0;
    __syncthreads();
    {
        uint32_t dyn = 0, fix = 0, ml = 0, md = 0;
        for (int s = t; s < 286; s += DF_NT) {
            if (S.litlen[s]) ml = max(ml, (uint32_t)s + 1);
            const uint32_t f = S.litfreq[s];
            if (!f) continue;
            const uint32_t ex = s > 256 ? kLenExtra[s - 257] : 0;
            dyn += f * (S.litlen[s] + ex);
            fix += f * (fixed_lit_len(s) + ex);
        }
        if (t < 30) {
            const uint32_t f = S.distfreq[t];
            dyn += f * (S.distlen[t] + kDistExtra[t]);
            fix += f * (5 + kDistExtra[t]);
            if (S.distlen[t]) md = t + 1;
        }
        atomicAdd(&S.sh[32], dyn);
        atomicAdd(&S.sh[33], fix);
        atomicMax(&S.sh[34], ml);
        atomicMax(&S.sh[35], md);
    }
    __syncthreads();
    const uint32_t dyn_tok = S.sh[32], fix_tok = S.sh[33];
    const uint32_t nlit = max(257u, S.sh[34]), ndist = max(1u, S.sh[35]);
    const uint32_t nall = nlit + ndist;

    // ---- dynamic header: RLE runs over (litlen[0..nlit), distlen[0..ndist)) -------------
    RunPlan plan[2];
    uint32_t runv[2] = {0, 0};
    bool isrun[2] = {false, false};
    for (int k = 0; k < 2; k++) {
        const uint32_t i = t + k * DF_NT;
        if (i >= nall) continue;
        const uint32_t send = i < nlit ? nlit : nall;
        const uint32_t v = i < nlit ? S.litlen[i] : S.distlen[i - nlit];
        bool start = (i == 0 || i == nlit);
        if (!start) {
            const uint32_t pv = (i - 1) < nlit ? S.litlen[i - 1] : S.distlen[i - 1 - nlit];
            start = pv != v;
        }
        if (!start) continue;
        uint32_t j = i + 1;
        while (j < send && (j < nlit ? S.litlen[j] : S.distlen[j - nlit]) == v) j++;
        isrun[k] = true;
        runv[k] = v;
        plan[k] = plan_run(v, j - i);
        const RunPlan& p = plan[k];
        if (p.n18) atomicAdd(&S.prefreq[18], p.n18);
        if (p.n17) atomicAdd(&S.prefreq[17], p.n17);
        if (p.n16) atomicAdd(&S.prefreq[16], p.n16);
        if (p.nlit) atomicAdd(&S.prefreq[v], p.nlit);
    }
    __syncthreads();
    build_lengths(S.prefreq, 19, 7, S.prelen, S.order, S.sh);
    assign_codes(S.prelen, 19, S.precode, S.sh);
    uint32_t hclen = 4;
    for (int i = 18; i >= 4; i--)
        if (S.prelen[kPerm[i]]) { hclen = i + 1; break; }
    uint32_t runbits[2] = {0, 0};
    for (int k = 0; k < 2; k++) {
        if (!isrun[k]) continue;
        const RunPlan& p = plan[k];
        runbits[k] = p.n18 * (S.prelen[18] + 7) + p.n17 * (S.prelen[17] + 3) +
                     p.n16 * (S.prelen[16] + 2) + p.nlit * S.prelen[runv[k]];
    }
    uint32_t rtot0, rtot1;
    const uint32_t off0 = block_excl_scan(runbits[0], S.scan, &rtot0);
    const uint32_t off1 = block_excl_scan(runbits[1], S.scan, &rtot1);
    const uint32_t hdr_bits = 14 + 3 * hclen + rtot0 + rtot1;  // after the 3-bit block header

    // ---- choose the block type (reference deflate.hpp:739-746 picks the smallest too) ----
    const uint64_t dyn_bits = 3ull + hdr_bits + dyn_tok;
    const uint64_t fix_bits = 3ull + fix_tok;
    const bool use_dyn = dyn_bits <= fix_bits;
    const uint64_t bits = use_dyn ? dyn_bits : fix_bits;
    const uint64_t hbytes = is_final ? (bits + 7) / 8 : (bits + 3 + 7) / 8 + 4;
    const uint64_t stored_bytes = 5ull + nb + (is_final ? 0 : 5);
    if (hbytes >= stored_bytes) return false;

    if (!use_dyn) {
        for (int s = t; s < 286; s += DF_NT) S.litcode[s] = (fixed_lit_len(s) << 16) | fixed_lit_code(s);
        if (t < 30) S.distcode[t] = (5u << 16) | bitrev(t, 5);
        __syncthreads();
    }

    // ---- per-lane token bit counts and block scan ---------------------------------------
    uint32_t mybits = 0;
    if (t < NWALK) {
        const uint32_t lo = t * DF_CHUNK, hi = min(lo + DF_CHUNK, nb);
        uint32_t p = lo;
        while (p < hi) {
            const uint32_t d = S.cand[p];
            if (d) {
                const uint32_t L = S.cand[p + 1];
                const uint32_t ls = len_sym(L), ds = dist_sym(d);
                mybits += (S.litcode[ls] >> 16) + kLenExtra[ls - 257] + (S.distcode[ds] >> 16) +
                          kDistExtra[ds];
                p += L;
            } else {
                mybits += S.litcode[data_byte(S.data32, p)] >> 16;
                p++;
            }
        }
    }
    uint32_t tok_total;
    const uint32_t tok_off = block_excl_scan(mybits, S.scan, &tok_total);
    const uint32_t hdr_end = 3 + (use_dyn ? hdr_bits : 0);

    // ---- emission into the zeroed LDS image ---------------------------------------------
    if (t == 0) {
        BitOr bw;
        bw.init(S.U, 0);
        bw.put((is_final ? 1u : 0u) | ((use_dyn ? 2u : 1u) << 1), 3);
        if (use_dyn) {
            bw.put(nlit - 257, 5);
            bw.put(ndist - 1, 5);
            bw.put(hclen - 4, 4);
            for (uint32_t i = 0; i < hclen; i++) bw.put(S.prelen[kPerm[i]], 3);
        }
        bw.flush();
    }
    if (use_dyn) {
        const uint32_t rbase = 3 + 14 + 3 * hclen;
        for (int k = 0; k < 2; k++) {
            if (!isrun[k]) continue;
            const RunPlan& p = plan[k];
            BitOr bw;
            bw.init(S.U, rbase + (k == 0 ? off0 : rtot0 + off1));
            const uint32_t v = runv[k];
            if (v == 0) {
                const uint32_t c18 = S.precode[18] & 0xFFFF, l18 = S.precode[18] >> 16;
                for (uint32_t q = 0; q < p.n18; q++) {
                    const uint32_t rep = (q + 1 == p.n18) ? p.last18 : 138;
                    bw.put(c18, l18);
                    bw.put(rep - 11, 7);
                }
                if (p.n17) {
                    bw.put(S.precode[17] & 0xFFFF, S.precode[17] >> 16);
                    bw.put(p.r17 - 3, 3);
                }
                for (uint32_t q = 0; q < p.nlit; q++) bw.put(S.precode[0] & 0xFFFF, S.precode[0] >> 16);
            } else {
                const uint32_t cv = S.precode[v] & 0xFFFF, lv = S.precode[v] >> 16;
                bw.put(cv, lv);
                const uint32_t c16 = S.precode[16] & 0xFFFF, l16 = S.precode[16] >> 16;
                for (uint32_t q = 0; q < p.n16; q++) {
                    const uint32_t rep = (q + 1 == p.n16) ? p.last16 : 6;
                    bw.put(c16, l16);
                    bw.put(rep - 3, 2);
                }
                for (uint32_t q = 1; q < p.nlit; q++) bw.put(cv, lv);
            }
            bw.flush();
        }
    }
    if (t < NWALK) {
        BitOr bw;
        bw.init(S.U, hdr_end + tok_off);
        const uint32_t lo = t * DF_CHUNK, hi = min(lo + DF_CHUNK, nb);
        uint32_t p = lo;
        while (p < hi) {
            const uint32_t d = S.cand[p];
            if (d) {
                const uint32_t L = S.cand[p + 1];
                const uint32_t ls = len_sym(L), ds = dist_sym(d);
                const uint32_t lc = S.litcode[ls];
                bw.put(lc & 0xFFFF, lc >> 16);
                const uint32_t le = kLenExtra[ls - 257];
                if (le) bw.put(L - kLenBase[ls - 257], le);
                const uint32_t dc = S.distcode[ds];
                bw.put(dc & 0xFFFF, dc >> 16);
                const uint32_t de = kDistExtra[ds];
                if (de) bw.put(d - kDistBase[ds], de);
                p += L;
            } else {
                const uint32_t lc = S.litcode[data_byte(S.data32, p)];
                bw.put(lc & 0xFFFF, lc >> 16);
                p++;
            }
        }
        bw.flush();
    }
    // end of block, then (non-final) the byte-aligning empty stored block 000|pad|0000|FFFF
    const uint32_t eob_at = hdr_end + tok_total;
    const uint32_t eob = S.litcode[256];
    const uint32_t end_bits = eob_at + (eob >> 16);
    const uint32_t total = is_final ? (end_bits + 7) / 8 : (end_bits + 3 + 7) / 8 + 4;
    if (t == 0) {
        BitOr bw;
        bw.init(S.U, eob_at);
        bw.put(eob & 0xFFFF, eob >> 16);
        bw.flush();
        if (!is_final) {
            atomicOr(&S.U[(total - 2) >> 2], 0xFFu << (((total - 2) & 3) * 8));
            atomicOr(&S.U[(total - 1) >> 2], 0xFFu << (((total - 1) & 3) * 8));
        }
    }
    __syncthreads();
    const uint32_t nv = (total + 15) / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(S.U);
    uint4* d4 = reinterpret_cast<uint4*>(slot);
    for (uint32_t i = t; i < nv; i += DF_NT) d4[i] = s4[i];
    if (t == 0) *size_out = total;
    return true;
}

template <int SEG>
__global__ __launch_bounds__(DF_NT) void k_deflate_segments(DeflateArgs A) {
    __shared__ DfSmem<SEG> S;
    constexpr int HB = DfSmem<SEG>::HB;
    constexpr int NWALK = DfSmem<SEG>::NWALK;
    const int t = threadIdx.x;
    const uint64_t seg = blockIdx.x;
    const uint64_t base = seg * (uint64_t)SEG;
    const uint32_t nb = (uint32_t)min((uint64_t)SEG, A.n - base);
    const bool is_final = (seg + 1 == A.nseg) && A.final_last;
    const int level = A.level;
    uint8_t* const slot = A.slots + seg * (uint64_t)A.slot_bytes;
    uint8_t* const dbytes = reinterpret_cast<uint8_t*>(S.data32);

    // ---- load the segment into LDS (16 B per lane when aligned) ------------------------
    {
        const uint8_t* src = A.in + base;
        const uint32_t nvec = nb / 16;
        if ((((uintptr_t)src) & 15) == 0) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src);
            uint4* d4 = reinterpret_cast<uint4*>(S.data32);
            for (uint32_t i = t; i < nvec; i += DF_NT) d4[i] = s4[i];
            for (uint32_t i = nvec * 16 + t; i < nb; i += DF_NT) dbytes[i] = src[i];
        } else {
            for (uint32_t i = t; i < nb; i += DF_NT) dbytes[i] = src[i];
        }
        // zero padding after the data (match compares read up to 8 bytes past)
        for (uint32_t i = nb + t; i < ((nb + 3) & ~3u) + 32; i += DF_NT) dbytes[i] = 0;
        for (int i = t; i < 288; i += DF_NT) S.litfreq[i] = 0;
        if (t < 32) { S.distfreq[t] = 0; S.prefreq[t] = 0; }
        if (level >= 2)
            for (int i = t; i < (1 << HB); i += DF_NT) S.U[i] = 0;
    }
    __syncthreads();

    if (level != 0) {
        // ---- match candidates: rounds of 1024 positions, 4 consecutive per thread ------
        if (level >= 2) {
            for (uint32_t r0 = 0; r0 < nb; r0 += 4 * DF_NT) {
                const uint32_t p0 = r0 + 4 * t;
                uint32_t h[4];
                bool ok[4] = {false, false, false, false};
                if (p0 < nb) {
                    const uint32_t w0 = S.data32[p0 >> 2], w1 = S.data32[(p0 >> 2) + 1];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t p = p0 + j;
                        ok[j] = p + 4 <= nb;
                        const uint32_t v = __builtin_amdgcn_alignbyte(w1, w0, j);
                        h[j] = (v * 0x1E35A7BDu) >> (32 - HB);
                        uint32_t c = 0;
                        if (ok[j]) {
                            const uint32_t q = S.U[h[j]];
                            if (q) {
                                c = p - (q - 1);
                                if (c > 32768) c = 0;
                            }
                        }
                        if (p < nb) S.cand[p] = (uint16_t)c;
                    }
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (ok[j]) atomicMax(&S.U[h[j]], p0 + j + 1);
                __syncthreads();
            }
        }

        // ---- tokenize walk: one 256-byte chunk per lane ----------------------------------
        if (t < NWALK) {
            const uint32_t lo = t * DF_CHUNK;
            const uint32_t hi = min(lo + DF_CHUNK, nb);
            uint32_t p = lo;
            while (p < hi) {
                const uint32_t d = (level >= 2) ? S.cand[p] : 0;
                uint32_t L = 0;
                if (d) L = matchlen(S.data32, p, p - d, min(258u, hi - p));
                if (level == 3 && L >= 3 && L < 258 && p + 1 < hi) {
                    const uint32_t d2 = S.cand[p + 1];
                    if (d2) {
                        const uint32_t L2 = matchlen(S.data32, p + 1, p + 1 - d2, min(258u, hi - p - 1));
                        if (L2 > L) L = 0;  // literal here, the longer match starts next
                    }
                }
                if (L >= 3) {
                    atomicAdd(&S.litfreq[len_sym(L)], 1u);
                    atomicAdd(&S.distfreq[dist_sym(d)], 1u);
                    S.cand[p + 1] = (uint16_t)L;
                    p += L;
                } else {
                    S.cand[p] = 0;
                    atomicAdd(&S.litfreq[dbytes[p]], 1u);
                    p++;
                }
            }
        }
        if (t == 0) S.litfreq[256] = 1;  // end-of-block
        __syncthreads();
        for (int i = t; i < DfSmem<SEG>::UW; i += DF_NT) S.U[i] = 0;
        // emit_huffman's first barrier orders the zeroing before any emission
        if (emit_huffman<SEG>(S, nb, is_final, slot, &A.sizes[seg])) return;
    }
    emit_stored<SEG>(S, nb, is_final, slot, &A.sizes[seg]);
}

// exclusive scan of segment sizes -> offsets (single workgroup of 1024 threads)
__global__ __launch_bounds__(1024) void k_scan_sizes(const uint32_t* sizes, uint64_t* offs,
                                                      uint64_t nseg, uint64_t* total) {
    __shared__ uint64_t part[1024];
    const int t = threadIdx.x;
    const uint64_t per = (nseg + 1023) / 1024;
    const uint64_t b = t * per, e = min(nseg, b + per);
    uint64_t s = 0;
    for (uint64_t i = b; i < e; i++) s += sizes[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t v = (t >= d) ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - s;
    for (uint64_t i = b; i < e; i++) {
        offs[i] = run;
        run += sizes[i];
    }
    if (t == 1023) *total = part[1023];
}

// copy each segment slot to its place in the contiguous stream
__global__ __launch_bounds__(256) void k_compact(const uint8_t* slots, uint32_t slot_bytes,
                                                  const uint32_t* sizes, const uint64_t* offs,
                                                  uint8_t* out, uint64_t cap) {
    const uint64_t s = blockIdx.x;
    const uint32_t sz = sizes[s];
    const uint64_t o = offs[s];
    const uint8_t* src = slots + s * (uint64_t)slot_bytes;
    if (o + sz > cap) return;
    uint8_t* dst = out + o;
    // align the destination to 4 bytes, then move words built with alignbyte
    const uint32_t head = (uint32_t)((4 - ((uintptr_t)dst & 3)) & 3);
    const uint32_t hb = min(head, sz);
    for (uint32_t i = threadIdx.x; i < hb; i += 256) dst[i] = src[i];
    if (sz <= hb) return;
    const uint32_t rem = sz - hb;
    const uint32_t nw = rem / 4;
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst + hb);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(src);  // slot is 256-B aligned
    for (uint32_t k = threadIdx.x; k < nw; k += 256) {
        const uint32_t p = hb + 4 * k;
        dw[k] = __builtin_amdgcn_alignbyte(sw[(p >> 2) + 1], sw[p >> 2], p & 3);
    }
    for (uint32_t i = hb + nw * 4 + threadIdx.x; i < sz; i += 256) dst[i] = src[i];
}

hipError_t launch_deflate(const DeflateArgs& A, uint32_t seg_bytes, hipStream_t st,
                          hipEvent_t ev_main0, hipEvent_t ev_main1) {
    if (ev_main0) (void)hipEventRecord(ev_main0, st);
    if (seg_bytes == 32768)
        hipLaunchKernelGGL(k_deflate_segments<32768>, dim3((uint32_t)A.nseg), dim3(DF_NT), 0, st, A);
    else
        hipLaunchKernelGGL(k_deflate_segments<16384>, dim3((uint32_t)A.nseg), dim3(DF_NT), 0, st, A);
    if (ev_main1) (void)hipEventRecord(ev_main1, st);
    hipLaunchKernelGGL(k_scan_sizes, dim3(1), dim3(1024), 0, st, A.sizes, A.offsets, A.nseg, A.total);
    hipLaunchKernelGGL(k_compact, dim3((uint32_t)A.nseg), dim3(256), 0, st, A.slots, A.slot_bytes,
                       A.sizes, A.offsets, A.out, A.cap);
    return hipGetLastError();
}

hipError_t launch_scan_u32(const uint32_t* v, uint64_t* offs, uint64_t n, uint64_t* total,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_scan_sizes, dim3(1), dim3(1024), 0, st, v, offs, n, total);
    return hipGetLastError();
}

}  // namespace dmx
