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
#include "inflate_common.h"

namespace dmx {

// output sink of the segment-parallel path: the segment's bytes in LDS
struct SegSink {
    uint8_t* win;
    uint32_t pos;
    bool stream_start;
    uint32_t err;
    uint32_t cap = SEG_CAP;  // window bytes (the segment check takes 64 KiB segments)
    __device__ bool full() const { return false; }
    __device__ bool literal(uint32_t b) {
        if (pos >= cap) { err |= SEGF_OVERFLOW; return false; }
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
        if (pos + L > cap) { err |= SEGF_OVERFLOW; return false; }
        lz_copy_lds<0xFFFFFFFFu>(win, pos, L, dist);
        pos += L;
        return true;
    }
    template <class BR>
    __device__ bool stored(const BR& br, uint64_t b0, uint32_t len) {
        if (pos + len > cap) { err |= SEGF_OVERFLOW; return false; }
        for (uint32_t i = lane_id(); i < len; i += 64) win[pos + i] = br.byte_at(b0 + i);
        pos += len;
        return true;
    }
};


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
                                                        uint64_t* cands, uint64_t cand_cap) {
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
        if (o < cand_cap) cands[o] = 16 * g + i - misalign;
        o++;
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
                               uint64_t cand_cap, hipStream_t st) {
    hipLaunchKernelGGL(k_marker_write, dim3((uint32_t)ntiles), dim3(MK_NT), 0, st, in_words,
                       misalign, n, tile_offs, cands, cand_cap);
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
    SegSink sk{win, 0, j == 0 && !(A.flags & DMX_IFLAG_PIECE), 0};
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
#ifndef PJ_MINBITS_
#define PJ_MINBITS_ 192u  // (256: +7 % on text, 384: +14 %; measured with the 320-bit warm-up)
#endif
constexpr uint32_t PJ_MINBITS = PJ_MINBITS_;  // shortest range (bits) a lane decodes
#ifndef PJ_LIST_NT
#define PJ_LIST_NT 512  // lanes per workgroup of the heavy route (k_inflate_pj_list)
#endif
#ifndef PJ_MINBITS_1K
#define PJ_MINBITS_1K 128u  // shortest range with 1024 lanes
#endif
#ifndef PJ_WARM
#define PJ_WARM 320u  // warm-up bits before a range's first pass (128: +25 % on text, 512: +1 %)
#endif

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

template <int SEG, int NT>
__device__ __forceinline__ void pj_segment(const InflateArgs& A, PjSmem<SEG, NT>& S, const uint64_t j) {
    using Smem = PjSmem<SEG, NT>;
    constexpr int NW = NT / 64;
    const int t = threadIdx.x;
    const int wave = t >> 6;
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
        const uint32_t nl = max(1u, min((uint32_t)NT, hlen / (NT >= 1024 ? PJ_MINBITS_1K : PJ_MINBITS)));
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
        // Warm-up: a range's first pass starts PJ_WARM bits before the range and decodes up to
        // it without recording, so by the range start it has usually synchronised with the
        // true token path; its first boundary >= sp is then where the previous range's path
        // crosses in, and no settle redo is needed (text: 16.6 settle rounds per segment
        // without it, the redos cascading through ranges that had not synchronised).
        uint32_t s0 = sp;
        if (r > 0 && r < nl) {
            uint32_t p = sp > PJ_WARM ? sp - PJ_WARM : 0u, pa = hs + p;
            bool ok = true;
            while (p < sp) {
                uint32_t a, d;
                const uint32_t k = pj_token(win, &pa, S.llut, S.dlut, S.T, &a, &d);
                if (k == TK_BAD || k == TK_EOB) { ok = false; break; }
                p = pa - hs;
            }
            if (ok && p < sp1) s0 = p;
        }
        uint32_t qc = s0, cc = 0;  // token boundary ccap of the first pass, its count
        uint32_t e1, cnt1 = 0, st1 = 0, nb = 0;
        {
            uint32_t p = s0, pa = hs + s0;
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
        uint32_t s = s0, e = e1, cnt = cnt1, st = st1;
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
                    bad = (j == 0 && !(A.flags & DMX_IFLAG_PIECE)) ? SEGF_EXOTIC : SEGF_XREF;
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

template <int SEG, int NT>
__global__ __launch_bounds__(NT) void k_inflate_pj(InflateArgs A) {
    __shared__ __attribute__((aligned(16))) PjSmem<SEG, NT> S;
    pj_segment<SEG, NT>(A, S, blockIdx.x);
}

// Heavy-segment patch (mode 6): the candidates listed by k_lane_caps (hl[0] = count, the
// indices from hl[2] on) are decoded by persistent workgroups, candidate hl[2 + k] by workgroup
// k mod G.
template <int SEG, int NT>
__global__ __launch_bounds__(NT) void k_inflate_pj_list(InflateArgs A, const uint32_t* hl) {
    __shared__ __attribute__((aligned(16))) PjSmem<SEG, NT> S;
    const uint32_t cnt = hl[0];
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        pj_segment<SEG, NT>(A, S, hl[2 + k]);
        __syncthreads();  // the next candidate reuses the LDS
    }
}

hipError_t launch_inflate_pj_list(const InflateArgs& A, uint32_t seg, const uint32_t* hl, uint32_t grid,
                                  hipStream_t st, hipEvent_t ev1) {
    if (seg == 16384)
        hipLaunchKernelGGL((k_inflate_pj_list<16384, 256>), dim3(grid), dim3(256), 0, st, A, hl);
    else
        hipLaunchKernelGGL((k_inflate_pj_list<32768, PJ_LIST_NT>), dim3(grid), dim3(PJ_LIST_NT), 0, st, A, hl);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
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
// Validation in two launches: k_inflate_validate_scan spreads the candidate records over the
// whole GPU and folds them into five global words (first BFINAL, first break of the chain,
// first non-uniform size, first declined candidate, declined count); k_inflate_validate
// turns them into the result.  (A single workgroup walking 32K records serially on dependent
// loads took ~38 us per call.)  The minima are kept as maxima of ~j so that the five words start
// from one zero memset (0 = none).
__global__ __launch_bounds__(256) void k_inflate_validate_scan(InflateArgs A, ValidateWords* W) {
    __shared__ unsigned long long kmin, bmin, umin, xmin, xcnt;
    const int t = threadIdx.x;
    if (t == 0) { kmin = ~0ull; bmin = ~0ull; umin = ~0ull; xmin = ~0ull; xcnt = 0; }
    __syncthreads();
    // mode 2 / 4 placed segment j at j * slot
    const uint32_t size0 = A.mode >= 2 ? A.slot : A.recs[0].out_size;
    const uint64_t j = (uint64_t)blockIdx.x * 256 + t;
    const uint64_t nc = cand_count(A);
    if (j < nc) {
        const SegRecord r = A.recs[j];
        if (r.flags & SEGF_EXOTIC) {  // the pass declined this candidate
            atomicMin(&xmin, (unsigned long long)j);
            atomicAdd(&xcnt, 1ull);
        } else {
            const bool fin = (r.flags & SEGF_FINAL) != 0;
            const bool err = (r.flags & ~SEGF_FINAL) != 0;
            const bool chain = (j + 1 < nc) && r.end_byte == A.cands[j + 1];
            if (fin) atomicMin(&kmin, (unsigned long long)j);
            if (err || (!fin && !chain)) atomicMin(&bmin, (unsigned long long)j);
            if (!fin && r.out_size != size0) atomicMin(&umin, (unsigned long long)j);
        }
    }
    __syncthreads();
    if (t == 0) {
        if (kmin != ~0ull) atomicMax(&W->kmin, ~kmin);
        if (bmin != ~0ull) atomicMax(&W->bmin, ~bmin);
        if (umin != ~0ull) atomicMax(&W->umin, ~umin);
        if (xmin != ~0ull) atomicMax(&W->xmin, ~xmin);
        if (xcnt) atomicAdd(&W->xcnt, xcnt);
    }
}

__global__ void k_inflate_validate(InflateArgs A, const ValidateWords* W, InflateResult* res) {
    auto unmax = [](unsigned long long v) -> uint64_t { return v ? ~v : ~0ull; };
    const uint64_t k = unmax(W->kmin), bmin = unmax(W->bmin), umin = unmax(W->umin), xmin = unmax(W->xmin);
    res->fin_index = (uint32_t)k;
    res->exotic = W->xcnt;
    const uint64_t nc = cand_count(A);
    if (xmin < nc) {
        res->status = 1;
        res->total = 0;
    } else if (k < nc && bmin > k) {
        if (A.mode != 1 && umin < k) {
            res->status = 1;
            res->total = 0;
        } else {
            res->status = 0;
            res->total = A.recs[k].offset + A.recs[k].out_size;
            res->end_byte = A.recs[k].end_byte;
        }
    } else {
        res->total = 0;
        res->status = 2;
    }
}

// ---------------------------------------------------------------------------------------
// serial path: the whole stream by one wavefront, realDecompress (inflate.hpp:277-322) with
// the reference's error semantics.  The stream comes through an LDS ring (RingIn: every bit
// read is an LDS read; the scalar-cache reader waited ~1000 cycles per symbol), the output
// through a 64 KiB LDS ring that holds the 32 KiB window and is written to HBM by the whole
// wave in pieces of >= 32 KiB (instead of one single-byte global store per literal).  Bytes
// past `cap` are counted, not written: the host re-runs with a larger buffer only when the
// output did not fit.
// ---------------------------------------------------------------------------------------
struct FlushSink {
    uint8_t* ring;   // 64 KiB
    uint64_t pos;    // output bytes so far
    uint64_t flushed;  // bytes [0, flushed) are in `out`
    uint8_t* out;
    uint64_t cap;
    uint32_t err;
    bool piece;  // a reference before the first byte is an error (DMX_IFLAG_PIECE)
    uint64_t* cyc;  // optional phase counters (sk_loop)
    uint8_t* flag;  // 128 zeroed bytes of LDS (sk_loop's chain marks)
    __device__ bool full() const { return false; }
    __device__ void flush() {  // [flushed, pos) ring -> out (at most 64 KiB, held by the ring)
        const uint64_t hi = pos < cap ? pos : cap;
        for (uint64_t i = flushed + lane_id(); i < hi; i += 64) out[i] = ring[i & 0xFFFF];
        flushed = pos;
    }
    __device__ void grown() {
        if (pos - flushed >= 32768) flush();
    }
    __device__ bool literal(uint32_t b) {
        if (lane_id() == 0) ring[pos & 0xFFFF] = (uint8_t)b;
        pos++;
        grown();
        return true;
    }
    __device__ bool copy(uint32_t L, uint32_t dist) {
        if (L == 0 || dist == 0) return true;
        if (dist > pos) {
            if (!piece) return true;  // reference: nothing to copy (inflate.hpp:268-270)
            err |= SEGF_XREF;
            return false;
        }
        wave_sync();
        const uint32_t lane = lane_id();
        const uint64_t src = pos - dist;
        if (dist >= L || dist >= 64) {  // each group of 64 reads only bytes written before it
            for (uint32_t i = lane; i < L; i += 64) {
                ring[(pos + i) & 0xFFFF] = ring[(src + i) & 0xFFFF];
                wave_sync();
            }
        } else {  // periodic: byte i repeats byte i mod dist
            for (uint32_t i = lane; i < L; i += 64) ring[(pos + i) & 0xFFFF] = ring[(src + i % dist) & 0xFFFF];
        }
        wave_sync();
        pos += L;
        grown();
        return true;
    }
    template <class BR>
    __device__ bool stored(const BR& br, uint64_t b0, uint32_t len) {
        flush();
        wave_sync();
        for (uint32_t i = lane_id(); i < len; i += 64) {
            const uint8_t v = br.byte_at(b0 + i);
            ring[(pos + i) & 0xFFFF] = v;
            if (pos + i < cap) out[pos + i] = v;
        }
        wave_sync();
        pos += len;
        flushed = pos;
        return true;
    }
};

// A whole Huffman block for the serial path, 64 bit offsets at a time (the way fast_header reads
// code lengths): lane i decodes the token -- literal, length + distance, end of block -- that
// would start at bit p + i; the chain of true token starts from p is walked with v_readlane (a
// few scalar instructions per token instead of a dependent table lookup); the chain's output
// offsets come from one wave scan, its literals are written by one LDS store, its matches are
// copied in order.  Semantics of decode_huffman (inflate.hpp:226-275): length symbols 286+ and
// distance symbols 30+ copy nothing, a distance reaching before the stream start copies nothing
// (an error in piece mode), a token ending past the stream is an over-read.
constexpr uint32_t SK_LIT = 0, SK_MATCH = 1, SK_EOB = 2, SK_BAD = 3;
__device__ __forceinline__ void sk_ring_copy(uint8_t* ring, uint64_t dst, uint32_t d, uint32_t L) {
    const uint32_t lane = lane_id();
    const uint64_t src = dst - d;
    if (d >= L || d >= 64) {  // each group of 64 reads only bytes written before it
        for (uint32_t i = lane; i < L; i += 64) {
            ring[(dst + i) & 0xFFFF] = ring[(src + i) & 0xFFFF];
            wave_sync();
        }
    } else {  // periodic: byte i repeats byte i mod d
        for (uint32_t i = lane; i < L; i += 64) ring[(dst + i) & 0xFFFF] = ring[(src + i % d) & 0xFFFF];
    }
    wave_sync();
}

typedef __attribute__((address_space(3))) uint32_t LdsU32;
typedef __attribute__((address_space(3))) uint8_t LdsU8;
typedef __attribute__((address_space(3))) const Tables LdsTables;
typedef __attribute__((address_space(1))) uint8_t GlbU8;
typedef __attribute__((address_space(1))) const uint32_t GlbU32;

// the token that would start at bit b: info = length in bits | kind << 8; *L = literal byte or
// match length, *d = distance (0: symbols 286+ / 30+, no copy).  Branch-free: every lane reads
// both tables; codes longer than the primary tables take one wave-uniform branch (rare).
__device__ __noinline__ void sk_slow_lit(const LdsTables* T, uint32_t v, uint32_t* e) {
    uint32_t sym, len;
    *e = slow_decode(T->lm, T->lsorted, v & 0x7FFF, LUT_L + 1, &sym, &len) ? lit_entry(sym, len) : 0u;
}
__device__ __noinline__ void sk_slow_dist(const LdsTables* T, uint32_t dv, uint32_t* de) {
    uint32_t ds, dl;
    *de = slow_decode(T->dm, T->dsorted, dv & 0x7FFF, LUT_D + 1, &ds, &dl) ? dist_entry(ds, dl) : 0u;
}
// LIN: `ring` is a plain array of stream words (sw_walk's staging), not the FB_RW ring
template <bool LIN = false>
__device__ __forceinline__ uint32_t sk_token(const LdsU32* ring, const LdsTables* T, uint32_t b, uint32_t* L,
                                             uint32_t* d) {
    const uint32_t wi = b >> 5, sh = b & 31;
    const uint32_t x0 = ring[LIN ? wi : wi % FB_RW], x1 = ring[LIN ? wi + 1 : (wi + 1) % FB_RW],
                   x2 = ring[LIN ? wi + 2 : (wi + 2) % FB_RW];
    const uint32_t v = __builtin_amdgcn_alignbit(x1, x0, sh);
    const uint64_t W = (uint64_t)v | ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32);
    uint32_t e = T->llut[v & ((1u << LUT_L) - 1)];
    if (__ballot(e == 0)) {
        if (!e) sk_slow_lit(T, v, &e);
    }
    const uint32_t cl = e & 15, ty = (e >> 4) & 3, ex = (e >> 6) & 15;
    const uint32_t q = cl + ex;
    const uint32_t dv = (uint32_t)(W >> q);
    uint32_t de = T->dlut[dv & ((1u << LUT_D) - 1)];
    const bool ism = ty == 2;
    if (__ballot(ism && de == 0)) {
        if (ism && !de) sk_slow_dist(T, dv, &de);
    }
    const uint32_t dl = de & 15, dx = (de >> 6) & 15;
    const uint32_t lenv = (e >> 16) + ((v >> cl) & ((1u << ex) - 1u));  // literal byte or match length
    *L = ty == 1 ? 0u : lenv;
    *d = ism ? (de >> 16) + ((dv >> dl) & ((1u << dx) - 1u)) : 0u;
    const uint32_t kind = !e || (ism && !de) ? SK_BAD : ty == 0 ? SK_LIT : ty == 1 ? SK_EOB : SK_MATCH;
    const uint32_t tl = ism ? q + dl + dx : cl;
    return tl | (kind << 8);
}

// sk_token for sw_walk: stream words in a plain array, wider primary tables (SW_LL / SW_LD bits,
// built per walk region) -- a walk from a wrong offset meets long codes often, and every lane of
// the wave then waits for the slow path
constexpr int SW_LL = 11, SW_LD = 10;
__device__ __forceinline__ uint32_t sw_wtok(const LdsU32* win, const LdsTables* T, const LdsU32* llut,
                                            const LdsU32* dlut, uint32_t b, uint32_t* L, uint32_t* d) {
    const uint32_t wi = b >> 5, sh = b & 31;
    const uint32_t x0 = win[wi], x1 = win[wi + 1], x2 = win[wi + 2];
    const uint32_t v = __builtin_amdgcn_alignbit(x1, x0, sh);
    const uint64_t W = (uint64_t)v | ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32);
    uint32_t e = llut[v & ((1u << SW_LL) - 1)];
    if (__ballot(e == 0)) {
        if (!e) sk_slow_lit(T, v, &e);
    }
    const uint32_t cl = e & 15, ty = (e >> 4) & 3, ex = (e >> 6) & 15;
    const uint32_t q = cl + ex;
    const uint32_t dv = (uint32_t)(W >> q);
    const bool ism = ty == 2;
    uint32_t de = dlut[dv & ((1u << SW_LD) - 1)];
    if (__ballot(ism && de == 0)) {
        if (ism && !de) sk_slow_dist(T, dv, &de);
    }
    const uint32_t dl = de & 15, dx = (de >> 6) & 15;
    const uint32_t lenv = (e >> 16) + ((v >> cl) & ((1u << ex) - 1u));
    *L = ty == 1 ? 0u : lenv;
    *d = ism ? (de >> 16) + ((dv >> dl) & ((1u << dx) - 1u)) : 0u;
    const uint32_t kind = !e || (ism && !de) ? SK_BAD : ty == 0 ? SK_LIT : ty == 1 ? SK_EOB : SK_MATCH;
    const uint32_t tl = ism ? q + dl + dx : cl;
    return tl | (kind << 8);
}

__device__ __forceinline__ void sk_copy(LdsU8* ring, uint32_t dst, uint32_t d, uint32_t L) {
    const uint32_t lane = lane_id();
    const uint32_t src = dst - d;  // (ring positions: the low 16 bits matter)
    if (d >= L || d >= 64) {  // each group of 64 reads only bytes written before it
        for (uint32_t i = lane; i < L; i += 64) {
            ring[(dst + i) & 0xFFFF] = ring[(src + i) & 0xFFFF];
            wave_sync();
        }
    } else {  // periodic: byte i repeats byte i mod d
        for (uint32_t i = lane; i < L; i += 64) ring[(dst + i) & 0xFFFF] = ring[(src + i % d) & 0xFFFF];
    }
    wave_sync();
}

struct SkState {
    uint64_t p, rb, pos, flushed;
    uint32_t err;
    uint64_t* cyc;  // optional phase counters (6)
};

// the block loop proper, out of line (its own register allocation) with explicit LDS / global
// pointers (a flat pointer would send every ring and table read through the flat path)
__device__ __attribute__((noinline)) SkState sk_loop(GlbU32* w, uint64_t nwords, uint64_t end_bytes, LdsU32* ring,
                                                     const LdsTables* T, LdsU8* oring, GlbU8* out, uint64_t cap,
                                                     SkState S, bool piece, LdsU8* flag) {
    const uint32_t lane = lane_id();
    const uint64_t endb = end_bytes * 8;
    uint64_t p = S.p, rb = S.rb, pos = S.pos, flushed = S.flushed;
    uint64_t* const cyc = S.cyc;
    const bool timed = cyc != nullptr;
    uint64_t tc = timed ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t cy[6] = {0, 0, 0, 0, 0, 0};  // (registers: a memory update per stamp would skew them)
    auto stamp = [&](int k) {
        if (timed) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            cy[k] += t1 - tc;
            tc = t1;
        }
    };
    auto flush = [&]() {
        const uint64_t hi = pos < cap ? pos : cap;
        for (uint64_t i = flushed + lane; i < hi; i += 64) out[i] = oring[i & 0xFFFF];
        flushed = pos;
    };
    for (;;) {
        // ring: words [p / 32, p / 32 + 7) (a token at p + 127 ends within 48 bits)
        const uint64_t w0 = p >> 5;
        if (w0 < rb || w0 + 10 >= rb + FB_RW) {
            rb = w0;
            for (uint64_t i = w0 + lane; i < w0 + FB_RW; i += 64) {
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
        stamp(4);
        uint32_t La, da, Lb, db;
        const uint32_t ia = sk_token(ring, T, (uint32_t)p + lane, &La, &da);       // offsets 0..63
        const uint32_t ib = sk_token(ring, T, (uint32_t)p + 64 + lane, &Lb, &db);  // offsets 64..127
        if (timed) __builtin_amdgcn_s_waitcnt(0);
        stamp(0);
        // The chain of true token starts in [0, 128), walked four tokens per step.  N1(o) = the
        // position after the token at offset o (a token that ends the block -- end of block, no
        // code -- steps by 128 + its length, past the window); N2 = N1(N1), N3 = N1(N2), N4 =
        // N2(N2), gathered across lanes with ds_bpermute (a position >= 128 stays where it is).
        // The scalar loop follows N4 from 0 and records the entries e it visits; the chain is
        // {e, N1(e), N2(e), N3(e)}, marked in parallel through an LDS flag per offset.
        const uint32_t n1a = min(lane + (ia & 255) + ((ia >> 8) >= SK_EOB ? 128u : 0u), 255u);
        const uint32_t n1b = min(64 + lane + (ib & 255) + ((ib >> 8) >= SK_EOB ? 128u : 0u), 255u);
        auto gather = [](uint32_t xa, uint32_t xb, uint32_t idx) -> uint32_t {  // X[idx], idx < 128
            const int sel = (int)((idx & 63) << 2);
            const uint32_t va = (uint32_t)__builtin_amdgcn_ds_bpermute(sel, (int)xa);
            const uint32_t vb = (uint32_t)__builtin_amdgcn_ds_bpermute(sel, (int)xb);
            return idx < 64 ? va : idx < 128 ? vb : idx;
        };
        const uint32_t n2a = gather(n1a, n1b, n1a), n2b = gather(n1a, n1b, n1b);
        const uint32_t n3a = gather(n1a, n1b, n2a), n3b = gather(n1a, n1b, n2b);
        const uint32_t n4a = gather(n2a, n2b, n2a), n4b = gather(n2a, n2b, n2b);
        uint64_t Ea = 0, Eb = 0;
        uint32_t q = 0;
        do {
            Ea |= 1ull << q;
            q = (uint32_t)__builtin_amdgcn_readlane((int)n4a, (int)q);
        } while (q < 64);
        while (q < 128) {
            Eb |= 1ull << (q - 64);
            q = (uint32_t)__builtin_amdgcn_readlane((int)n4b, (int)(q - 64));
        }
        const bool ea = (Ea >> lane) & 1ull, eb = (Eb >> lane) & 1ull;
        if (ea) {
            flag[lane] = 1;
            if (n1a < 128) flag[n1a] = 1;
            if (n2a < 128) flag[n2a] = 1;
            if (n3a < 128) flag[n3a] = 1;
        }
        if (eb) {
            flag[64 + lane] = 1;
            if (n1b < 128) flag[n1b] = 1;
            if (n2b < 128) flag[n2b] = 1;
            if (n3b < 128) flag[n3b] = 1;
        }
        wave_sync();
        const uint64_t Ma = __ballot(flag[lane] != 0), Mb = __ballot(flag[64 + lane] != 0);
        flag[lane] = 0;
        flag[64 + lane] = 0;
        // a token that ends the block: the last chain member, if its kind says so
        uint32_t stopk = SK_LIT;
        {
            const uint32_t last = Mb ? 127u - (uint32_t)__clzll(Mb) : 63u - (uint32_t)__clzll(Ma);
            const uint32_t t = last < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ia, (int)last)
                                         : (uint32_t)__builtin_amdgcn_readlane((int)ib, (int)(last - 64));
            if ((t >> 8) >= SK_EOB) {
                stopk = t >> 8;
                q = last + (t & 255);
            }
        }
        stamp(1);
        const bool ona = (Ma >> lane) & 1ull, onb = (Mb >> lane) & 1ull;
        const uint32_t ka = ia >> 8, kb = ib >> 8;
        // over-read: a chain token ending past the stream (the reference throws there); a token
        // ends within 48 bits of its start, so only the stream's last window can
        if (p + 128 + 48 > endb &&
            __ballot((ona && ka != SK_BAD && p + lane + (ia & 255) > endb) ||
                     (onb && kb != SK_BAD && p + 64 + lane + (ib & 255) > endb))) {
            S.err = SEGF_OVERREAD;
            break;
        }
        // output offsets: literals count one (mbcnt), matches their length (a scalar loop over
        // the few match lanes)
        const bool la = ona && ka == SK_LIT, lb = onb && kb == SK_LIT;
        bool ma = ona && ka == SK_MATCH && La && da, mb = onb && kb == SK_MATCH && Lb && db;
        const uint64_t mla = __ballot(la), mlb = __ballot(lb);
        uint32_t offa = __builtin_amdgcn_mbcnt_hi((uint32_t)(mla >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mla, 0u));
        uint32_t offb = __builtin_amdgcn_mbcnt_hi((uint32_t)(mlb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mlb, 0u));
        uint32_t tot = (uint32_t)__popcll(mla);
        bool xref = false;
        // (a distance reaches before the stream start only within its first 32 KiB)
        const bool early = pos < 32768;
        for (uint64_t m = __ballot(ma); m; m &= m - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            const uint32_t Lk = (uint32_t)__builtin_amdgcn_readlane((int)La, (int)k);
            if (early) {
                const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)da, (int)k);
                const uint32_t ok = (uint32_t)__builtin_amdgcn_readlane((int)offa, (int)k);
                if ((uint64_t)dk > pos + ok) {  // before the stream start: the reference copies nothing
                    xref = true;
                    if (lane == k) ma = false;
                    continue;
                }
            }
            if (lane > k) offa += Lk;
            tot += Lk;
        }
        offb += tot;
        tot += (uint32_t)__popcll(mlb);
        for (uint64_t m = __ballot(mb); m; m &= m - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            const uint32_t Lk = (uint32_t)__builtin_amdgcn_readlane((int)Lb, (int)k);
            if (early) {
                const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)db, (int)k);
                const uint32_t ok = (uint32_t)__builtin_amdgcn_readlane((int)offb, (int)k);
                if ((uint64_t)dk > pos + ok) {
                    xref = true;
                    if (lane == k) mb = false;
                    continue;
                }
            }
            if (lane > k) offb += Lk;
            tot += Lk;
        }
        if (xref && piece) {  // a piece of a larger stream: a reference before it is an error
            S.err = SEGF_XREF;
            break;
        }
        stamp(2);
        const uint32_t pos32 = (uint32_t)pos;
        if (la) oring[(pos32 + offa) & 0xFFFF] = (uint8_t)La;
        if (lb) oring[(pos32 + offb) & 0xFFFF] = (uint8_t)Lb;
        wave_sync();
        for (uint64_t m = __ballot(ma); m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            sk_copy(oring, pos32 + (uint32_t)__builtin_amdgcn_readlane((int)offa, k),
                    (uint32_t)__builtin_amdgcn_readlane((int)da, k), (uint32_t)__builtin_amdgcn_readlane((int)La, k));
        }
        for (uint64_t m = __ballot(mb); m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            sk_copy(oring, pos32 + (uint32_t)__builtin_amdgcn_readlane((int)offb, k),
                    (uint32_t)__builtin_amdgcn_readlane((int)db, k), (uint32_t)__builtin_amdgcn_readlane((int)Lb, k));
        }
        if (timed) __builtin_amdgcn_s_waitcnt(0);
        stamp(3);
        pos += tot;
        if (pos - flushed >= 32768) flush();
        cy[5]++;
        p += q;
        if (stopk == SK_BAD) {
            S.err = SEGF_ERR_DATA;
            break;
        }
        if (stopk == SK_EOB) {
            S.err = 0;
            break;
        }
    }
    if (timed && lane_id() == 0)
        for (int k = 0; k < 6; k++) cyc[k] += cy[k];
    S.p = p;
    S.rb = rb;
    S.pos = pos;
    S.flushed = flushed;
    return S;
}

__device__ uint32_t decode_block(RingIn& br, const Tables& T, FlushSink& sk) {
    SkState S{br.abspos(), br.rb, sk.pos, sk.flushed, 0, sk.cyc};
    S = sk_loop((GlbU32*)br.w, br.nwords, br.end_bytes, (LdsU32*)br.ring, (const LdsTables*)&T, (LdsU8*)sk.ring,
                (GlbU8*)sk.out, sk.cap, S, sk.piece, (LdsU8*)sk.flag);
    br.rb = S.rb;
    sk.pos = S.pos;
    sk.flushed = S.flushed;
    if (S.err) {
        sk.err |= S.err == SEGF_XREF ? SEGF_XREF : 0u;
        return S.err;
    }
    br.seek(S.p);
    return 0;
}

__global__ __launch_bounds__(IF_NT) void k_inflate_serial(InflateArgs A, int count_only,
                                                          InflateResult* res) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[65536];
    __shared__ uint32_t inring[FB_RW];
    __shared__ Tables T;
    if (threadIdx.x == 0) T.fixed_loaded = 0;
    __syncthreads();
    RingIn br;
    br.init(A.in_words, A.misalign, A.n, inring);
    br.seek(A.misalign * 8);
    __shared__ uint64_t cyc[6];
    __shared__ uint8_t flag[128];
    if (threadIdx.x < 6) cyc[threadIdx.x] = 0;
    flag[threadIdx.x] = 0;
    flag[64 + threadIdx.x] = 0;
    __syncthreads();
    FlushSink sk{ring, 0, 0, A.out, count_only ? 0 : A.cap, 0, (A.flags & DMX_IFLAG_PIECE) != 0,
                 A.dbg ? cyc : nullptr, flag};
    uint64_t end_byte = 0;
    bool fin = false;
    const uint32_t err =
        inflate_blocks(br, T, sk, (A.flags & DMX_CFG_RFC_STRICT) != 0, false, &end_byte, &fin);
    sk.flush();
    if (threadIdx.x == 0) {
        res->total = sk.pos;
        res->status = err == 0 ? 0 : (err & SEGF_OVERREAD) ? DMX_ERR_OVERREAD : DMX_ERR_DATA;
        res->fin_index = 0;
        res->end_byte = fin ? end_byte - A.misalign : 0;
    }
    if (threadIdx.x < 12) res->cycles[threadIdx.x] = threadIdx.x < 6 ? cyc[threadIdx.x] : 0ull;
}

// ---------------------------------------------------------------------------------------
// Workgroup serial decoder (k_inflate_serial_wg, the default serial path): the same
// realDecompress (inflate.hpp:277-322) and output ring as k_inflate_serial, but each Huffman
// block is decoded 2048 bit offsets at a time by 1024 threads (16 wavefronts):
//   1. every thread decodes the token that would start at two of the region's bit offsets
//      (sk_token) and its successor offset J0 (end-of-block / bad codes end a chain);
//   2. pointer doubling, J_k = J_{k-1} o J_{k-1}, up to the chain length the block's shortest
//      lit/len code allows (one barrier per level);
//   3. the chain's i-th member is J_{b_m} o .. o J_{b_0}(0) for the bits of i -- every thread
//      finds two members with no barrier in between, and the members come out in order;
//   4. one workgroup scan of their output lengths gives each token's output offset; the region
//      is cut at 16 KiB of output, at a distance reaching before the stream start (the
//      reference copies nothing there: the token is skipped; an error in piece mode) and at an
//      over-read (the reference's error, nothing of the region written);
//   5. literals and matches whose source lies before the region go to the ring in parallel
//      (short ones one thread each, long ones one wave each), then wave 0 copies the matches
//      that read the region's own output, in token order.
// Headers, stored blocks and the block loop stay on wave 0 (inflate_blocks); the other waves
// wait at the workgroup barrier and join every Huffman block (decode_block below).
// ---------------------------------------------------------------------------------------
#ifndef DMX_SW_DIAG
#define DMX_SW_DIAG 0  // developer aid: the cycle slots 0-3 count walk attempts / successes / rounds / failures
#endif
constexpr int SW_NT = 1024;
constexpr uint32_t SW_R = 2048;        // bit offsets per region
constexpr uint32_t SW_LMAX = 11;       // doubling levels for 2048 one-bit tokens
constexpr uint32_t SW_OUTCAP = 16384;  // output bytes per region (the 64 KiB ring: window + unflushed)
enum : uint32_t { SW_CMD_DECODE = 1, SW_CMD_EXIT = 2 };

// walk regions (sw_walk): one 32-bit slice of the stream per thread
constexpr uint32_t SW_WS = 64;                 // bits per slice
constexpr uint32_t SW_NS = 512;                // slices (threads that walk)
constexpr uint32_t SW_RW = SW_NS * SW_WS;      // 32768 bits per walk region
constexpr uint32_t SW_WW = SW_RW / 32 + 4;     // staged stream words
constexpr uint32_t SW_KMAX = 24;               // synchronisation rounds before the doubling fallback
constexpr uint32_t SW_WARM = 128;              // bits each slice's first walk starts before it
constexpr uint32_t SW_TERM = 1u << 31, SW_BADT = 1u << 30;
struct SwWalk {
    uint32_t win[SW_WW];                // the region's stream words
    uint32_t ex[2][SW_NS];              // each slice's exit (first token start past it; SW_TERM: a
                                        // path that ended in the slice, SW_BADT: at a bad code)
    uint16_t R[SW_OUTCAP];              // dependent output bytes: the byte they copy, + 32768
    uint32_t llut[1 << SW_LL];          // the block's codes, wider primary tables
    uint32_t dlut[1 << SW_LD];
    uint32_t cutq, cutxo, term;
};

struct SwSmem {
    uint8_t oring[65536];
    uint32_t inring[FB_RW];
    Tables T;
    union {
        struct {  // a doubling region
            uint32_t E[SW_R];               // tl | kind << 6 | L << 8 | (d & 0x7FFF) << 17
            uint16_t J[SW_LMAX][SW_R + 2];  // successors after 2^k tokens; SW_R = out of the chain
            uint16_t node[SW_R + 2];        // the chain's members in order
            uint32_t X[SW_R];               // their output offsets in the region
        };
        SwWalk W;  // a walk region
    };
    uint32_t DB[SW_R / 32];             // members whose match reads the region's own output
    uint16_t DL[SW_R];                  // those members, in order
    uint32_t PB[SW_OUTCAP / 32];        // the output bytes of those matches
    uint32_t wsum[SW_NT / 64];
    uint32_t more[3];
    uint8_t flag[128];                  // (k_inflate_serial's sk_loop marks; unused here)
    uint64_t p, pos, flushed, rb;
    uint32_t cmd, err, nmem, cut, cutx, cutov;
    uint64_t cyc[12];  // phase cycles (DMX_FB_DEBUG): sw_block's 6, then sw_walk's 5 and its rounds
};

__device__ __forceinline__ uint32_t sw_len(uint32_t e) {
    const uint32_t k = (e >> 6) & 3;
    return k == SK_LIT ? 1u : k == SK_MATCH ? (e >> 8) & 0x1FFu : 0u;
}
__device__ __forceinline__ uint32_t sw_dist(uint32_t e) {
    const uint32_t d = e >> 17;
    return d ? d : 32768u;
}

// short copy by one thread, source wholly before the destination (d >= L): reads first, then
// exact-size stores (neighbouring tokens store beside it); byte loop across the ring's end
__device__ __forceinline__ void sw_copy_short(LdsU8* ring, uint32_t dst, uint32_t d, uint32_t L) {
    const uint32_t s = (dst - d) & 0xFFFFu, o = dst & 0xFFFFu;
    if (s + 32 > 65536u || o + 32 > 65536u) {
        for (uint32_t i = 0; i < L; i++) ring[(o + i) & 0xFFFFu] = ring[(s + i) & 0xFFFFu];
        return;
    }
    typedef __attribute__((address_space(3))) uint64_t __attribute__((aligned(1))) LdsU64u;
    typedef __attribute__((address_space(3))) uint32_t __attribute__((aligned(1))) LdsU32u;
    typedef __attribute__((address_space(3))) uint16_t __attribute__((aligned(1))) LdsU16u;
    uint64_t v[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) v[k] = 8 * k < L ? *reinterpret_cast<LdsU64u*>(ring + s + 8 * k) : 0ull;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t b = 8 * k;
        if (b + 8 <= L) {
            *reinterpret_cast<LdsU64u*>(ring + o + b) = v[k];
        } else if (b < L) {
            uint32_t r = L - b, q = o + b;
            uint64_t x = v[k];
            if (r & 4) {
                *reinterpret_cast<LdsU32u*>(ring + q) = (uint32_t)x;
                q += 4;
                x >>= 32;
            }
            if (r & 2) {
                *reinterpret_cast<LdsU16u*>(ring + q) = (uint16_t)x;
                q += 2;
                x >>= 16;
            }
            if (r & 1) ring[q] = (uint8_t)x;
        }
    }
}

// Wave 0, one batch of up to 64 matches that read their region's own output (lane: have, output
// offset xo in the region, length ln, distance d), in output order: those whose source (the first
// period of a periodic one) holds no such match's output (PB) copy first, side by side; then the
// rest, one after the other.
__device__ __forceinline__ void sw_deps(LdsU8* ring, const uint32_t* PB, uint32_t pos, bool have, uint32_t xo,
                                        uint32_t ln, uint32_t d) {
    const uint32_t lane = lane_id();
    bool chained = false;
    const uint32_t a0 = xo > d ? xo - d : 0u, a1 = d >= ln ? xo - d + ln : xo;
    for (uint32_t b = a0; have && b < a1 && !chained;) {
        const uint32_t n = min(32u - (b & 31), a1 - b);
        chained = (PB[b >> 5] >> (b & 31)) & (n == 32 ? ~0u : ((1u << n) - 1u));
        b += n;
    }
    const bool freec = have && !chained;
    const bool lanec = freec && ln <= 32 && d >= ln;  // one lane copies it
    if (lanec) sw_copy_short(ring, pos + xo, d, ln);
    // then the long or periodic free ones, then the chained ones in order
    for (int pass = 0; pass < 2; pass++) {
        for (uint64_t q = __ballot(pass ? have && chained : freec && !lanec); q; q &= q - 1) {
            const int k = __builtin_ctzll(q);
            const uint32_t ko = pos + (uint32_t)__builtin_amdgcn_readlane((int)xo, k);
            const uint32_t kd = (uint32_t)__builtin_amdgcn_readlane((int)d, k);
            const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)ln, k);
            if (kd >= kl) {
                for (uint32_t b = lane; b < kl; b += 64) ring[(ko + b) & 0xFFFFu] = ring[(ko - kd + b) & 0xFFFFu];
            } else {  // periodic: byte b repeats byte b mod d of the first period
                for (uint32_t b = lane; b < kl; b += 64) ring[(ko + b) & 0xFFFFu] = ring[(ko - kd + b % kd) & 0xFFFFu];
            }
            if (pass) wave_sync();
        }
        wave_sync();
    }
}

// One walk region of SW_RW bits from stream bit p (output position pos >= 32 KiB, the region
// inside the stream): thread t < SW_NS walks the tokens of its 64-bit slice, starting SW_WARM
// bits before it (thread 0 from p); then, in rounds, every thread whose entry -- its
// predecessor's exit -- differs from the token it started at walks again from there until its
// path meets a token start of its old path (from there on the paths are the same).  When no exit
// changes, every slice holds the stream's true tokens.  A second walk sums each slice's output
// (workgroup scan: output offsets), a third writes literals and the matches whose source precedes
// the region; the bytes of the other matches are resolved by pointer jumping over the region's
// output (R[b] = b - d, then R[b] = R[R[b]]) and copied side by side.
// Returns 0 (region done: *np, *ntot), 1 (the block's end of block was in it: *np after it) or
// 2 (not converged in kmax rounds, or a bad code on the path: the caller decodes the same span
// as doubling regions, which also rewrite anything written here).
__device__ __attribute__((noinline)) uint32_t sw_walk(SwSmem& S, GlbU32* w, uint64_t nwords, uint64_t end_bytes,
                                                      uint64_t p, uint64_t pos, uint64_t* np, uint32_t* ntot,
                                                      uint32_t* rounds, bool timed, uint32_t warm, uint32_t kmax) {
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t tc = timed ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) {  // (thread 0 adds the phase to S.cyc[6 + k])
        if (timed && t == 0) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            S.cyc[6 + k] += t1 - tc;
            tc = t1;
        }
    };
    SwWalk& W = S.W;
    LdsU8* const ring = (LdsU8*)S.oring;
    const LdsTables* const T = (const LdsTables*)&S.T;
    const LdsU32* const win = (const LdsU32*)W.win;
    const uint64_t w0 = p >> 5;
    const uint32_t q0 = (uint32_t)(p & 31);
    for (uint32_t i = t; i < SW_WW; i += SW_NT) {
        uint32_t v = 0;
        if (w0 + i < nwords) {
            v = w[w0 + i];
            const uint64_t lm = end_bytes - 4 * (w0 + i);
            if (lm < 4) v &= (1u << (8 * lm)) - 1u;
        }
        W.win[i] = v;
    }
    if (t == 0) {
        W.cutq = ~0u;
        W.term = ~0u;
        S.more[0] = 0;
    }
    if (t < SW_OUTCAP / 32) S.PB[t] = 0;
    fill_lut32_wg<SW_LL, false>(W.llut, S.T.lm, S.T.lsorted, (int)t, SW_NT);
    fill_lut32_wg<SW_LD, true>(W.dlut, S.T.dm, S.T.dsorted, (int)t, SW_NT);
    const LdsU32* const wl = (const LdsU32*)W.llut;
    const LdsU32* const wd = (const LdsU32*)W.dlut;
    __syncthreads();
    const bool walker = t < SW_NS;
    const uint32_t lo = SW_WS * t, hi = walker ? lo + SW_WS : lo;
    uint32_t Lv, dv;
    // the path from en through the slice: bw = its token starts, ex = its exit
    // (the first walk starts SW_WARM bits early: by its slice's start it has most likely met
    // the stream's true tokens, so the rounds below seldom have anything to do)
    uint32_t en = ~0u, ex = ~0u;
    uint64_t bw = 0;
    {
        uint32_t q = t ? (lo >= warm ? lo - warm : 0u) : q0;
        while (q < hi) {
            if (q >= lo) {
                if (en == ~0u) en = q;
                bw |= 1ull << (q - lo);
            }
            const uint32_t info = sw_wtok(win, T, wl, wd, q, &Lv, &dv);
            const uint32_t kind = info >> 8;
            q += info & 255;
            if (kind >= SK_EOB) {
                ex = q | SW_TERM | (kind == SK_BAD ? SW_BADT : 0u);
                break;
            }
        }
        if (ex == ~0u) ex = q;
        if (en == ~0u) {
            if (ex & SW_TERM) {  // ended before the slice: (its mark is not the slice's) walk from lo
                ex = ~0u;
                bw = 0;
                en = lo;
                for (q = lo; q < hi;) {
                    bw |= 1ull << (q - lo);
                    const uint32_t info = sw_wtok(win, T, wl, wd, q, &Lv, &dv);
                    const uint32_t kind = info >> 8;
                    q += info & 255;
                    if (kind >= SK_EOB) {
                        ex = q | SW_TERM | (kind == SK_BAD ? SW_BADT : 0u);
                        break;
                    }
                }
                if (ex == ~0u) ex = q;
            } else {
                en = q;  // (a token crossed the whole slice)
            }
        }
    }
    if (walker) W.ex[0][t] = ex;
    __syncthreads();
    stamp(0);
    uint32_t cur = 0;
    bool conv = false;
    for (uint32_t k = 0; k < kmax; k++) {
        if (t == 0) S.more[(k + 1) % 3] = 0;
        bool ch = false;
        if (t > 0 && walker) {
            const uint32_t pe = W.ex[cur][t - 1];
            uint32_t nex = ex;
            // (a predecessor's path that ends -- an end of block or a bad code -- leaves this
            // slice as it is: on the true path that is the block's end, and the slice is unused)
            if (!(pe & SW_TERM) && pe != en) {
                uint32_t q = pe;
                uint64_t nb = 0;
                nex = ~0u;
                while (q < hi) {
                    if ((bw >> (q - lo)) & 1u) {  // met the old path: the same tokens from here
                        nb |= bw & (~0ull << (q - lo));
                        nex = ex;
                        break;
                    }
                    nb |= 1ull << (q - lo);
                    const uint32_t info = sw_wtok(win, T, wl, wd, q, &Lv, &dv);
                    const uint32_t kind = info >> 8;
                    q += info & 255;
                    if (kind >= SK_EOB) {
                        nex = q | SW_TERM | (kind == SK_BAD ? SW_BADT : 0u);
                        break;
                    }
                }
                if (nex == ~0u) nex = q;
                en = pe;
                bw = nb;
            }
            ch = nex != ex;
            ex = nex;
        }
        if (walker) W.ex[cur ^ 1][t] = ex;
        if (ch) S.more[k % 3] = 1;
        __syncthreads();
        cur ^= 1;
        if (!S.more[k % 3]) {
            conv = true;
            *rounds = k + 1;
            break;
        }
    }
    stamp(1);
    if (!conv) {
        *rounds = 1000u;
        return 2;
    }
    if (timed && t == 0) S.cyc[11] += *rounds;
    // the slice whose path ends the block: the first with SW_TERM (every slice before it holds
    // the true path, each starting at its predecessor's exit)
    if (walker && (ex & SW_TERM)) atomicMin(&W.term, t);
    __syncthreads();
    const uint32_t tterm = W.term;
    if (tterm != ~0u && (W.ex[cur][tterm] & SW_BADT)) return 2;  // (the doubling region reports it)
    const bool live = walker && t <= tterm;
    // output bytes of each slice
    uint32_t ol = 0;
    if (live)
        for (uint32_t q = en; q < hi;) {
            const uint32_t info = sw_wtok(win, T, wl, wd, q, &Lv, &dv);
            const uint32_t kind = info >> 8;
            q += info & 255;
            if (kind >= SK_EOB) break;
            ol += kind == SK_LIT ? 1u : (Lv && dv) ? Lv : 0u;
        }
    const uint32_t incl = wave_incl_scan(ol);
    if (lane == 63) S.wsum[wv] = incl;
    __syncthreads();
    const uint32_t wpre = wave_incl_scan(lane < SW_NT / 64 ? S.wsum[lane] : 0u);
    const uint32_t base = (wv ? (uint32_t)__builtin_amdgcn_readlane((int)wpre, (int)wv - 1) : 0u) + incl - ol;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)wpre, SW_NT / 64 - 1);
    stamp(2);
    if (t == 0) S.more[0] = 0;  // (for the dependent-byte rounds; the last read of it is behind a barrier)
    // writes
    if (live && base <= SW_OUTCAP) {  // (base == cap: the crossing token may be this slice's first)
        uint32_t xo = base;
        for (uint32_t q = en; q < hi;) {
            const uint32_t info = sw_wtok(win, T, wl, wd, q, &Lv, &dv);
            const uint32_t kind = info >> 8;
            if (kind >= SK_EOB) break;
            const uint32_t ln = kind == SK_LIT ? 1u : (Lv && dv) ? Lv : 0u;
            if (xo + ln > SW_OUTCAP) {  // (one token crosses the cap)
                W.cutq = q;
                W.cutxo = xo;
                break;
            }
            const uint32_t dst = (uint32_t)pos + xo;
            if (kind == SK_LIT) {
                ring[dst & 0xFFFFu] = (uint8_t)Lv;
            } else if (ln) {
                if (dv >= xo + ln) {  // the source precedes the region
                    for (uint32_t b = 0; b < ln; b += 32) sw_copy_short(ring, dst + b, dv, min(32u, ln - b));
                } else {  // reads the region's own output: resolved below, byte by byte
                    for (uint32_t b = xo; b < xo + ln; b++) W.R[b] = (uint16_t)(b + 32768u - dv);
                    for (uint32_t b = xo; b < xo + ln;) {
                        const uint32_t n = min(32u - (b & 31), xo + ln - b);
                        atomicOr(&S.PB[b >> 5], (n == 32 ? ~0u : ((1u << n) - 1u)) << (b & 31));
                        b += n;
                    }
                }
            }
            xo += ln;
            q += info & 255;
        }
    }
    __syncthreads();
    stamp(3);
    // dependent bytes: R[b] = R[R[b]] until every R[b] is a byte no dependent match writes (a
    // literal, a match reading before the region, or a byte before the region): the
    // reference's byte-serial copy out[b] = out[b - d], in log2(chain length) rounds
    const uint32_t cutq = W.cutq;
    const uint32_t tot = cutq != ~0u ? W.cutxo : total;
    auto dep_byte = [&](int v) -> bool { return v >= 0 && ((S.PB[(uint32_t)v >> 5] >> ((uint32_t)v & 31)) & 1u); };
    for (uint32_t r = 0;; r++) {
        if (t == 0) S.more[(r + 1) % 3] = 0;
        bool more = false;
        for (uint32_t b = t; b < tot; b += SW_NT) {
            if (!dep_byte((int)b)) continue;
            const int v = (int)W.R[b] - 32768;
            if (!dep_byte(v)) continue;
            const uint32_t w2 = W.R[v];
            W.R[b] = (uint16_t)w2;
            more |= dep_byte((int)w2 - 32768);
        }
        if (more) S.more[r % 3] = 1;
        __syncthreads();
        if (!S.more[r % 3]) break;
    }
    for (uint32_t b = t; b < tot; b += SW_NT)
        if (dep_byte((int)b)) ring[((uint32_t)pos + b) & 0xFFFFu] = ring[((uint32_t)pos + (uint32_t)W.R[b] - 32768u) & 0xFFFFu];
    stamp(4);
    uint32_t r = 0;
    if (cutq != ~0u) {
        *np = w0 * 32 + cutq;
        *ntot = W.cutxo;
    } else if (tterm != ~0u) {
        *np = w0 * 32 + (W.ex[cur][tterm] & ~(SW_TERM | SW_BADT));
        *ntot = total;
        r = 1;
    } else {
        *np = w0 * 32 + W.ex[cur][SW_NS - 1];
        *ntot = total;
    }
    __syncthreads();
    return r;
}

// One Huffman block by the whole workgroup, from S.p / S.pos / S.flushed / S.rb; results back in
// S (err, p after the block, pos, flushed, rb), published by the final barrier.
__device__ __attribute__((noinline)) void sw_block(SwSmem& S, GlbU32* w, uint64_t nwords, uint64_t end_bytes,
                                                   GlbU8* out, uint64_t cap, bool piece, bool timed, uint32_t walk) {
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t endb = end_bytes * 8;
    LdsU8* const ring = (LdsU8*)S.oring;
    const LdsTables* const T = (const LdsTables*)&S.T;
    // the shortest lit/len code bounds the chain length, hence the doubling levels
    uint32_t minb = 0;
    for (uint32_t k = 1; k < 16 && !minb; k++)
        if (S.T.lm.cnt[k]) minb = k;
    if (!minb) minb = 1;
    const uint32_t maxn = (SW_R - 1) / minb + 1;                        // chain members at most
    const uint32_t L = maxn <= 1 ? 1u : 32u - (uint32_t)__clz(maxn - 1);  // 2^L >= maxn
    const uint32_t lim = min(1u << L, SW_R);
    uint64_t p = S.p, pos = S.pos, flushed = S.flushed, rb = S.rb;
    uint32_t err = 0;
    uint64_t tc = timed ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t cy[6] = {0, 0, 0, 0, 0, 0};
    auto stamp = [&](int k) {
        if (timed && (!DMX_SW_DIAG || k >= 4)) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            cy[k] += t1 - tc;
            tc = t1;
        }
    };
    auto flush_if = [&]() {
        if (pos - flushed >= 32768) {
            const uint64_t hi = pos < cap ? pos : cap;
            for (uint64_t i = flushed + t; i < hi; i += SW_NT) out[i] = ring[i & 0xFFFF];
            flushed = pos;
        }
    };
    uint32_t wait = 0, backoff = 8;  // doubling regions before the next walk attempt
    const bool fixed = S.T.fixed_loaded != 0;
    for (;;) {
        // walk regions where they apply: past the first 32 KiB of output (no distance can reach
        // before the stream start) and SW_RW + 64 bits before the stream end (no over-read)
        // (dynamic-code blocks only: walks through fixed-code literal runs seldom resynchronise)
        if (walk && !fixed && !wait && pos >= 32768 && p + SW_RW + 64 <= endb) {
            uint64_t np = 0;
            uint32_t nt = 0, rounds = 0;
            const uint32_t r = sw_walk(S, w, nwords, end_bytes, p, pos, &np, &nt, &rounds, timed, walk & 0xFFFFu,
                                       walk >> 16);
            stamp(4);
#ifdef DMX_SW_TRACE
            if (t == 0 && pos + 40000 > DMX_SW_TRACE && pos < DMX_SW_TRACE + 1000)
                printf("walk p %llu pos %llu -> r %u np %llu nt %u rounds %u\n", (unsigned long long)p,
                       (unsigned long long)pos, r, (unsigned long long)np, nt, rounds);
#endif
#if DMX_SW_DIAG
            cy[0] += 1;                           // attempts
            cy[1] += r != 2;                      // successes
            cy[2] += rounds < 1000 ? rounds : 0;  // rounds of the converged ones
            cy[3] += rounds >= 1000;              // not converged
#endif
            if (r != 2) {
                pos += nt;
                p = np;
                flush_if();
                cy[5]++;
                backoff = 8;
                if (r == 1) break;
                continue;
            }
            // no convergence (long runs of codes that do not resynchronise, e.g. literal-only
            // fixed-code data): doubling regions for a while, longer after each failure
            wait = backoff;
            backoff = min(backoff * 2, 512u);
        }
        if (wait) wait--;
        const uint64_t w0 = p >> 5;
        if (w0 < rb || w0 + SW_R / 32 + 4 > rb + FB_RW) {  // (uniform: every thread holds p, rb)
            rb = w0;
            for (uint64_t i = w0 + t; i < w0 + FB_RW; i += SW_NT) {
                uint32_t v = 0;
                if (i < nwords) {
                    v = w[i];
                    const uint64_t lm = end_bytes - 4 * i;
                    if (lm < 4) v &= (1u << (8 * lm)) - 1u;
                }
                S.inring[i % FB_RW] = v;
            }
            __syncthreads();
        }
        if (t == 0) {
            S.cut = S.cutx = S.cutov = ~0u;
        }
        if (t < L) S.J[t][SW_R] = (uint16_t)SW_R;
        if (t < SW_R / 32) S.DB[t] = 0;
        if (t < SW_OUTCAP / 32) S.PB[t] = 0;
        // 1. tokens at every offset
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t o = t + h * SW_NT;
            uint32_t Lv, dv;
            const uint32_t info = sk_token((const LdsU32*)S.inring, T, (uint32_t)p + o, &Lv, &dv);
            const uint32_t kind = info >> 8, tl = info & 255;
            uint32_t e = min(tl, 63u) | (kind << 6);
            if (kind == SK_LIT) e |= Lv << 8;
            else if (kind == SK_MATCH && Lv && dv) e |= (Lv << 8) | ((dv & 0x7FFFu) << 17);
            S.E[o] = e;
            S.J[0][o] = (uint16_t)(kind <= SK_MATCH ? min(o + tl, SW_R) : SW_R);
        }
        __syncthreads();
        stamp(4);
        // 2. doubling
        for (uint32_t k = 1; k < L; k++) {
            const uint32_t a = S.J[k - 1][S.J[k - 1][t]], b = S.J[k - 1][S.J[k - 1][t + SW_NT]];
            S.J[k][t] = (uint16_t)a;
            S.J[k][t + SW_NT] = (uint16_t)b;
            __syncthreads();
        }
        stamp(0);
        // 3. members 2t, 2t + 1
        uint32_t x[2];
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t i = 2 * t + h;
            uint32_t v = SW_R;
            if (i < lim) {
                v = 0;
                for (uint32_t k = 0; k < L; k++) {
                    const uint32_t nv = S.J[k][v];
                    v = ((i >> k) & 1u) ? nv : v;
                }
            }
            x[h] = v;
            S.node[i] = (uint16_t)v;
        }
        if (t == 0) S.node[SW_R] = (uint16_t)SW_R;
        // 4. output offsets
        const uint32_t e0 = x[0] < SW_R ? S.E[x[0]] : 0u, e1 = x[1] < SW_R ? S.E[x[1]] : 0u;
        const uint32_t l0 = x[0] < SW_R ? sw_len(e0) : 0u, l1 = x[1] < SW_R ? sw_len(e1) : 0u;
        const uint32_t incl = wave_incl_scan(l0 + l1);
        if (lane == 63) S.wsum[wv] = incl;
        __syncthreads();
        // (the last member: the one whose successor is out of the chain)
        if (x[0] < SW_R && x[1] == SW_R) S.nmem = 2 * t + 1;
        if (x[1] < SW_R && (2 * t + 2 >= lim || S.node[2 * t + 2] == SW_R)) S.nmem = 2 * t + 2;
        const uint32_t wpre = wave_incl_scan(lane < SW_NT / 64 ? S.wsum[lane] : 0u);
        const uint32_t base = wv ? (uint32_t)__builtin_amdgcn_readlane((int)wpre, (int)wv - 1) : 0u;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)wpre, SW_NT / 64 - 1);
        const uint32_t x0 = base + incl - l0 - l1, x1 = x0 + l0;
        S.X[2 * t] = x0;
        S.X[2 * t + 1] = x1;
        // cuts: 16 KiB of output, a distance before the stream start, an over-read
        const bool near_end = p + SW_R + 48 > endb;
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t i = 2 * t + h, v = x[h];
            if (v >= SW_R) continue;
            const uint32_t e = h ? e1 : e0, ln = h ? l1 : l0, xo = h ? x1 : x0;
            if (xo + ln > SW_OUTCAP) atomicMin(&S.cut, i);
            if (ln && ((e >> 6) & 3) == SK_MATCH && sw_dist(e) > pos + xo) atomicMin(&S.cutx, i);
            if (near_end && ((e >> 6) & 3) != SK_BAD && p + v + (e & 63) > endb) atomicMin(&S.cutov, i);
        }
        __syncthreads();
        stamp(1);
        const uint32_t nmem = S.nmem, cutc = S.cut, cutx = S.cutx, cutov = S.cutov;
        const uint32_t ev = min(cutx, cutov);
        if (cutov < nmem && cutov <= cutx && cutov < cutc) {  // over-read first: the region is not written
            err = SEGF_OVERREAD;
            break;
        }
        uint32_t C = min(min(cutc, ev), nmem);  // members [0, C) are written
        const uint32_t tot = C < nmem ? S.X[C] : total;
        // where the next region starts (read now: once the region's last barrier is passed, the
        // faster waves overwrite node[] and E[] with the next region's)
        uint64_t nextp = p;
        bool done = false;
        if (C == cutc && cutc < ev && cutc < nmem) {  // 16 KiB: the next region starts at member C
            nextp += S.node[C];
        } else if (C == cutx && cutx < nmem) {  // a distance before the stream start
            if (piece) {
                err = SEGF_XREF;
                done = true;
            } else {
                const uint32_t v = S.node[C];
                nextp += v + (S.E[v] & 63);
            }
        } else {  // the chain's last member: end of block, a bad code, or past the region
            const uint32_t v = S.node[nmem - 1], e = S.E[v], kind = (e >> 6) & 3;
            nextp += v + (e & 63);
            if (kind == SK_EOB) {
                done = true;
            } else if (kind == SK_BAD) {
                err = SEGF_ERR_DATA;
                done = true;
            }
        }
        // 5. parallel writes: literals, matches whose source precedes the region.  The other
        // ("dependent") matches read the region's own output: their members are flagged in
        // S.DB and their output bytes in S.PB, for wave 0
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t i = 2 * t + h;
            const uint32_t e = h ? e1 : e0, ln = h ? l1 : l0, xo = h ? x1 : x0;
            const bool mine = i < C && ln;
            const uint32_t kind = (e >> 6) & 3;
            const uint32_t dst = (uint32_t)pos + xo;
            if (mine && kind == SK_LIT) ring[dst & 0xFFFFu] = (uint8_t)(e >> 8);
            const uint32_t d = sw_dist(e);
            const bool indep = mine && kind == SK_MATCH && d >= xo + ln;
            if (indep && ln <= 32) sw_copy_short(ring, dst, d, ln);
            if (mine && kind == SK_MATCH && !indep) {
                atomicOr(&S.DB[i >> 5], 1u << (i & 31));
                for (uint32_t b = xo; b < xo + ln;) {
                    const uint32_t n = min(32u - (b & 31), xo + ln - b);
                    atomicOr(&S.PB[b >> 5], (n == 32 ? ~0u : ((1u << n) - 1u)) << (b & 31));
                    b += n;
                }
            }
            const uint64_t m = __ballot(indep && ln > 32);
            for (uint64_t q = m; q; q &= q - 1) {  // long ones: the wave copies each, 64 bytes per step
                const int k = __builtin_ctzll(q);
                const uint32_t kd = (uint32_t)__builtin_amdgcn_readlane((int)dst, k);
                const uint32_t kdist = (uint32_t)__builtin_amdgcn_readlane((int)d, k);
                const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)ln, k);
                for (uint32_t b = lane; b < kl; b += 64) ring[(kd + b) & 0xFFFFu] = ring[(kd - kdist + b) & 0xFFFFu];
            }
        }
        __syncthreads();
        stamp(2);
        // wave 0: the dependent matches, listed in token order.  Those whose source (the first
        // period of a periodic one) holds no dependent output copy first, side by side; then
        // the rest, one after the other.
        if (wv == 0) {
            const uint32_t bits = S.DB[lane];
            const uint32_t nb = (uint32_t)__popc(bits);
            const uint32_t inc = wave_incl_scan(nb);
            const uint32_t ndep = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            uint32_t at = inc - nb;
            for (uint32_t b = bits; b; b &= b - 1) S.DL[at++] = (uint16_t)(32 * lane + (uint32_t)__builtin_ctz(b));
            wave_sync();
            for (uint32_t b0 = 0; b0 < ndep; b0 += 64) {
                uint32_t e = 0, xo = 0;
                const bool have = b0 + lane < ndep;
                if (have) {
                    const uint32_t i = S.DL[b0 + lane];
                    e = S.E[S.node[i]];
                    xo = S.X[i];
                }
                sw_deps(ring, S.PB, (uint32_t)pos, have, xo, have ? sw_len(e) : 0u, sw_dist(e));
            }
        }
        __syncthreads();
        stamp(3);
#ifdef DMX_SW_TRACE
        if (t == 0 && pos + 40000 > DMX_SW_TRACE && pos < DMX_SW_TRACE + 1000)
            printf("dbl p %llu pos %llu tot %u C %u nmem %u\n", (unsigned long long)p, (unsigned long long)pos, tot, C, nmem);
#endif
        pos += tot;
        p = nextp;
        flush_if();
        stamp(3);
        cy[5]++;
        if (done) break;
    }
    if (t == 0) {
        S.p = p;
        S.pos = pos;
        S.flushed = flushed;
        S.rb = rb;
        S.err = err;
        if (timed)
            for (int k = 0; k < 6; k++) S.cyc[k] += cy[k];
    }
    __syncthreads();
}

struct WgSink : FlushSink {
    SwSmem* S;
    uint32_t walk;  // 0: doubling regions only; else walk regions, warm-up bits | rounds << 16
    const uint32_t* words;
    uint64_t nwords, end_bytes;
};

// the Huffman blocks of k_inflate_serial_wg (found by ADL from inflate_blocks): wave 0 hands the
// state to the waiting waves and decodes the block with them
__device__ uint32_t decode_block(RingIn& br, const Tables&, WgSink& sk) {
    SwSmem& S = *sk.S;
    if (lane_id() == 0) {
        S.cmd = SW_CMD_DECODE;
        S.p = br.abspos();
        S.pos = sk.pos;
        S.flushed = sk.flushed;
        S.rb = br.rb;
    }
    __syncthreads();  // the other waves wait here (k_inflate_serial_wg)
    sw_block(S, (GlbU32*)sk.words, sk.nwords, sk.end_bytes, (GlbU8*)sk.out, sk.cap, sk.piece, sk.cyc != nullptr,
             sk.walk);
    br.rb = S.rb;
    sk.pos = S.pos;
    sk.flushed = S.flushed;
    if (S.err) {
        sk.err |= S.err == SEGF_XREF ? SEGF_XREF : 0u;
        return S.err;
    }
    br.seek(S.p);
    return 0;
}

__global__ __launch_bounds__(SW_NT) void k_inflate_serial_wg(InflateArgs A, int count_only, InflateResult* res,
                                                             int walk) {
    __shared__ __attribute__((aligned(16))) SwSmem S;
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        S.T.fixed_loaded = 0;
        S.cmd = 0;
    }
    if (t < 12) S.cyc[t] = 0;
    if (t < 128) S.flag[t] = 0;
    __syncthreads();
    if (t < 64) {  // wave 0: the block loop
        RingIn br;
        br.init(A.in_words, A.misalign, A.n, S.inring);
        br.seek(A.misalign * 8);
        WgSink sk;
        sk.ring = S.oring;
        sk.pos = 0;
        sk.flushed = 0;
        sk.out = A.out;
        sk.cap = count_only ? 0 : A.cap;
        sk.err = 0;
        sk.piece = (A.flags & DMX_IFLAG_PIECE) != 0;
        sk.cyc = A.dbg ? S.cyc : nullptr;
        sk.flag = S.flag;
        sk.S = &S;
        sk.walk = (uint32_t)walk;
        sk.words = A.in_words;
        sk.end_bytes = A.misalign + A.n;
        sk.nwords = (sk.end_bytes + 3) / 4;
        uint64_t end_byte = 0;
        bool fin = false;
        const uint32_t err = inflate_blocks(br, S.T, sk, (A.flags & DMX_CFG_RFC_STRICT) != 0, false, &end_byte, &fin);
        sk.flush();
        if (t == 0) {
            res->total = sk.pos;
            res->status = err == 0 ? 0 : (err & SEGF_OVERREAD) ? DMX_ERR_OVERREAD : DMX_ERR_DATA;
            res->fin_index = 0;
            res->end_byte = fin ? end_byte - A.misalign : 0;
            S.cmd = SW_CMD_EXIT;
        }
        if (t < 12) res->cycles[t] = S.cyc[t];
        __syncthreads();  // releases the other waves
    } else {
        for (;;) {
            __syncthreads();  // wave 0 publishes a command
            if (S.cmd == SW_CMD_EXIT) break;
            sw_block(S, (GlbU32*)A.in_words, (A.misalign + A.n + 3) / 4, A.misalign + A.n, (GlbU8*)A.out,
                     count_only ? 0 : A.cap, (A.flags & DMX_IFLAG_PIECE) != 0, A.dbg != nullptr, (uint32_t)walk);
        }
    }
}

// ---------------------------------------------------------------------------------------
// dmx_segment_check_device: for each given start, the one segment that begins there, decoded
// by the exact wave decoder in piece mode (no reference before the start, <= 64 KiB of
// output: libdmx's 32 KiB segments and C4's 64 KiB blocks); ends[i] = the stream byte after its
// closing empty stored block (or after its BFINAL block), ~0 when it does not decode.
// Validates multi-GPU cut points (shard.py).
// ---------------------------------------------------------------------------------------
constexpr uint32_t CHECK_CAP = 65536;
__global__ __launch_bounds__(IF_NT) void k_segment_check(InflateArgs A, const uint64_t* starts, uint64_t k,
                                                         uint64_t* ends) {
    __shared__ __attribute__((aligned(16))) uint8_t win[CHECK_CAP + 16];
    __shared__ Tables T;
    const uint64_t i = blockIdx.x;
    if (i >= k) return;
    if (threadIdx.x == 0) T.fixed_loaded = 0;
    __syncthreads();
    const uint64_t start = starts[i];
    uint64_t end = ~0ull;
    if (start < A.n) {
        SegSink sk{win, 0, false, 0, CHECK_CAP};
        BitIn br;
        br.init(A.in_words, A.misalign, A.n);
        br.seek((A.misalign + start) * 8);
        uint64_t end_byte = 0;
        bool fin = false;
        const uint32_t err = inflate_blocks(br, T, sk, (A.flags & DMX_CFG_RFC_STRICT) != 0, true, &end_byte, &fin);
        if (!err) end = end_byte - A.misalign;
    }
    if (threadIdx.x == 0) ends[i] = end;
}

hipError_t launch_segment_check(const InflateArgs& A, const uint64_t* starts, uint64_t k, uint64_t* ends,
                                hipStream_t st) {
    if (k) hipLaunchKernelGGL(k_segment_check, dim3((uint32_t)k), dim3(IF_NT), 0, st, A, starts, k, ends);
    return hipGetLastError();
}

hipError_t launch_inflate_segments(const InflateArgs& A, hipStream_t st, hipEvent_t ev0,
                                   hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, st);
    hipLaunchKernelGGL(k_inflate_segments, dim3((uint32_t)A.ncand), dim3(IF_NT), 0, st, A);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

__global__ void k_async_prep(const uint64_t* nmarkers, uint64_t* ncand) { *ncand = *nmarkers + 1; }
// status 0 only when the lane pass decoded the whole chain up to BFINAL, every candidate fit the
// provisioned scratch and the output fits cap; anything else is the general path's (the caller's
// synchronous dmx_inflate_device)
__global__ void k_async_result(const InflateResult* res, const uint64_t* ncand, uint64_t cand_cap, uint64_t cap,
                               uint64_t* d_result) {
    const bool ok = res->status == 0 && *ncand <= cand_cap && res->total <= cap;
    d_result[0] = ok ? res->total : 0;
    d_result[1] = ok ? 0 : 1;
}
hipError_t launch_async_prep(const uint64_t* nmarkers, uint64_t* ncand, hipStream_t st) {
    hipLaunchKernelGGL(k_async_prep, dim3(1), dim3(1), 0, st, nmarkers, ncand);
    return hipGetLastError();
}
hipError_t launch_async_result(const InflateResult* res, const uint64_t* ncand, uint64_t cand_cap, uint64_t cap,
                               uint64_t* d_result, hipStream_t st) {
    hipLaunchKernelGGL(k_async_result, dim3(1), dim3(1), 0, st, res, ncand, cand_cap, cap, d_result);
    return hipGetLastError();
}

hipError_t launch_inflate_validate(const InflateArgs& A, ValidateWords* W, InflateResult* res,
                                   hipStream_t st) {
    hipError_t e = hipMemsetAsync(W, 0, sizeof(ValidateWords), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_inflate_validate_scan, dim3((uint32_t)((A.ncand + 255) / 256)), dim3(256), 0, st, A, W);
    hipLaunchKernelGGL(k_inflate_validate, dim3(1), dim3(1), 0, st, A, (const ValidateWords*)W, res);
    return hipGetLastError();
}

hipError_t launch_inflate_serial(const InflateArgs& A, int count_only, InflateResult* res,
                                 hipStream_t st) {
    // DMX_SERIAL_WAVE=1: the one-wavefront decoder (developer A/B)
    static const bool one_wave = [] {
        const char* e = std::getenv("DMX_SERIAL_WAVE");
        return e && *e == '1';
    }();
    // DMX_SERIAL_WALK=0: doubling regions only; DMX_SERIAL_WARM / DMX_SERIAL_ROUNDS: the walk's
    // warm-up bits and synchronisation rounds (developer A/B)
    static const int walk = [] {
        const char* e = std::getenv("DMX_SERIAL_WALK");
        if (e && *e == '0') return 0;
        const char* w = std::getenv("DMX_SERIAL_WARM");
        const char* k = std::getenv("DMX_SERIAL_ROUNDS");
        const int warm = w && *w ? std::atoi(w) : (int)SW_WARM;
        const int kmax = k && *k ? std::atoi(k) : (int)SW_KMAX;
        return (warm & 0xFFFF) | (kmax << 16);
    }();
    if (!one_wave) {
        hipLaunchKernelGGL(k_inflate_serial_wg, dim3(1), dim3(SW_NT), 0, st, A, count_only, res, walk);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_inflate_serial, dim3(1), dim3(IF_NT), 0, st, A, count_only, res);
    return hipGetLastError();
}

}  // namespace dmx
