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
constexpr int SEG_CAP = 32768;
constexpr int LUT_L = 10;  // primary lit/len lookup bits
constexpr int LUT_D = 8;   // primary distance lookup bits

struct TreeMeta {
    uint32_t lo[16], hi[16], cnt[16], offs[16];
};

struct Tables {
    uint16_t llut[1 << LUT_L];
    uint16_t dlut[1 << LUT_D];
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

    __device__ void init(const uint32_t* words, uint64_t misalign, uint64_t n) {
        w = words;
        end_bytes = misalign + n;
        end_bits = end_bytes * 8;
        nwords = (end_bytes + 3) / 4;
    }
    // Unconditional load with a clamped index (no branch, so the wait lands at first use).
    // The decoder state is wave-uniform, so the input is read through the scalar cache
    // (s_load, constant address space): a vector load would be waited on immediately to move
    // its value into an SGPR, defeating the two-word prefetch.
    __device__ uint32_t raw(uint64_t i) const {
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

// primary LUT over PB bits: entry = sym | (len << 9), 0 = no code of length <= PB matches
template <int PB>
__device__ void fill_lut(uint16_t* lut, const TreeMeta& m, const uint16_t* sorted) {
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
        lut[wv] = len ? (uint16_t)(sorted[idx] | (len << 9)) : (uint16_t)0;
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
    fill_lut<LUT_L>(T.llut, T.lm, T.lsorted);
    fill_lut<LUT_D>(T.dlut, T.dm, T.dsorted);
    wave_sync();
}

// code-length sequence(s) (inflate.hpp:166-206).  Reference mode: called once per sequence,
// last literal length starts at 0, a repeat may overshoot (entries keep their index as the
// symbol value).  RFC mode: one call over both sequences (nb > 0).  Returns SEGF_* or 0 and
// the number of entries written to a (and b).
__device__ uint32_t read_code_lengths(BitIn& br, const Tables& T, uint8_t* a, uint32_t na,
                                      uint8_t* b, uint32_t nb, bool rfc, uint32_t* outa,
                                      uint32_t* outb) {
    const int lane = lane_id();
    const uint32_t total = na + nb;
    const uint32_t cap = rfc ? total : 300;
    uint32_t i = 0, last = 0;
    while (i < total) {
        br.ensure(14);
        const uint16_t e = T.plut[br.peek(7)];
        if (!e) return SEGF_ERR_DATA;
        br.consume(e >> 9);
        const uint32_t s = e & 511;
        uint32_t rep, val;
        if (s == 16) {
            if (rfc && i == 0) return SEGF_ERR_DATA;
            rep = 3 + br.bits(2);
            val = last;
        } else if (s == 17) {
            rep = 3 + br.bits(3);
            val = 0;
        } else if (s == 18) {
            rep = 11 + br.bits(7);
            val = 0;
        } else {
            rep = 1;
            val = s;
        }
        if (rfc || s < 16) last = val;
        if (br.over()) return SEGF_OVERREAD;
        if (i + rep > cap) {
            if (rfc || val != 0) return SEGF_ERR_DATA;  // reference: value >= 300 is UB
        }
        for (uint32_t j = lane; j < rep; j += 64) {
            const uint32_t idx = i + j;
            if (idx < cap) {
                if (!rfc || idx < na) a[idx] = (uint8_t)val;  // reference: overshoot entries
                else b[idx - na] = (uint8_t)val;               // keep their index as value
            }
        }
        i += rep;
    }
    wave_sync();
    if (!rfc) {
        *outa = min(i, 300u);
        *outb = 0;
    } else {
        *outa = na;
        *outb = nb;
    }
    return 0;
}

__device__ uint32_t read_dynamic_header(BitIn& br, Tables& T, bool rfc) {
    const int lane = lane_id();
    br.ensure(14);
    const uint32_t hlit = br.bits(5), hdist = br.bits(5), hclen = br.bits(4);
    if (lane < 32) T.plen[lane] = 0;
    wave_sync();
    for (uint32_t i = 0; i < hclen + 4; i++) {
        const uint32_t v = br.bits(3);
        if (lane == 0) T.plen[kPerm[i]] = (uint8_t)v;
    }
    if (br.over()) return SEGF_OVERREAD;
    wave_sync();
    build_tree(T.plen, 19, T.psorted, T.pm);
    fill_prelut(T.plut, T.pm, T.psorted);
    wave_sync();
    uint32_t nl, nd, err;
    if (!rfc) {
        uint32_t dummy;
        err = read_code_lengths(br, T, T.llen, 257 + hlit, nullptr, 0, false, &nl, &dummy);
        if (err) return err;
        err = read_code_lengths(br, T, T.dlen, 1 + hdist, nullptr, 0, false, &nd, &dummy);
        if (err) return err;
    } else {
        err = read_code_lengths(br, T, T.llen, 257 + hlit, T.dlen, 1 + hdist, true, &nl, &nd);
        if (err) return err;
    }
    build_tree(T.llen, nl, T.lsorted, T.lm);
    build_tree(T.dlen, nd, T.dsorted, T.dm);
    fill_lut<LUT_L>(T.llut, T.lm, T.lsorted);
    fill_lut<LUT_D>(T.dlut, T.dm, T.dsorted);
    wave_sync();
    return 0;
}

// periodic LZ77 copy: out[pos + i] = out[pos - dist + (i mod dist)], i < L (equal to the
// reference's byte-serial overlapping copy, inflate.hpp:268-270); every source byte lies
// before pos, so all lanes copy independently.
template <uint32_t MASK>
__device__ __forceinline__ void lz_copy_lds(uint8_t* win, uint32_t pos, uint32_t L, uint32_t dist) {
    const uint32_t lane = lane_id();
    const uint32_t src = pos - dist;
    if (dist >= L) {
        for (uint32_t i = lane; i < L; i += 64) win[(pos + i) & MASK] = win[(src + i) & MASK];
    } else {
        uint32_t r = dist >= 64 ? lane : lane % dist;
        const uint32_t step = dist >= 64 ? 64 : 64 % dist;
        for (uint32_t i = lane; i < L; i += 64) {
            win[(pos + i) & MASK] = win[(src + r) & MASK];
            r += step;
            if (r >= dist) r -= dist;
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
    __device__ bool stored(const BitIn& br, uint64_t b0, uint32_t len) {
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
    __device__ bool stored(const BitIn& br, uint64_t b0, uint32_t len) {
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

// decompressHuffmanBlock (inflate.hpp:226-275) with table lookups
template <class Sink>
__device__ uint32_t decode_huffman(BitIn& br, const Tables& T, Sink& sk) {
    for (;;) {
        br.ensure(20);
        uint32_t v = br.peek(15);
        uint32_t e = T.llut[v & ((1u << LUT_L) - 1)];
        uint32_t sym, len;
        if (e) {
            sym = e & 511;
            len = e >> 9;
        } else if (!slow_decode(T.lm, T.lsorted, v, LUT_L + 1, &sym, &len)) {
            return SEGF_ERR_DATA;
        }
        br.consume(len);
        if (sym < 256) {
            if (br.over()) return SEGF_OVERREAD;
            if (!sk.literal(sym)) return sk.err;
            continue;
        }
        if (sym == 256) return br.over() ? SEGF_OVERREAD : 0;
        uint32_t L = 0;
        if (sym <= 285) {
            const uint32_t ex = len_extra(sym);
            L = len_base(sym) + (ex ? br.bits(ex) : 0);
        }
        br.ensure(28);
        v = br.peek(15);
        e = T.dlut[v & ((1u << LUT_D) - 1)];
        uint32_t ds, dl;
        if (e) {
            ds = e & 511;
            dl = e >> 9;
        } else if (!slow_decode(T.dm, T.dsorted, v, LUT_D + 1, &ds, &dl)) {
            return SEGF_ERR_DATA;
        }
        br.consume(dl);
        uint32_t dist = 0;
        if (ds < 30) {
            const uint32_t ex = dist_extra(ds);
            dist = dist_base(ds) + (ex ? br.bits(ex) : 0);
        }
        if (br.over()) return SEGF_OVERREAD;
        if (!sk.copy(L, dist)) return sk.err;
    }
}

// realDecompress (inflate.hpp:277-322).  With stop_at_marker the segment ends at an empty,
// non-final stored block whose NLEN is FFFF (the "00 00 FF FF" the scanner keyed on).
template <class Sink>
__device__ uint32_t inflate_blocks(BitIn& br, Tables& T, Sink& sk, bool rfc, bool stop_at_marker,
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
            const uint64_t b0 = br.pos >> 3;
            if (stop_at_marker && !bfinal && len == 0 && nlen == 0xFFFF) {
                *end_byte = b0;
                return 0;
            }
            if (b0 + len > br.end_bytes) return SEGF_OVERREAD;
            if (!sk.stored(br, b0, len)) return sk.err;
            br.seek(br.pos + 8ull * len);
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
            uint32_t err = read_dynamic_header(br, T, rfc);
            if (hdr_cycles) *hdr_cycles += __builtin_amdgcn_s_memtime() - h0;
            if (err) return err;
            err = decode_huffman(br, T, sk);
            if (err) return err;
        }  // btype 3: no-op block (inflate.hpp:292 has no case 3)
        if (bfinal) {
            *fin = true;
            *end_byte = (br.pos + 7) >> 3;
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
    __shared__ unsigned long long s_j, s_excl;
    const int lane = threadIdx.x;
    // dynamic segment index: workgroups that start earlier take earlier segments, so a
    // look-back only ever waits on a workgroup that is already running
    if (lane == 0) s_j = atomicAdd(A.ticket, 1u);
    if (lane == 0) T.fixed_loaded = 0;
    __syncthreads();
    const uint64_t j = s_j;
    if (j >= A.ncand) return;
    DMX_PHASE(A.dbg, j, 0);
    const uint64_t start = A.cands[j];
    uint64_t hdr_cycles = 0;

    BitIn br;
    br.init(A.in_words, A.misalign, A.n);
    br.seek((A.misalign + start) * 8);
    SegSink sk{win, 0, j == 0, 0};
    uint64_t end_byte = 0;
    bool fin = false;
    uint32_t err = inflate_blocks(br, T, sk, (A.flags & DMX_CFG_RFC_STRICT) != 0, true, &end_byte, &fin,
                                  A.dbg ? &hdr_cycles : nullptr);
    const uint32_t size = err ? 0 : sk.pos;
    DMX_PHASE(A.dbg, j, 1);
    if (A.dbg && lane_id() == 0) A.dbg[j * kPhaseSlots + 8] = hdr_cycles;

    if (lane == 0) {
        uint64_t excl = 0;
        if (A.mode == 0) {
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
// k_inflate_pj: one workgroup of PJ_NT lanes per candidate segment.
//   1. wave 0 reads the block header (wave-uniform, as above) into shared tables;
//   2. the segment's Huffman bits are split into PJ_NT equal ranges; lane t decodes tokens
//      from the start of its range (an arbitrary bit: Huffman decoding self-synchronises
//      within a few tokens) until its path crosses into the next range, keeping the first
//      PJ_K token boundaries it passed;
//   3. settle: lane t restarts where lane t-1's path left its range and decodes until it
//      reaches a boundary of its own first path (merged: the rest of its count is known) --
//      repeated until every range starts where the previous one ended (normally one round);
//   4. exclusive scan of the per-lane output counts, then every lane re-decodes its range and
//      writes P[x] for each output byte x: 0x8000 | byte for a literal, or the position the
//      byte is copied from (LZ77 copy out[o + i] = out[o - d + (i mod d)], always < x);
//   5. pointer jumping P[x] = P[P[x]] until every entry is a literal (chains halve per round);
//   6. the low bytes of P go to HBM with 16-byte stores at the segment's slot j * 32768.
// Everything else -- several blocks in one segment, stored + Huffman mixes, an output above
// 32 KiB, a split that does not settle -- is flagged SEGF_EXOTIC and the whole stream is
// redone by k_inflate_segments, so results never depend on this path's coverage.
// ---------------------------------------------------------------------------------------
constexpr int PJ_NT = 256;
constexpr int PJ_K = 8;
constexpr uint32_t PJ_LIT = 0x8000u;
constexpr uint32_t PJ_MAXBITS = 1u << 20;  // Huffman bits of one segment (32 KiB * 15 < 2^19)
constexpr int PJ_ROUNDS = 16;
constexpr uint32_t PJ_MINBITS = 256;

// LSB-first bit reader whose position differs per lane: plain (vector) loads
struct LBits {
    const uint32_t* w;
    uint64_t nwords, end_bytes;
    uint64_t pos;
    uint64_t buf;
    uint32_t cnt;
    uint64_t wi;
    uint32_t q0, q1;

    __device__ void init(const uint32_t* words, uint64_t misalign, uint64_t n) {
        w = words;
        end_bytes = misalign + n;
        nwords = (end_bytes + 3) / 4;
    }
    __device__ uint32_t raw(uint64_t i) const { return w[i < nwords ? i : nwords - 1]; }
    __device__ uint32_t mask(uint64_t i) const {
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
    __device__ void ensure(uint32_t k) {
        if (cnt < k) refill();
    }
    __device__ uint32_t peek(uint32_t k) const { return (uint32_t)buf & ((1u << k) - 1u); }
    __device__ void consume(uint32_t k) {
        buf >>= k;
        cnt -= k;
        pos += k;
    }
    __device__ uint32_t bits(uint32_t k) {
        ensure(k);
        const uint32_t v = peek(k);
        consume(k);
        return v;
    }
};

enum : uint32_t { TK_LIT = 0, TK_MATCH = 1, TK_EOB = 2, TK_BAD = 3 };

// one token of decompressHuffmanBlock (inflate.hpp:226-275): a literal (*a = byte), a match
// (*a = length, *d = distance; 0 for symbols 286+ / 30+), the end of block, or no code
__device__ __forceinline__ uint32_t pj_token(LBits& br, const Tables& T, uint32_t* a, uint32_t* d) {
    br.ensure(20);
    uint32_t v = br.peek(15);
    uint32_t e = T.llut[v & ((1u << LUT_L) - 1)];
    uint32_t sym, len;
    if (e) {
        sym = e & 511;
        len = e >> 9;
    } else if (!slow_decode(T.lm, T.lsorted, v, LUT_L + 1, &sym, &len)) {
        return TK_BAD;
    }
    br.consume(len);
    if (sym < 256) {
        *a = sym;
        return TK_LIT;
    }
    if (sym == 256) return TK_EOB;
    uint32_t L = 0;
    if (sym <= 285) {
        const uint32_t ex = len_extra(sym);
        L = len_base(sym) + (ex ? br.bits(ex) : 0);
    }
    br.ensure(28);
    v = br.peek(15);
    e = T.dlut[v & ((1u << LUT_D) - 1)];
    uint32_t ds, dl;
    if (e) {
        ds = e & 511;
        dl = e >> 9;
    } else if (!slow_decode(T.dm, T.dsorted, v, LUT_D + 1, &ds, &dl)) {
        return TK_BAD;
    }
    br.consume(dl);
    uint32_t dist = 0;
    if (ds < 30) {
        const uint32_t ex = dist_extra(ds);
        dist = dist_base(ds) + (ex ? br.bits(ex) : 0);
    }
    *a = L;
    *d = dist;
    return TK_MATCH;
}

__device__ __forceinline__ uint32_t tok_bytes(uint32_t k, uint32_t a, uint32_t d) {
    return k == TK_LIT ? 1u : (k == TK_MATCH && a && d) ? a : 0u;
}

struct PjSmem {
    uint16_t P[SEG_CAP];
    Tables T;
    uint32_t endp[PJ_NT];   // where lane t's current path crossed into range t+1 (relative)
    uint32_t part[PJ_NT / 64];
    uint64_t hs;            // absolute bit of the first Huffman token
    uint32_t hlen;          // bits split among the lanes
    uint32_t kind;          // 0 Huffman, 1 stored, 2 done (empty segment / error)
    uint32_t bfinal;
    uint32_t err;
    uint32_t slen;
    uint64_t sb0;
    uint32_t tew[PJ_NT / 64];  // per wave: first lane whose path ends (EOB / no code)
    uint32_t total;
    uint64_t end_byte;
};

__global__ __launch_bounds__(PJ_NT) void k_inflate_pj(InflateArgs A) {
    __shared__ __attribute__((aligned(16))) PjSmem S;
    const int t = threadIdx.x;
    const int wave = t >> 6;
    const uint64_t j = blockIdx.x;
    const bool rfc = (A.flags & DMX_CFG_RFC_STRICT) != 0;
    const uint64_t obase = j * (uint64_t)SEG_CAP;
    DMX_PHASE(A.dbg, j, 0);

    // ---- 1. block header (wave 0) ----
    if (wave == 0) {
        BitIn br;
        br.init(A.in_words, A.misalign, A.n);
        br.seek((A.misalign + A.cands[j]) * 8);
        br.ensure(3);
        const uint32_t bfinal = br.bits(1);
        const uint32_t btype = br.bits(2);
        uint32_t kind = 2, err = 0;
        uint64_t end_byte = 0, sb0 = 0;
        uint32_t slen = 0, hlen = 0;
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
            if (btype == 1) {
                load_fixed(S.T);
            } else {
                err = read_dynamic_header(br, S.T, rfc);
            }
            if (!err) {
                const uint64_t hs = br.pos;
                const uint64_t he = j + 1 < A.ncand ? (A.misalign + A.cands[j + 1] - 4) * 8 - 3
                                                    : (A.misalign + A.n) * 8;
                if (he <= hs || he - hs > PJ_MAXBITS) {
                    err = SEGF_EXOTIC;
                } else {
                    kind = 0;
                    hlen = (uint32_t)(he - hs);
                }
                if (lane_id() == 0) S.hs = hs;
            }
        }
        if (lane_id() == 0) {
            S.kind = err ? 2 : kind;
            S.err = err;
            S.bfinal = bfinal;
            S.end_byte = end_byte;
            S.slen = slen;
            S.sb0 = sb0;
            S.hlen = hlen;
            S.total = kind == 1 ? slen : 0;
        }
    }
    __syncthreads();
    DMX_PHASE(A.dbg, j, 1);
    const uint32_t kind = S.kind;

    if (kind == 1) {
        // ---- stored segment: bytes straight to the slot ----
        const uint32_t len = S.slen;
        if (len > SEG_CAP) {
            if (t == 0) S.err = SEGF_OVERFLOW;
        } else {
            const uint64_t b0 = S.sb0;
            const uint8_t* src = reinterpret_cast<const uint8_t*>(A.in_words);
            for (uint32_t i = t; i < len; i += PJ_NT)
                if (obase + i < A.cap) A.out[obase + i] = src[b0 + i];
        }
    } else if (kind == 0) {
        // ---- 2. first pass over the lane ranges ----
        const uint64_t hs = S.hs;
        const uint32_t hlen = S.hlen;
        // ranges of at least PJ_MINBITS (a few dozen tokens) so that a path started at an
        // arbitrary bit re-synchronises inside its own range; surplus lanes stay empty
        const uint32_t nl = max(1u, min((uint32_t)PJ_NT, hlen / PJ_MINBITS));
        const uint32_t sp = t < (int)nl ? (uint32_t)(((uint64_t)hlen * t) / nl) : hlen;
        const uint32_t sp1 = t + 1 < (int)nl ? (uint32_t)(((uint64_t)hlen * (t + 1)) / nl) : hlen;
        LBits br;
        br.init(A.in_words, A.misalign, A.n);
        uint32_t q[PJ_K], c[PJ_K];
#pragma unroll
        for (int k = 0; k < PJ_K; k++) q[k] = c[k] = 0xFFFFFFFFu;
        uint32_t e1, cnt1 = 0, st1 = 0, nb = 0;
        {
            br.seek(hs + sp);
            uint32_t p = sp;
            while (p < sp1) {
                uint32_t a, d;
                const uint32_t k = pj_token(br, S.T, &a, &d);
                if (k == TK_BAD) { st1 = 2; break; }
                p = (uint32_t)(br.pos - hs);
                if (k == TK_EOB) { st1 = 1; break; }
                cnt1 += tok_bytes(k, a, d);
                if (nb < PJ_K) {
#pragma unroll
                    for (int m = 0; m < PJ_K; m++)
                        if (m == (int)nb) { q[m] = p; c[m] = cnt1; }
                    nb++;
                }
            }
            e1 = p;
        }
        // ---- 3. settle the range starts ----
        // per round: [publish end, first-ending lane per wave] | read: te, want | or-barrier |
        // redo | barrier.  Every shared word is written and read on opposite sides of a barrier.
        uint32_t s = sp, e = e1, cnt = cnt1, st = st1;
        uint32_t te = PJ_NT;
        bool settled = false;
        for (int round = 0; round <= PJ_ROUNDS; round++) {
            S.endp[t] = e;
            {
                const uint64_t bm = __ballot(st != 0);
                if ((t & 63) == 0) S.tew[wave] = bm ? (uint32_t)(wave * 64 + __ffsll((long long)bm) - 1) : PJ_NT;
            }
            __syncthreads();
            te = min(min(S.tew[0], S.tew[1]), min(S.tew[2], S.tew[3]));
            const uint32_t want = t == 0 ? 0 : S.endp[t - 1];
            const bool redo = t > 0 && t <= (int)te && want != s;
            if (!__syncthreads_or(redo)) {
                settled = true;
                break;
            }
            if (round == PJ_ROUNDS) break;
            if (redo) {
                // decode from the true start until the path meets a boundary of the first pass
                s = want;
                uint32_t p = want, acc = 0, stn = 0;
                bool merged = false;
                br.seek(hs + p);
                for (;;) {
                    if (p == sp) {
                        merged = true;
                        cnt = acc + cnt1;
                    }
#pragma unroll
                    for (int m = 0; m < PJ_K; m++)
                        if (!merged && p == q[m]) {
                            merged = true;
                            cnt = acc + cnt1 - c[m];
                        }
                    if (merged || p >= sp1) break;
                    uint32_t a, d;
                    const uint32_t k = pj_token(br, S.T, &a, &d);
                    if (k == TK_BAD) { stn = 2; break; }
                    p = (uint32_t)(br.pos - hs);
                    if (k == TK_EOB) { stn = 1; break; }
                    acc += tok_bytes(k, a, d);
                }
                if (merged) {
                    e = e1;
                    st = st1;
                } else {
                    e = p;
                    cnt = acc;
                    st = stn;
                }
            }
            __syncthreads();
        }
        if (t == 0 && !settled) S.err |= SEGF_EXOTIC;
        if (t == (int)te) {
            if (st == 2) {
                S.err |= SEGF_ERR_DATA;
            } else {
                // end of block: BFINAL ends the stream, else the marker block must follow
                const uint64_t pe = hs + e;
                if (S.bfinal) {
                    S.end_byte = (pe + 7) >> 3;
                } else {
                    br.seek(pe);
                    const uint32_t h3 = br.bits(3);
                    const uint64_t m = (pe + 3 + 7) >> 3;
                    const uint8_t* src = reinterpret_cast<const uint8_t*>(A.in_words);
                    if (h3 == 0 && m + 4 <= A.misalign + A.n && src[m] == 0 && src[m + 1] == 0 &&
                        src[m + 2] == 0xFF && src[m + 3] == 0xFF)
                        S.end_byte = m + 4;
                    else
                        S.err |= SEGF_EXOTIC;
                }
            }
        }
        // no end of block before the split end: several blocks, or the next candidate is not
        // this segment's end
        if (te >= PJ_NT && t == 0) S.err |= SEGF_EXOTIC;
        const uint32_t mycnt = t <= (int)te ? cnt : 0u;
        // ---- 4. scan + emit ----
        const uint32_t inc = wave_incl_scan(mycnt);
        if ((t & 63) == 63) S.part[wave] = inc;
        __syncthreads();
        uint32_t base = 0;
        for (int w = 0; w < wave; w++) base += S.part[w];
        const uint32_t total = S.part[0] + S.part[1] + S.part[2] + S.part[3];
        if (t == 0) {
            S.total = total;
            if (total > SEG_CAP) S.err |= SEGF_OVERFLOW;
        }
        __syncthreads();
        if (!S.err && t <= (int)te && mycnt) {
            uint32_t o = base + inc - mycnt;
            br.seek(hs + s);
            uint32_t p = s;
            uint32_t bad = 0;
            while (p < sp1) {
                uint32_t a, d;
                const uint32_t k = pj_token(br, S.T, &a, &d);
                p = (uint32_t)(br.pos - hs);
                if (k == TK_LIT) {
                    S.P[o++] = (uint16_t)(PJ_LIT | a);
                } else if (k == TK_MATCH) {
                    if (!a || !d) continue;
                    if (d > o) {  // before the segment: cross-segment or stream-start reference
                        bad = j == 0 ? SEGF_EXOTIC : SEGF_XREF;
                        break;
                    }
                    uint32_t src = o - d, r = 0;
                    for (uint32_t i = 0; i < a; i++) {
                        S.P[o + i] = (uint16_t)(src + r);
                        if (++r == d) r = 0;
                    }
                    o += a;
                } else {
                    break;
                }
            }
            if (bad) atomicOr(&S.err, bad);
        }
        __syncthreads();
        DMX_PHASE(A.dbg, j, 2);
        // ---- 5. pointer jumping ----
        if (!S.err) {
            uint32_t* P2 = reinterpret_cast<uint32_t*>(S.P);
            const uint32_t npair = (total + 1) / 2;
            bool open = true;
            for (int round = 0; round < 24 && open; round++) {
                uint32_t any = 0;
                for (uint32_t i = t; i < npair; i += PJ_NT) {
                    const uint32_t v = P2[i];
                    uint32_t lo = v & 0xFFFF, hi = v >> 16;
                    const bool plo = !(lo & PJ_LIT), phi = !(hi & PJ_LIT) && 2 * i + 1 < total;
                    if (plo | phi) {
                        if (plo) lo = S.P[lo];
                        if (phi) hi = S.P[hi];
                        if (phi) S.P[2 * i + 1] = (uint16_t)hi;
                        if (plo) S.P[2 * i] = (uint16_t)lo;
                        any |= (plo && !(lo & PJ_LIT)) || (phi && !(hi & PJ_LIT));
                    }
                }
                open = __syncthreads_or(any) != 0;
            }
            if (open && t == 0) S.err |= SEGF_EXOTIC;
            __syncthreads();
        }
        DMX_PHASE(A.dbg, j, 3);
        // ---- 6. low bytes of P to the slot ----
        if (!S.err) {
            const uint32_t nb16 = total / 16;
            uint8_t* dst = A.out + obase;
            const bool vec = (((uintptr_t)dst) & 15) == 0 && obase + total <= A.cap;
            const uint4* P4 = reinterpret_cast<const uint4*>(S.P);
            if (vec) {
                for (uint32_t i = t; i < nb16; i += PJ_NT) {
                    const uint4 a = P4[2 * i], b = P4[2 * i + 1];
                    uint4 o;
                    o.x = __builtin_amdgcn_perm(a.y, a.x, 0x06040200u);
                    o.y = __builtin_amdgcn_perm(a.w, a.z, 0x06040200u);
                    o.z = __builtin_amdgcn_perm(b.y, b.x, 0x06040200u);
                    o.w = __builtin_amdgcn_perm(b.w, b.z, 0x06040200u);
                    reinterpret_cast<uint4*>(dst)[i] = o;
                }
                for (uint32_t i = nb16 * 16 + t; i < total; i += PJ_NT) dst[i] = (uint8_t)S.P[i];
            } else {
                for (uint32_t i = t; i < total; i += PJ_NT)
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
    DMX_PHASE(A.dbg, j, 4);
}

hipError_t launch_inflate_pj(const InflateArgs& A, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, st);
    hipLaunchKernelGGL(k_inflate_pj, dim3((uint32_t)A.ncand), dim3(PJ_NT), 0, st, A);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// Candidate chain check.  Valid iff, up to the first BFINAL segment k, every segment decoded
// without error and ended exactly at the next candidate.  Speculative mode additionally needs
// every segment before k to have segment 0's size (else status 1: re-run with look-back).
__global__ __launch_bounds__(1024) void k_inflate_validate(InflateArgs A, InflateResult* res) {
    __shared__ unsigned long long kmin, bmin, umin, xmin;
    const int t = threadIdx.x;
    if (t == 0) { kmin = ~0ull; bmin = ~0ull; umin = ~0ull; xmin = ~0ull; }
    __syncthreads();
    // mode 2 (k_inflate_lanes) placed segment j at j * 32768
    const uint32_t size0 = A.mode == 2 ? 32768u : A.recs[0].out_size;
    for (uint64_t j = t; j < A.ncand; j += 1024) {
        const SegRecord r = A.recs[j];
        if (r.flags & SEGF_EXOTIC) {  // k_inflate_pj declined this candidate
            atomicMin(&xmin, (unsigned long long)j);
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
