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

constexpr uint32_t FB_SCAN_BITS = 32768;  // bit offsets tested per wavefront (4 KiB of stream)
constexpr uint32_t FB_STAGE_WORDS = FB_SCAN_BITS / 32 + 128;  // + 4096 bits of header lookahead
constexpr uint32_t FB_HITS = 12;          // hits kept per scan chunk (stored headers in zero
                                          // padding are found at several offsets)
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

// Full check of a candidate whose precode is complete.  pl: 19 precode lengths (3 bits each,
// by symbol).  p: bit position (in the staged image) of the first code-length symbol.
// RFC 1951 rules as zlib's inflate enforces them; A-11/A-12 streams are not block starts any
// real encoder writes, so rejecting them only costs parallelism.
__device__ bool fb_check_lengths(const uint32_t* w, uint32_t p, uint64_t pl, uint32_t nlit,
                                 uint32_t ndist, uint32_t plim) {
    // canonical precode decoder "by counts": cnt[l] in 5-bit fields, symbols sorted by
    // (length, value) in 5-bit fields of two words
    uint64_t cnt = 0, sa = 0, sb = 0;
    uint32_t ns = 0;
    for (uint32_t l = 1; l <= 7; l++) {
        for (uint32_t s = 0; s < 19; s++) {
            if (((pl >> (3 * s)) & 7) == l) {
                if (ns < 12) sa |= (uint64_t)s << (5 * ns);
                else sb |= (uint64_t)s << (5 * (ns - 12));
                ns++;
                cnt += 1ull << (5 * l);
            }
        }
    }
    const uint32_t total = nlit + ndist;
    uint32_t i = 0, prev = 0;
    uint32_t kl = 0, kd = 0, nd = 0;  // Kraft sums in units of 2^-15, used distance codes
    bool eob = false;
    while (i < total) {
        if (p > plim) return false;  // longer than any header a real encoder writes
        const uint32_t v = fb_bits(w, p);
        // decode one precode symbol MSB-first from the bit-reversed stream order
        uint32_t code = 0, first = 0, index = 0, sym = 0xFF, len = 0;
        for (uint32_t l = 1; l <= 7; l++) {
            code |= (v >> (l - 1)) & 1u;
            const uint32_t c = (uint32_t)(cnt >> (5 * l)) & 31;
            if (code - first < c) {
                const uint32_t k = index + code - first;
                sym = (uint32_t)((k < 12 ? sa >> (5 * k) : sb >> (5 * (k - 12))) & 31);
                len = l;
                break;
            }
            index += c;
            first = (first + c) << 1;
            code <<= 1;
        }
        if (sym == 0xFF) return false;
        p += len;
        uint32_t val = sym, run = 1;
        if (sym == 16) {
            if (i == 0) return false;
            val = prev;
            run = 3 + ((v >> len) & 3);
            p += 2;
        } else if (sym == 17) {
            val = 0;
            run = 3 + ((v >> len) & 7);
            p += 3;
        } else if (sym == 18) {
            val = 0;
            run = 11 + ((v >> len) & 127);
            p += 7;
        }
        if (i + run > total) return false;
        if (val) {
            // lengths [i, i + run): split at nlit
            const uint32_t a = i < nlit ? min(i + run, nlit) - i : 0;
            const uint32_t b = run - a;
            kl += a << (15 - val);
            kd += b << (15 - val);
            nd += b;
            if (i <= 256 && 256 < i + a) eob = true;
            if (kl > 32768 || kd > 32768) return false;
        }
        prev = val;
        i += run;
    }
    return eob && kl == 32768 && (kd == 32768 || nd <= 1);
}

__global__ __launch_bounds__(64) void k_fb_scan(const uint32_t* in_words, uint64_t misalign,
                                                 uint64_t n, uint32_t* counts, uint64_t* hits) {
    __shared__ uint32_t stg[FB_STAGE_WORDS + 2];
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
    uint32_t found = 0;
    for (uint32_t it = 0; it < FB_SCAN_BITS / 64 && found < FB_HITS; it++) {
        const uint32_t r = it * 64 + lane;  // offset tested by this lane, relative to b0
        const uint64_t sb = b0 + r;         // stream bit
        bool hit = false, stored = false;
        if (sb + 17 + 12 < nbits) {
            const uint32_t q = sh + r;      // staged-image bit
            const uint32_t h = fb_bits(stg, q);
            if (((h >> 1) & 3) == 0) {
                // stored block: LEN and NLEN = ~LEN at the next byte boundary, data inside the
                // stream (zlib writes these for incompressible runs; without them a unit ending
                // before a stored block had no unit to continue the chain).  A header in zero
                // padding is found at several offsets; the chain takes the one the unit before
                // ends at, the others only cost parallelism.
                const uint64_t bb = (sb + 3 + 7) & ~7ull;  // stream bit of LEN
                if (bb + 32 <= nbits) {
                    const uint32_t ln = fb_bits(stg, q + (uint32_t)(bb - sb));
                    hit = stored = ((ln ^ (ln >> 16)) & 0xFFFFu) == 0xFFFFu && bb / 8 + 4 + (ln & 0xFFFFu) <= n;
                }
            }
            const uint32_t hlit = (h >> 3) & 31, hdist = (h >> 8) & 31, hclen = ((h >> 13) & 15) + 4;
            if (((h >> 1) & 3) == 2 && hlit <= 29 && hdist <= 29) {
                const uint32_t x0 = fb_bits(stg, q + 17), x1 = fb_bits(stg, q + 49);
                const uint64_t x = (uint64_t)x0 | ((uint64_t)x1 << 32);
                uint64_t pl = 0;
                uint32_t kr = 0, lastl = 0;
                for (uint32_t i = 0; i < 19; i++) {
                    if (i < hclen) {
                        const uint32_t l = (uint32_t)(x >> (3 * i)) & 7;
                        pl |= (uint64_t)l << (3 * kPerm[i]);
                        kr += l ? 128u >> l : 0u;
                        lastl = l;
                    }
                }
                // zlib / libdeflate / libdmx send HCLEN up to the last nonzero length (>= 4)
                if (kr == 128 && (lastl != 0 || hclen == 4))
                    hit = fb_check_lengths(stg, q + 17 + 3 * hclen, pl, hlit + 257, hdist + 1,
                                           (FB_STAGE_WORDS - 1) * 32);
            }
        }
        const uint64_t m = __ballot(hit);
        if (m) {
            const uint32_t before = __popcll(m & ((1ull << lane) - 1ull));
            if (hit && found + before < FB_HITS)
                hits[c * FB_HITS + found + before] = sb | (stored ? FB_HIT_STORED : 0ull);
            found += __popcll(m);
        }
    }
    if (lane == 0) counts[c] = min(found, FB_HITS);
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


// Wave-uniform bit reader over a sliding LDS ring of the stream (k_fb_decode).  BitIn reads
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
};
struct RingWords {
    const uint32_t* ring;
    __device__ uint32_t word(uint64_t i) const { return ring[i % FB_RW]; }
};
__device__ __forceinline__ RingWords reader_words(const RingIn& br) { return RingWords{br.ring}; }

__global__ __launch_bounds__(64) void k_fb_decode(const uint32_t* in_words, uint64_t misalign,
                                                   uint64_t n, const uint64_t* starts,
                                                   const uint64_t* stops, uint64_t nunits,
                                                   const uint64_t* tokoff, uint32_t* tok,
                                                   FbUnit* units, uint32_t flags) {
    __shared__ Tables T;
    __shared__ uint32_t ring[FB_RW];
    const uint64_t u = blockIdx.x;
    if (u >= nunits) return;
    if (lane_id() == 0) T.fixed_loaded = 0;
    wave_sync();
    const uint64_t start = starts[u];
    // A unit ends after the first block that lands exactly on another unit's start, or that
    // passes the next dynamic-header start (stored-header starts can be false: passing one
    // inside a block is no reason to stop, landing on one is a chain link).
    // A unit at a stored-header start (bit 63 of its stop) decodes stored blocks only and ends
    // before the first other block: such a start can be false, and a false one then costs one
    // bounded copy instead of a run of Huffman decoding over arbitrary bits.
    const bool weak = (stops[u] >> 63) != 0;
    const uint64_t stop = stops[u] & ~(1ull << 63);
    uint64_t jn = u + 1;  // first unit start not below the current position
    uint64_t end_at = 0;  // (weak units) stream bit of the first block they leave undecoded
    const uint64_t base = misalign * 8;  // stream bit 0 in the aligned image
    RingIn br;
    br.init(in_words, misalign, n, ring);
    br.seek(base + start);
    TokSink sk;
    sk.tk = tok + tokoff[u];
    sk.cap = (uint32_t)(tokoff[u + 1] - tokoff[u]);
    sk.n = sk.k = sk.reg = sk.pend = sk.pendn = 0;
    sk.pos = 0;
    sk.unit_byte0 = (base + start) >> 3;
    sk.stream_start = u == 0 && !(flags & DMX_IFLAG_PIECE);
    sk.err = 0;
    const bool rfc = (flags & DMX_CFG_RFC_STRICT) != 0;
    uint32_t err = 0;
    bool fin = false;
    // realDecompress (inflate.hpp:277-322) until the next unit's start or BFINAL
    for (bool first = true;; first = false) {
        if (!first) {
            const uint64_t pos = br.abspos() - base;
            if (pos >= stop) break;
            while (jn < nunits && starts[jn] < pos) jn++;
            if (jn < nunits && starts[jn] == pos) break;
        }
        const uint64_t hpos = br.abspos();
        br.ensure(3);
        const uint32_t bfinal = br.bits(1);
        const uint32_t btype = br.bits(2);
        if (br.over()) { err = SEGF_OVERREAD; break; }
        if (weak && btype != 0) {
            end_at = hpos;
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
            err = decode_huffman(br, T, sk);
            if (err) break;
        } else if (btype == 2) {
            T.fixed_loaded = 0;
            uint64_t hp = br.abspos();
            err = fast_header(reader_words(br), &hp, br.end_bits, T, rfc, true);
            if (err) break;
            br.seek(hp);
            err = decode_huffman(br, T, sk);
            if (err) break;
        }  // BTYPE 3: an empty block (inflate.hpp:292 has no case 3)
        if (bfinal) {
            fin = true;
            break;
        }
    }
    if (!err && !sk.finish()) err = sk.err;
    if (lane_id() == 0) {
        FbUnit r;
        r.start = start;
        r.end = (end_at ? end_at : br.abspos()) - base;
        r.size = sk.pos;
        r.ntok = sk.n;
        r.flags = err | (fin ? SEGF_FINAL : 0u);
        units[u] = r;
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
    while (t0 < n) {
        const uint32_t ti = t0 + lane;
        const uint32_t w = ti < n ? tk[ti] : 0u;
        // the word after a stored header is its offset (any 32-bit value, bit 31 included):
        // lane ti - 1 is that header
        const uint32_t wprev = (uint32_t)__shfl((int)w, (int)lane - 1, 64);
        const uint32_t wp = lane == 0 ? (t0 > 0 ? tk[t0 - 1] : 0u) : wprev;
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
            const uint32_t so = tk[t0 + 1];
            const uint8_t* src = A.stream + byte0 + so;
            for (uint32_t p0 = 0; p0 < len; p0 += FB_GROUP_MAX) {
                const uint32_t m = min(FB_GROUP_MAX, len - p0);
                for (uint32_t i = lane; i < m; i += 64) ring[(pos + p0 + i) & (FB_RING - 1)] = src[p0 + i];
                wave_sync();
                for (uint32_t i = lane; i < m; i += 64) img[pos + p0 + i] = ring[(pos + p0 + i) & (FB_RING - 1)];
                wave_sync();
            }
            pos += len;
            t0 += 2;
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
                const uint32_t so = tk[t0 + k + 1];
                const uint8_t* src = A.stream + byte0 + so;
                for (uint32_t i = lane; i < Lk; i += 64) ring[(dst + i) & (FB_RING - 1)] = src[i];
            }
            wave_sync();
        }
        // 4. the group's entries to the image
        for (uint32_t i = lane; i < T; i += 64) img[pos + i] = ring[(pos + i) & (FB_RING - 1)];
        wave_sync();
        pos += T;
        t0 += ntk;
    }
    if (__ballot(bad) && lane == 0) atomicOr(A.err, 1u);
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
// k_fb_final: every entry before its unit's tail.  One workgroup per FB_FIN_SPAN entries; the
// unit of the span's first entry is found by binary search over the chain offsets.
// ---------------------------------------------------------------------------------------
constexpr uint32_t FB_FIN_SPAN = 16384;
__global__ __launch_bounds__(256) void k_fb_final(const uint16_t* img, const uint64_t* offs,
                                                  const uint64_t* sizes, uint64_t nchain,
                                                  uint64_t total, uint8_t* out) {
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
    for (uint64_t x = s0 + threadIdx.x; x < s1; x += 256) {
        while (x >= uend) {
            k++;
            uoff = offs[k];
            uend = uoff + sizes[k];
        }
        const uint64_t s = uend - uoff;
        if (x - uoff >= s - min(s, (uint64_t)FB_RING)) continue;  // tail: k_fb_tails wrote it
        const uint32_t v = img[x];
        const uint64_t b = (v & 0x7FFFu) + 1;  // a marker before the stream start was flagged
        out[x] = v < 0x8000u ? (uint8_t)v : (b <= uoff ? out[uoff - b] : (uint8_t)0);
    }
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

hipError_t launch_fb_compact(const uint32_t* counts, const uint64_t* offs, const uint64_t* hits,
                             uint64_t nchunks, uint64_t* list, hipStream_t st) {
    hipLaunchKernelGGL(k_fb_compact, dim3((uint32_t)((nchunks + 255) / 256)), dim3(256), 0, st,
                       counts, offs, hits, nchunks, list);
    return hipGetLastError();
}

hipError_t launch_fb_decode(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                            const uint64_t* starts, const uint64_t* stops, uint64_t nunits,
                            const uint64_t* tokoff, uint32_t* tok, FbUnit* units, uint32_t flags,
                            hipStream_t st) {
    hipLaunchKernelGGL(k_fb_decode, dim3((uint32_t)nunits), dim3(64), 0, st, in_words, misalign, n,
                       starts, stops, nunits, tokoff, tok, units, flags);
    return hipGetLastError();
}

hipError_t launch_fb_resolve(const uint8_t* stream, const uint64_t* starts, const uint32_t* chain,
                             const uint64_t* offs, const uint64_t* sizes, uint64_t nchain,
                             const uint64_t* tokoff, const uint32_t* tok, const FbUnit* units,
                             uint16_t* img, uint64_t total, uint8_t* out, uint32_t* err,
                             hipStream_t st) {
    FbReplayArgs R{stream, starts, chain, offs, tokoff, tok, units, img, err};
    hipLaunchKernelGGL(k_fb_replay, dim3((uint32_t)nchain), dim3(64), 0, st, R);
    hipLaunchKernelGGL(k_fb_tails, dim3(1), dim3(FB_TNT), 0, st, img, offs, sizes, nchain, out);
    const uint64_t nb = (total + FB_FIN_SPAN - 1) / FB_FIN_SPAN;
    if (nb) hipLaunchKernelGGL(k_fb_final, dim3((uint32_t)nb), dim3(256), 0, st, img, offs, sizes, nchain, total, out);
    return hipGetLastError();
}

}  // namespace dmx
