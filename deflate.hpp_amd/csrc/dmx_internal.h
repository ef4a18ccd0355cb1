// dmx_internal.h -- kernel launch interfaces shared by the host runtime and the .hip files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmx {

struct DeflateArgs {
    const uint8_t* in;
    uint64_t n;
    uint64_t nseg;
    int level;
    int final_last;       // set BFINAL on the last segment
    uint8_t* slots;       // nseg * slot_bytes scratch: each segment's bitstream
    uint32_t slot_bytes;
    uint32_t* tok;        // nseg * tok_stride words: the front kernel's token words (levels 2-3)
    uint32_t tok_stride;  // words per segment (a multiple of 4), deflate_tok_stride(segment bytes)
    uint32_t* ntok;       // nseg token word counts
    uint32_t* sizes;      // nseg
    uint64_t* offsets;    // nseg
    uint64_t* total;      // 1
    uint8_t* out;
    uint64_t cap;
    uint64_t* dbg;        // optional per-block phase timestamps (DMX_PHASES), else nullptr
};

// Token words per segment of the front kernel: a literal word covers 1-3 input bytes, a match
// word at least 3, so at most seg / 2 words (one literal between every two 3-byte matches), plus
// one partial literal word per thread's token range (1024 threads); the last kDeflateHistWords
// words hold the segment's symbol histogram (320 counts as u16 pairs: lit/len symbols at 0..287,
// distance symbols at 288..319, end of block not counted), which the emission kernel reads.
constexpr uint32_t kDeflateHistWords = 160;
constexpr uint32_t deflate_tok_stride(uint32_t seg) { return seg / 2 + 1024 + 64 + kDeflateHistWords; }

hipError_t launch_deflate(const DeflateArgs& A, uint32_t seg_bytes, hipStream_t st, hipEvent_t ev0,
                          hipEvent_t ev1);

// per-candidate record of the segment-parallel inflate
struct SegRecord {
    uint64_t end_byte;  // byte offset (relative to the stream) just past the segment's marker
    uint64_t offset;    // output offset the segment was written at
    uint32_t out_size;
    uint32_t flags;     // SEGF_*
};
enum : uint32_t {
    SEGF_FINAL = 1u,      // the segment ended with a BFINAL block
    SEGF_ERR_DATA = 2u,   // undecodable code / table
    SEGF_OVERREAD = 4u,   // ran past the end of the input
    SEGF_OVERFLOW = 8u,   // output exceeded the LDS window
    SEGF_XREF = 16u,      // back-reference reaches before the segment start
    SEGF_TIMEOUT = 32u,   // look-back spin bound hit
    SEGF_EXOTIC = 64u,    // layout the workgroup decoder does not take (several blocks, > 32 KiB,
                          // unsettled split): the wave-per-segment decoder redoes the stream
};

// InflateArgs::flags bit (internal): the stream is a piece of a larger stream (multi-GPU
// scatter): a back-reference before its first byte is an error, not the stream-start no-op.
constexpr uint32_t DMX_IFLAG_PIECE = 1u << 31;

struct InflateArgs {
    const uint32_t* in_words;  // 4-byte aligned base at or below the stream start
    uint64_t misalign;         // stream start = in_words bytes + misalign
    uint64_t n;                // stream bytes
    const uint64_t* cands;     // candidate segment starts (bytes, relative to stream)
    uint64_t ncand;
    uint8_t* out;
    uint64_t cap;
    SegRecord* recs;
    unsigned long long* status;  // ncand look-back words (zeroed)
    unsigned int* ticket;        // zeroed
    uint32_t flags;              // DMX_CFG_RFC_STRICT, DMX_IFLAG_PIECE
    uint32_t mode;               // 0 = speculative uniform segment sizes, 1 = decoupled look-back,
                                 // 2 = k_inflate_pj (segment j at j * slot),
                                 // 3 = k_inflate_segments redoing only SEGF_EXOTIC candidates
                                 //     of a mode-2 / mode-4 pass, at the same slots,
                                 // 4 = k_inflate_lanes + k_inflate_resolve (segment j at j * slot),
                                 // 6 = k_inflate_pj_list patching the heavy candidates of mode 4
    uint32_t slot;               // mode 2: segment bytes (16384 or 32768)
    uint64_t* dbg;               // optional per-segment phase timestamps (DMX_PHASES)
    // dmx_inflate_device_async: the candidate count lives on the device (<= ncand, which is then
    // the capacity the grids are sized for); nullptr: ncand is the count
    const uint64_t* ncand_dev = nullptr;
};
// the candidate count a kernel works on
__device__ __forceinline__ uint64_t cand_count(const InflateArgs& A) {
    return A.ncand_dev ? (*A.ncand_dev < A.ncand ? *A.ncand_dev : A.ncand) : A.ncand;
}

constexpr int kPhaseSlots = 16;
#define DMX_PHASE(dbg, idx, slot)                                                   \
    do {                                                                            \
        if ((dbg) && threadIdx.x == 0) (dbg)[(idx) * kPhaseSlots + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// result of validation / serial decode, copied to the host
struct InflateResult {
    uint64_t total;   // decoded bytes
    int32_t status;   // fast path: 0 ok, 1 re-run with look-back, 2 serial; serial: 0 / DMX_ERR_*
    uint32_t fin_index;
    uint64_t exotic;  // candidates flagged SEGF_EXOTIC by the pass
    uint64_t end_byte;  // status 0: the stream byte just past the final block (relative to the stream)
    uint64_t cycles[12];  // serial decoder (DMX_FB_DEBUG): s_memtime per phase -- decode, walk,
                         // offsets, literals + copies, flush + refill, steps
};

hipError_t launch_marker_count(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                               uint32_t* tile_counts, uint64_t ntiles, hipStream_t st);
// cands holds cand_cap entries: candidates past them are not written (the async inflate sizes
// its scratch before the count is known)
hipError_t launch_marker_write(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                               const uint64_t* tile_offs, uint64_t ntiles, uint64_t* cands,
                               uint64_t cand_cap, hipStream_t st);
// dmx_inflate_device_async: *ncand = min(nmarkers + 1, ...) on the device; the result words
// {decoded bytes, status} from the validation (status 0: decoded; 1: needs the general path)
hipError_t launch_async_prep(const uint64_t* nmarkers, uint64_t* ncand, hipStream_t st);
hipError_t launch_async_result(const InflateResult* res, const uint64_t* ncand, uint64_t cand_cap, uint64_t cap,
                               uint64_t* d_result, hipStream_t st);
uint64_t marker_tiles(uint64_t n, uint64_t misalign);
// exclusive scan of n values into offs (64-bit) and *total; offs must hold scan_words(n)
// entries (the block sums of the multi-workgroup scan follow the n offsets)
uint64_t scan_words(uint64_t n);
hipError_t launch_scan_u32(const uint32_t* v, uint64_t* offs, uint64_t n, uint64_t* total,
                           hipStream_t st);
hipError_t launch_inflate_segments(const InflateArgs& A, hipStream_t st, hipEvent_t ev0,
                                   hipEvent_t ev1);
// workgroup-per-segment decoder (lane-parallel Huffman decode + pointer-jumping LZ77);
// segment j lands at j * 32768 (mode 2)
hipError_t launch_inflate_pj(const InflateArgs& A, uint32_t seg, hipStream_t st, hipEvent_t ev0,
                             hipEvent_t ev1);
// lane-per-segment Huffman decode (k_inflate_lanes) + wave-per-segment LZ77 resolve
// (k_inflate_resolve); segment j lands at j * A.slot (mode 4).  tok holds
// min(ncand * 16404, 8 * n + 20 * ncand) words; tokoff ncand + 1, ntok / caps ncand entries.
// heavy != 0: when at most `limit` candidates span more than `heavy` bytes (counted on the
// device into hl[1]), those are declined and listed in hl (hl[0] = count, the indices from
// hl[2] on; ncand + 2 words) for launch_inflate_pj_list.
// split: ncand words when A.slot is 64 KiB (the halves' split), else unused
hipError_t launch_inflate_lanes(const InflateArgs& A, uint32_t* tok, uint64_t* tokoff,
                                uint32_t* ntok, uint32_t* caps, uint32_t heavy, uint32_t limit,
                                uint32_t* hl, uint32_t* split, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1);
// mode 6: the workgroup decoder over the candidates listed in hl, `grid` persistent workgroups
hipError_t launch_inflate_pj_list(const InflateArgs& A, uint32_t seg, const uint32_t* hl, uint32_t grid,
                                  hipStream_t st, hipEvent_t ev1);
// validation scratch: five device words, zeroed by the launch
struct ValidateWords {
    unsigned long long kmin, bmin, umin, xmin, xcnt;
};
hipError_t launch_inflate_validate(const InflateArgs& A, ValidateWords* W, InflateResult* res,
                                   hipStream_t st);

// block-parallel inflate of arbitrary streams (inflate_blocks.hip, path 5)
struct FbUnit {         // per-unit record written by k_fb_pdecode / k_fb_decode
    uint64_t start;     // stream bit of the unit's first token (a block header, or a token
                        // boundary inside a block: region and repair units)
    uint64_t end;       // stream bit where it stopped: past its last block, or (soft stop) the
                        // first token boundary at or past its stop
    uint64_t size;      // output bytes
    uint64_t hdr;       // state at `end`: FB_AT_HEADER, else the code in force (FB_STATE_*)
    uint32_t ntok;      // token words
    uint32_t flags;     // SEGF_*
};
// Units and their stops (path 5).  stops[u]: the stream bit where unit u ends, with
constexpr uint64_t FB_STOP_WEAK = 1ull << 63;  // a stored-header (weak) unit
constexpr uint64_t FB_STOP_SOFT = 1ull << 62;  // the next unit starts inside a block: end at the
                                               // first token boundary at or past the stop
constexpr uint64_t FB_STOP_REGION = 1ull << 61;  // the head of a long gap between dynamic-header
                                                 // starts: a first block that is not dynamic ends
                                                 // the unit at once (the region map decodes the run)
constexpr uint64_t FB_STOP_MASK = FB_STOP_REGION - 1;
// A code state (FbUnit.hdr, the per-unit vhdr): the stream bit of the dynamic block header whose
// code is in force, or FB_STATE_FIXED for the fixed code; FB_STATE_FINAL: that block has BFINAL.
constexpr uint64_t FB_STATE_FIXED = 1ull << 62;
constexpr uint64_t FB_STATE_FINAL = 1ull << 61;
constexpr uint64_t FB_STATE_POS = FB_STATE_FINAL - 1;
constexpr uint64_t FB_AT_HEADER = ~0ull;       // the unit ended at a block header
// how a unit starts (vmode)
enum : uint8_t {
    FB_V_HEADER = 0,   // at a block header (bit 0, a scanned dynamic or stored header)
    FB_V_EXACT = 2,    // exactly at its start bit inside a block whose code is vhdr (a repair)
};
constexpr uint32_t SEGF_SOFT = 1u << 30;  // internal: decode_huffman reached the soft stop
// FbUnit flag (not an error): the unit's decode passed at least one block header after its
// start (diagnostics)
constexpr uint32_t SEGF_CROSSED = 1u << 29;
constexpr uint32_t SEGF_ERRORS = ~(SEGF_FINAL | SEGF_CROSSED);
uint64_t fb_scan_chunks(uint64_t n);
uint32_t fb_hits_per_chunk();
// header scan of every bit offset: counts[nchunks], hits[nchunks * fb_hits_per_chunk()],
// offs = exclusive scan of counts, *nhits = total
hipError_t launch_fb_scan(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                          uint32_t* counts, uint64_t* hits, uint64_t* offs, uint64_t* nhits,
                          hipStream_t st);
// compacts the scan's candidates into one sorted list of count entries and runs the full header
// test on them (k_fb_check): a candidate that fails it gets FB_HIT_REJECT.  *pcount: the
// candidates (device), max_count: the most there can be (sizes the grids).  keep (host memory
// mapped into the device, or nullptr): the accepted starts, unordered, *nkeep of them (entries
// past keep_cap dropped).  ph: DMX_FB_DEBUG counters (or nullptr)
constexpr uint64_t FB_HIT_REJECT = 1ull << 63;
hipError_t launch_fb_compact(const uint32_t* in_words, uint64_t misalign, uint64_t n, const uint32_t* counts,
                             const uint64_t* offs, const uint64_t* hits, uint64_t nchunks, uint64_t* list,
                             const uint64_t* pcount, uint64_t max_count, unsigned long long* ph, uint64_t* keep,
                             uint32_t* nkeep, uint32_t keep_cap, hipStream_t st);
// hits carry bit 62 for a stored-block header; stops[u] = the next dynamic-header start after u
// units [u0, u0 + count) of the nunits listed; vmode / vhdr as above
// fixed-code regions (k_fb_smap + k_fb_swalk): reg = nreg x {E, T, first super block}, sbreg =
// the region of each of the nsb super blocks, J = nsb * fb_region_nodes() words, visit = nsb
// words (the node the path enters each super block at, ~0 = none: region chunk << 6 | f << 5 |
// offset, chunks of fb_region_chunk_bits()), rstat = nreg words (FB_REGION_END / _LINK / other)
constexpr uint32_t FB_REGION_END = 0x80000001u, FB_REGION_LINK = 0x80000002u;
uint64_t fb_region_super_bits();
uint64_t fb_region_chunk_bits();
uint32_t fb_region_nodes();
// Jraw (nsb * fb_region_nodes() words): the chunk maps before pointer jumping; cbit: the stream
// bit where the true path enters each chunk and sub-chunk (~0: not entered), k_fb_schunks
hipError_t launch_fb_regions(const uint32_t* in_words, uint64_t misalign, uint64_t n, const uint64_t* reg,
                             uint32_t nreg, const uint32_t* sbreg, uint64_t nsb, uint32_t* J, uint32_t* visit,
                             uint32_t* rstat, uint32_t* Jraw, uint64_t* Jsub, uint64_t* cbit, hipStream_t st);
// (Jsub: nsb * fb_region_nodes() 64-bit words; cbit: nsb * fb_region_entries() words)
uint32_t fb_region_entries();
hipError_t launch_fb_decode(const uint32_t* in_words, uint64_t misalign, uint64_t n,
                            const uint64_t* starts, const uint64_t* stops, const uint8_t* vmode,
                            const uint64_t* vhdr, uint64_t nunits, uint64_t u0, uint64_t count,
                            const uint64_t* tokoff, uint32_t* tok, FbUnit* units, uint32_t flags,
                            bool parallel, uint32_t* stats, const uint64_t* cbit, const uint32_t* ucb,
                            hipStream_t st);
// (cbit / ucb: the region units' exact chunk entries, see FbDecodeArgs; nullptr when none)
// replay + window hand-off + final resolve; *err (zeroed by the caller) becomes nonzero when a
// copy reaches before the stream start.  win (fb_window_entries(nchain) words, 0 = not
// available) and open (fb_window_rounds(nchain) words): the parallel hand-off; win == nullptr:
// the serial one (k_fb_tails).  workgroup: the workgroup replay k_fb_units (pieces in LDS),
// else the one-wave replay k_fb_replay
uint64_t fb_window_entries(uint64_t nchain);
uint32_t fb_window_rounds(uint64_t nchain);
hipError_t launch_fb_resolve(const uint8_t* stream, const uint64_t* starts, const uint32_t* chain,
                             const uint64_t* offs, const uint64_t* sizes, uint64_t nchain,
                             const uint64_t* tokoff, const uint32_t* tok, const FbUnit* units,
                             uint16_t* img, uint64_t total, uint8_t* out, uint32_t* err,
                             uint32_t* win, uint32_t* open, bool workgroup, unsigned long long* ph,
                             hipStream_t st);
// checksums (checksum.hip): scratch of checksum_scratch_bytes(n) bytes; results land in device
// memory (*d_out).  CRC-32: the zero-start register; crc32_finish applies start value and xor.
uint64_t checksum_scratch_bytes(uint64_t n);
hipError_t launch_adler32(const uint8_t* d, uint64_t n, uint32_t init, void* scratch, uint32_t* d_out,
                          hipStream_t st);
hipError_t launch_crc32_raw(const uint8_t* d, uint64_t n, void* scratch, uint32_t* d_out, hipStream_t st);
uint32_t crc32_finish(uint32_t raw, uint64_t n, uint32_t init);

hipError_t launch_place_segments(const uint8_t* src, uint32_t slot, const uint64_t* chain, const uint64_t* offs,
                                 const uint32_t* sizes, uint64_t nch, uint8_t* dst, hipStream_t st);
hipError_t launch_segment_check(const InflateArgs& A, const uint64_t* starts, uint64_t k, uint64_t* ends,
                                hipStream_t st);
hipError_t launch_inflate_serial(const InflateArgs& A, int count_only, InflateResult* res,
                                 hipStream_t st);

}  // namespace dmx
