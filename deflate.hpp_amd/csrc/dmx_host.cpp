// dmx_host.cpp -- host runtime and C-ABI of libdmx (see include/dmx.h).
//
// A context owns one HIP device, one non-blocking stream and grow-only device scratch
// (segment slots, size/offset arrays, candidate lists, look-back words).  Every entry point
// locks the context, so a context may be shared between threads; the default context is
// created once per process (std::call_once) on the caller's current device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <thread>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "../../include/dmx.h"
#include "dmx_internal.h"

using namespace dmx;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 8 + 4096;
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = want;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

constexpr uint32_t kSegCap = 32768;  // LDS window of k_inflate_segments
#ifndef DMX_FB_REPAIR_EXACT
#define DMX_FB_REPAIR_EXACT 0  // path-5 repair units inside fixed-code regions on exact chunk entries
#endif
constexpr uint64_t LN_OUT_CAP_BYTES = 32768;  // largest segment output of the lane decoder

}  // namespace

struct dmx_ctx {
    int device = 0;
    uint32_t seg = 32768;
    uint32_t flags = 0;
    int inflate_pass = -1;     // dmx_config.dev_inflate_pass - 1: forced pass, -1 = the plan
    uint32_t heavy_bytes = 0;  // dmx_config.dev_heavy_bytes
    uint32_t diag = 0;         // DIAG_* bits, read once from the environment at dmx_create
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevBuf in, out, slots, sizes, offs, scal, cands, tiles, tileoffs, recs, status, dbg;
    DevBuf dtok, dntok;                  // deflate: the front kernel's token words and counts
    DevBuf rtmp, rchain;                 // chain repair: scratch output, chain / offsets / sizes
    DevBuf ltok, ltokoff, lntok, lcaps, lsplit;  // lane decoder token lists (mode 4), 64 KiB halves
    DevBuf lheavy;                       // heavy-candidate list for the workgroup decoder (mode 6)
    int ncu = 0;                         // compute units (mode 6 grid)
    // block-parallel path (path 5): scan counts / hits / offsets, hit list, unit starts, token
    // offsets and words, unit records, chain (unit index, offset, size), 16-bit image
    DevBuf fbc, fbh, fbo, fbl, fbs, fbt, fbk, fbu, fbch, fbco, fbcs, fbimg, fbstop, fbwin, fbopen;
    DevBuf fbvm, fbvh;  // per-unit start mode and code state (region and repair units)
    DevBuf fbph;  // DMX_FB_DEBUG: k_fb_units phase cycles
    // path 5: the accepted unit starts, written by k_fb_check straight into host memory
    uint64_t* fbkeep_h = nullptr;
    uint64_t* fbkeep_d = nullptr;
    // path 5: pinned staging of host-to-device uploads (a copy from pageable memory goes through
    // the driver's own staging); reused per batch -- a stream sync separates the batches
    uint8_t* pin = nullptr;
    size_t pin_cap = 0, pin_off = 0;
    DevBuf fbreg, fbJ, fbvis;  // fixed-code regions: {E, T, first super block} + super-block regions, jumps, visits
    DevBuf fbJraw, fbJsub, fbcbit, fbucb;  // regions: chunk maps, sub-chunk entries, chunk entries, unit chunk
    DevBuf ck;  // checksum scratch (checksum.hip) + the 4-byte result at its start
    bool timing = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_df = nullptr;          // end of the last deflate's work (its scratch is reused)
    hipEvent_t ev_inf = nullptr;         // end of the last asynchronous inflate's work
    bool inf_pending = false;
    bool df_pending = false;
    dmx_stats stats{};
    uint64_t last_end = 0;               // the last inflate: stream byte just past its final block
    std::vector<dmx_ctx*> subs;          // n_gpus > 1: one context per shard / piece
};

namespace {

// Diagnostics (never steer results): read from the environment once, at dmx_create.
//   DMX_DEBUG=1       names the failing HIP call on stderr (process-wide)
//   DMX_PHASES=<file> per-phase s_memtime timelines of the segmented kernels
//   DMX_FB_DEBUG=1    block-parallel path: unit outcomes and chain breaks on stderr
//   DMX_FB_HOSTTIME=1 block-parallel path: host wall clock per phase on stderr
//   DMX_RECS=1        segmented inflate: per-candidate outcome of each pass on stderr
enum : uint32_t { DIAG_PHASES = 1, DIAG_FB = 2, DIAG_RECS = 4, DIAG_DEBUG = 8, DIAG_FBT = 16 };
struct Diag {
    uint32_t bits = 0;
    std::string phases_path;
};
static const Diag& diag_env() {  // first use (a dmx_create) reads the environment
    static const Diag d = [] {
        Diag r;
        if (std::getenv("DMX_DEBUG")) r.bits |= DIAG_DEBUG;
        if (const char* e = std::getenv("DMX_PHASES")) r.bits |= DIAG_PHASES, r.phases_path = e;
        if (const char* e = std::getenv("DMX_FB_DEBUG"); e && *e) r.bits |= DIAG_FB;
        if (const char* e = std::getenv("DMX_FB_HOSTTIME"); e && *e) r.bits |= DIAG_FBT;
        if (std::getenv("DMX_RECS")) r.bits |= DIAG_RECS;
        return r;
    }();
    return d;
}
static void hipchk_report(const char* what, hipError_t e, int line) {
    if (diag_env().bits & DIAG_DEBUG)
        std::fprintf(stderr, "dmx: %s failed (dmx_host.cpp:%d): %s\n", what, line, hipGetErrorString(e));
}
#define HIPCHK(x)                                   \
    do {                                            \
        const hipError_t e_ = (x);                  \
        if (e_ != hipSuccess) {                     \
            hipchk_report(#x, e_, __LINE__);        \
            return DMX_ERR_DEVICE;                  \
        }                                           \
    } while (0)

struct Scal {  // small device-side scalars, one allocation
    uint64_t total;
    uint64_t nmarkers;
    uint32_t ticket;
    uint32_t fb_err;  // block-parallel path: a copy reached before the stream start
    uint32_t fb_nkeep;  // block-parallel path: accepted unit starts (k_fb_check)
    uint64_t ncand;     // dmx_inflate_device_async: the candidate count, on the device
    InflateResult res;
    ValidateWords vw;
};

// DMX_PHASES=<file>: kernels record s_memtime per phase and segment; the host appends one line
// "<kernel> <nsegs> <mean cycles of phase k - phase k-1 ...>" per call (developer profiling).
uint64_t* phase_buf(dmx_ctx* c, uint64_t nidx) {
    if (!(c->diag & DIAG_PHASES)) return nullptr;
    if (!c->dbg.ensure(nidx * kPhaseSlots * 8)) return nullptr;
    (void)hipMemset(c->dbg.p, 0, nidx * kPhaseSlots * 8);
    return c->dbg.as<uint64_t>();
}
void phase_dump(dmx_ctx* c, const char* kernel, uint64_t nidx, hipStream_t st) {
    if (!(c->diag & DIAG_PHASES) || !c->dbg.p) return;
    const char* path = diag_env().phases_path.c_str();
    std::vector<uint64_t> h(nidx * kPhaseSlots);
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(h.data(), c->dbg.p, h.size() * 8, hipMemcpyDeviceToHost);
    double sum[kPhaseSlots] = {0}, xsum[kPhaseSlots] = {0};
    uint64_t xcnt[kPhaseSlots] = {0};
    uint64_t cnt[kPhaseSlots] = {0};
    const bool inf = std::string(kernel) == "inflate";
    for (uint64_t i = 0; i < nidx; i++) {
        const uint64_t* r = &h[i * kPhaseSlots];
        uint64_t prev = r[0];
        for (int k = 1; k < (inf ? 8 : 12); k++) {
            if (!inf && k == 12) break;
            if (!r[k]) continue;
            sum[k] += (double)(r[k] - prev);
            cnt[k]++;
            prev = r[k];
        }
        if (inf) {  // slots 8..10: raw per-segment values (header cycles / settle and jump rounds)
            for (int k = 8; k < 16; k++) { xsum[k] += (double)r[k]; xcnt[k]++; }
        }
        if (!inf && r[12] && r[13] && r[3] && r[14]) {  // Huffman build sub-phases, match rounds
            sum[12] += (double)(r[12] - r[3]); cnt[12]++;
            sum[13] += (double)(r[13] - r[12]); cnt[13]++;
            sum[14] += (double)(r[14] - r[1]); cnt[14]++;
        }
    }
    FILE* f = std::fopen(path, "a");
    if (!f) return;
    std::fprintf(f, "%s %llu", kernel, (unsigned long long)nidx);
    for (int k = 1; k < kPhaseSlots; k++) std::fprintf(f, " p%d=%.0f", k, cnt[k] ? sum[k] / cnt[k] : 0.0);
    if (!inf) {  // timeline: mean cycles from slot 0 to every recorded slot (developer aid)
        for (int k = 1; k < kPhaseSlots; k++) {
            double a = 0;
            uint64_t m = 0;
            for (uint64_t i = 0; i < nidx; i++) {
                const uint64_t* r = &h[i * kPhaseSlots];
                if (r[k] && r[0] && r[k] >= r[0]) { a += (double)(r[k] - r[0]); m++; }
            }
            if (m) std::fprintf(f, " t%d=%.0f", k, a / m);
        }
    }
    if (inf)
        for (int k = 8; k < kPhaseSlots; k++) std::fprintf(f, " x%d=%.1f", k, xcnt[k] ? xsum[k] / xcnt[k] : 0.0);

    std::fprintf(f, "\n");
    std::fclose(f);
}

void begin_timing(dmx_ctx* c, hipStream_t st) {
    c->stats = dmx_stats{};
    if (c->timing) (void)hipEventRecord(c->ev[0], st);
}
void end_timing(dmx_ctx* c, hipStream_t st) {
    if (!c->timing) return;
    (void)hipEventRecord(c->ev[3], st);
    (void)hipEventSynchronize(c->ev[3]);
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, c->ev[0], c->ev[3]);
    (void)hipEventElapsedTime(&b, c->ev[1], c->ev[2]);
    (void)hipGetLastError();  // a failed query must not surface in the caller's next HIP call
    c->stats.ms_device_total = a;
    c->stats.ms_main_kernel = b;
}

// d_total != nullptr: asynchronous (dmx_deflate_device_async): the length goes to that device
// word, nothing waits for the work.  Every deflate on a context waits for the previous one's work
// (ev_df), whatever streams they run on: the slots, sizes and token words are reused.
int deflate_device_locked(dmx_ctx* c, const uint8_t* d_in, size_t n, int level, uint32_t flags,
                          uint8_t* d_out, size_t cap, size_t* out_len, hipStream_t st,
                          uint64_t* d_total = nullptr) {
    if (level < 0 || level > 3) level = 1;  // reference switch has no default (deflate.hpp:699)
    const bool final_last = (flags & DMX_DEFLATE_NOT_FINAL) == 0;
    const bool async = d_total != nullptr;
    if (c->df_pending) HIPCHK(hipStreamWaitEvent(st, c->ev_df, 0));
    if (!async) begin_timing(c, st);
    if (n == 0) {
        // empty input: one empty fixed-Huffman final block, as the reference's levels 1-3
        static const uint8_t empty_final[2] = {0x03, 0x00};
        static const uint64_t lens[2] = {0, 2};
        if (out_len) *out_len = final_last ? 2 : 0;
        if (async) {
            if (final_last && cap >= 2) HIPCHK(hipMemcpyAsync(d_out, empty_final, 2, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(d_total, &lens[final_last ? 1 : 0], 8, hipMemcpyHostToDevice, st));
            return DMX_OK;
        }
        if (!final_last) return DMX_OK;
        if (cap < 2) return DMX_ERR_CAPACITY;
        HIPCHK(hipMemcpyAsync(d_out, empty_final, 2, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        return DMX_OK;
    }
    const uint64_t nseg = (n + c->seg - 1) / c->seg;
    const uint32_t slot_bytes = c->seg + 256;
    // the front kernel's segments: 64 KiB blocks are matched as two 32 KiB halves
    const uint32_t fseg_bytes = std::min<uint32_t>(c->seg, 32768);
    const uint64_t nfront = (n + fseg_bytes - 1) / fseg_bytes;
    const uint32_t tok_stride = level >= 2 ? deflate_tok_stride(fseg_bytes) : 0u;
    if (!c->slots.ensure(nseg * (size_t)slot_bytes) || !c->sizes.ensure(nseg * 4) ||
        !c->offs.ensure(scan_words(nseg) * 8) || !c->scal.ensure(sizeof(Scal)) ||
        !c->dtok.ensure(std::max<uint64_t>(1, nfront * (uint64_t)tok_stride) * 4) || !c->dntok.ensure(nfront * 4))
        return DMX_ERR_NOMEM;
    DeflateArgs A;
    A.in = d_in;
    A.n = n;
    A.nseg = nseg;
    A.level = level;
    A.final_last = final_last ? 1 : 0;
    A.slots = c->slots.as<uint8_t>();
    A.slot_bytes = slot_bytes;
    A.tok = c->dtok.as<uint32_t>();
    A.tok_stride = tok_stride;
    A.ntok = c->dntok.as<uint32_t>();
    A.sizes = c->sizes.as<uint32_t>();
    A.offsets = c->offs.as<uint64_t>();
    A.total = async ? d_total : &c->scal.as<Scal>()->total;
    A.out = d_out;
    A.cap = cap;
    A.dbg = async ? nullptr : phase_buf(c, nseg);
    const bool tm = c->timing && !async;
    HIPCHK(launch_deflate(A, c->seg, st, tm ? c->ev[1] : nullptr, tm ? c->ev[2] : nullptr));
    HIPCHK(hipEventRecord(c->ev_df, st));
    c->df_pending = true;
    if (async) return DMX_OK;
    if (A.dbg) phase_dump(c, "deflate", nseg, st);
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, A.total, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    end_timing(c, st);
    c->stats.segments = nseg;
    c->stats.in_bytes = n;
    c->stats.out_bytes = total;
    *out_len = total;
    return total > cap ? DMX_ERR_CAPACITY : DMX_OK;
}

// Block-parallel inflate of an arbitrary stream (inflate_blocks.hip): header scan, unit decode,
// chain walk here on the host, replay / window hand-off / resolve.  *handled = false sends the
// stream to the serial decoder (no chain from bit 0 to a BFINAL block, a unit that errors or
// runs out of token space, a copy from before the stream start): results and error codes are
// then the serial decoder's, i.e. the reference's.
// DMX_CFG_FB_SERIAL: path 5 decodes every unit with one wavefront (A/B reference for k_fb_pdecode)
static bool fb_serial_only(const dmx_ctx* c) { return (c->flags & DMX_CFG_FB_SERIAL) != 0; }

// host-to-device copy through the context's pinned staging (see dmx_ctx::pin); the caller
// resets c->pin_off once the previous batch's copies are known complete
static hipError_t pin_h2d(dmx_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (!bytes) return hipSuccess;
    constexpr size_t kPinCap = 1u << 20;
    if (!c->pin && hipHostMalloc(reinterpret_cast<void**>(&c->pin), kPinCap, hipHostMallocDefault) == hipSuccess)
        c->pin_cap = kPinCap;
    if (!c->pin || c->pin_off + bytes > c->pin_cap) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    uint8_t* h = c->pin + c->pin_off;
    std::memcpy(h, src, bytes);
    c->pin_off += (bytes + 255) & ~size_t(255);
    return hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st);
}

int inflate_fb_locked(dmx_ctx* c, const uint8_t* d_in, size_t n, uint8_t* fixed_out, size_t cap,
                      size_t* total_out, uint8_t** dev_out, hipStream_t st, bool* handled, uint32_t iflags) {
    *handled = false;
    Scal* ds = c->scal.as<Scal>();
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    // DMX_FB_HOSTTIME: host-side wall clock per phase (us)
    using hclock = std::chrono::steady_clock;
    hclock::time_point ht[8];
    auto hmark = [&](int k) { if (c->diag & DIAG_FBT) ht[k] = hclock::now(); };
    hmark(0);
    const uint64_t misalign = (uintptr_t)d_in & 3;
    const uint32_t* words = reinterpret_cast<const uint32_t*>(d_in - misalign);
    const uint64_t nc = fb_scan_chunks(n);
    if (!c->fbc.ensure(nc * 4) || !c->fbh.ensure(nc * fb_hits_per_chunk() * 8) || !c->fbo.ensure(scan_words(nc) * 8))
        return DMX_OK;
    HIPCHK(launch_fb_scan(words, misalign, n, c->fbc.as<uint32_t>(), c->fbh.as<uint64_t>(),
                          c->fbo.as<uint64_t>(), &ds->nmarkers, st));
    // The check appends the accepted starts to a host-mapped list, so one sync gives them (the
    // candidate count need not come back first); its grid is sized for the most the scan can
    // list.  Without that list (or when it overflows) the candidates come back in two steps.
    constexpr uint32_t kKeepCap = 1u << 20;
    if (!c->fbkeep_h) {
        void* h = nullptr;
        if (hipHostMalloc(&h, kKeepCap * 8ull, hipHostMallocMapped) == hipSuccess) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
                c->fbkeep_h = static_cast<uint64_t*>(h);
                c->fbkeep_d = static_cast<uint64_t*>(d);
            } else {
                (void)hipHostFree(h);
            }
        }
    }
    const uint64_t max_hits = nc * (uint64_t)fb_hits_per_chunk();
    const bool one_sync = c->fbkeep_d && c->fbl.ensure(max_hits * 8);
    unsigned long long* cph = nullptr;  // DMX_FB_DEBUG: k_fb_check counters
    if ((c->diag & DIAG_FB) && c->fbph.ensure(256)) {
        cph = c->fbph.as<unsigned long long>();
        HIPCHK(hipMemsetAsync(cph, 0, 256, st));
    }
    uint64_t nhits = 0;
    std::vector<uint64_t> hits;
    bool have_hits = false;
    if (one_sync) {
        HIPCHK(hipMemsetAsync(&ds->fb_nkeep, 0, 4, st));
        HIPCHK(launch_fb_compact(words, misalign, n, c->fbc.as<uint32_t>(), c->fbo.as<uint64_t>(),
                                 c->fbh.as<uint64_t>(), nc, c->fbl.as<uint64_t>(), &ds->nmarkers, max_hits, cph,
                                 c->fbkeep_d, &ds->fb_nkeep, kKeepCap, st));
        uint32_t nkeep = 0;
        HIPCHK(hipMemcpyAsync(&nhits, &ds->nmarkers, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&nkeep, &ds->fb_nkeep, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (nkeep <= kKeepCap) {
            hits.assign(c->fbkeep_h, c->fbkeep_h + nkeep);
            std::sort(hits.begin(), hits.end(), [](uint64_t a, uint64_t b) {
                return (a & FB_STOP_MASK) < (b & FB_STOP_MASK);
            });
            have_hits = true;
        }
    } else {
        HIPCHK(hipMemcpyAsync(&nhits, &ds->nmarkers, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (nhits) {
            if (!c->fbl.ensure(nhits * 8)) return DMX_OK;
            HIPCHK(launch_fb_compact(words, misalign, n, c->fbc.as<uint32_t>(), c->fbo.as<uint64_t>(),
                                     c->fbh.as<uint64_t>(), nc, c->fbl.as<uint64_t>(), &ds->nmarkers, nhits, cph,
                                     nullptr, nullptr, 0, st));
        }
    }
    if (cph) {
        unsigned long long q[5];
        HIPCHK(hipMemcpyAsync(q, cph + 8, sizeof(q), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const unsigned long long w = q[4] ? q[4] : 1;
        std::fprintf(stderr, "dmx fb: k_fb_check %llu candidates, %llu waves: per wave refill %llu cycles, "
                     "steps %llu cycles, %llu steps, %.1f busy lanes per step\n", (unsigned long long)nhits, w,
                     q[0] / w, q[1] / w, q[2] / w, q[2] ? (double)q[3] / (double)q[2] : 0.0);
    }
    if (!have_hits && nhits) {  // the candidates with their reject marks
        hits.resize(nhits);
        HIPCHK(hipMemcpyAsync(hits.data(), c->fbl.p, nhits * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    hmark(1);
    // units: bit 0, then every hit (sorted: chunks in order, lanes in order within a chunk);
    // dynamic-header hits are "strong" (practically never false), stored-header hits "weak".
    // A gap of more than kRegionGap bits between two strong starts is a run of blocks the scan
    // cannot split (fixed-code blocks -- zlib's Z_FIXED, the reference's own level-1/2 chunks --
    // or one huge block).  Its head unit decodes only a dynamic first block (and what follows
    // it up to the first far fixed-code header, FB_STOP_REGION); from where it stops, E, to the
    // next strong start T the region map (k_fb_smap / k_fb_swalk) finds the exact token path,
    // and one unit per 2^18 bits starts exactly on it.  The chain walk below verifies every link
    // (end bit and code state); a break gets a repair unit that starts exactly there.
    constexpr uint64_t kStored = 1ull << 62;
    const uint64_t kSuper = fb_region_super_bits();
    const uint64_t kRegionGap = kSuper + kSuper / 2;
    constexpr int kRepairRounds = 48;
    const uint64_t nbits = 8ull * n;
    std::vector<uint64_t> starts, vhdr;
    std::vector<uint8_t> strong, vmode;
    std::vector<uint32_t> ucb;  // region units: the first global chunk of their super block
    starts.push_back(0);
    strong.push_back(1);
    for (uint64_t h : hits) {
        if (h & FB_HIT_REJECT) continue;
        const uint64_t b = h & ~kStored;
        if (b > starts.back()) {
            starts.push_back(b);
            strong.push_back((h & kStored) ? 0 : 1);
        }
    }
    const uint64_t K = starts.size();
    std::vector<uint64_t> stops(K);
    {
        uint64_t next_strong = FB_STOP_MASK;
        for (uint64_t k = K; k-- > 0;) {
            stops[k] = next_strong;
            if (!strong[k]) stops[k] |= FB_STOP_WEAK;
            else if (std::min(next_strong, nbits) - starts[k] > kRegionGap) stops[k] |= FB_STOP_REGION;
            if (strong[k]) next_strong = starts[k];
        }
    }
    // Token words: up to where a unit can stop, plus room for the block that crosses its stop.
    // A token word takes at least 1.5 bits of stream: a match at least 2 (a lit/len and a
    // distance code, each at least 1 bit), a word of literals up to three of them; the densest
    // packing is a 1-bit literal then a 2-bit match, two words per 3 bits -- so 2/3 of a word per
    // bit always suffices (C3 uses 0.37).  A weak unit with a hard stop (a stored block -- two
    // words -- then possibly fixed-code blocks up to the next dynamic one) gets 64 Ki words; a
    // region head at most its staged first block.  A unit that fills its space stops softly and
    // a repair unit continues it.  Inside a fixed-code region a token word covers at least 7 bits
    // (fixed codes are 7-9 bits, three literals per word), so a third of a word per bit.  16-B
    // groups.
    auto words_of = [&](uint64_t pos, uint64_t stop) -> uint64_t {
        const uint64_t s = std::min<uint64_t>(stop & FB_STOP_MASK, nbits), p = std::min(pos, nbits);
        uint64_t w = 4096 + 65536;
        if (stop & FB_STOP_REGION) w = std::min<uint64_t>(2 * (s - p) / 3, 458752 + 65536) + 4096;
        else if (!(stop & FB_STOP_WEAK)) w = 2 * (s - p) / 3 + 4096;
        return (w + 63) & ~63ull;
    };
    auto region_words = [](uint64_t span) -> uint64_t { return ((span / 3 + 4096) + 63) & ~63ull; };
    // a repair unit (or the last unit of a failed region walk) whose stop is far: at most this
    // many words (>= 6 Mbit of the densest code); when they fill, it stops softly and the next
    // repair round continues it, instead of reserving 2/3 of a word per bit up to the stop
    constexpr uint64_t kOpenWords = (1ull << 22) + 4096;
    // region budget: every long gap could become one region of units, each with a repair
    uint64_t reg_budget = 0, reg_units_max = 0;
    for (uint64_t k = 0; k < K; k++)
        if (stops[k] & FB_STOP_REGION) {
            const uint64_t span = std::min(stops[k] & FB_STOP_MASK, nbits) - starts[k];
            const uint64_t nu = span / kSuper + 2;
            reg_units_max += nu;
            reg_budget += span / 3 + nu * (4096 + 64);
        }
    const uint64_t R = 2 * std::max<uint64_t>(256, K + reg_units_max);  // repair units
    const uint64_t Kcap = K + reg_units_max + R;
    std::vector<uint64_t> tokoff(Kcap + 1);
    starts.resize(Kcap);
    vhdr.assign(Kcap, 0);
    vmode.assign(Kcap, FB_V_HEADER);
    ucb.assign(Kcap, ~0u);
    stops.resize(Kcap);
    tokoff[0] = 0;
    for (uint64_t k = 0; k < K; k++) tokoff[k + 1] = tokoff[k] + words_of(starts[k], stops[k]);
    const uint64_t rep_words = std::min<uint64_t>(tokoff[K] + 2 * reg_budget + 4096 * R, 1ull << 29);
    if (!c->fbs.ensure(Kcap * 8) || !c->fbt.ensure((Kcap + 1) * 8) || !c->fbk.ensure((tokoff[K] + rep_words) * 4) ||
        !c->fbu.ensure(Kcap * sizeof(FbUnit)) || !c->fbstop.ensure(Kcap * 8) || !c->fbvm.ensure(Kcap) ||
        !c->fbvh.ensure(Kcap * 8) || !c->fbucb.ensure(Kcap * 4))
        return DMX_OK;
    const uint64_t* dcbit = nullptr;  // set once the regions' chunk entries exist
    auto upload = [&](uint64_t k0, uint64_t cnt) -> int {  // (each batch follows a stream sync)
        c->pin_off = 0;
        HIPCHK(pin_h2d(c, c->fbs.as<uint64_t>() + k0, &starts[k0], cnt * 8, st));
        HIPCHK(pin_h2d(c, c->fbstop.as<uint64_t>() + k0, &stops[k0], cnt * 8, st));
        HIPCHK(pin_h2d(c, c->fbt.as<uint64_t>() + k0, &tokoff[k0], (cnt + 1) * 8, st));
        HIPCHK(pin_h2d(c, c->fbvm.as<uint8_t>() + k0, &vmode[k0], cnt, st));
        HIPCHK(pin_h2d(c, c->fbvh.as<uint64_t>() + k0, &vhdr[k0], cnt * 8, st));
        HIPCHK(pin_h2d(c, c->fbucb.as<uint32_t>() + k0, &ucb[k0], cnt * 4, st));
        return DMX_OK;
    };
    hmark(2);
    if (upload(0, K) != DMX_OK) return DMX_ERR_DEVICE;
    hmark(3);
    const bool fb_debug = (c->diag & DIAG_FB) != 0;  // developer aid: unit outcomes, chain breaks
    uint32_t* dstats = nullptr;
    if (fb_debug && c->fbopen.ensure(256)) {
        dstats = c->fbopen.as<uint32_t>();
        HIPCHK(hipMemsetAsync(dstats, 0, 256, st));
    }
    std::vector<FbUnit> units(Kcap);
    auto decode = [&](uint64_t u0, uint64_t cnt) -> int {
        HIPCHK(launch_fb_decode(words, misalign, n, c->fbs.as<uint64_t>(), c->fbstop.as<uint64_t>(),
                                c->fbvm.as<uint8_t>(), c->fbvh.as<uint64_t>(), K, u0, cnt, c->fbt.as<uint64_t>(),
                                c->fbk.as<uint32_t>(), c->fbu.as<FbUnit>(), c->flags | iflags, !fb_serial_only(c),
                                dstats, dcbit, dcbit ? c->fbucb.as<uint32_t>() : nullptr, st));
        HIPCHK(hipMemcpyAsync(&units[u0], c->fbu.as<FbUnit>() + u0, cnt * sizeof(FbUnit), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return DMX_OK;
    };
    if (decode(0, K) != DMX_OK) return DMX_ERR_DEVICE;
    hmark(4);
    // DMX_FB_DEBUG: the decode counters so far (cumulative over the first pass, the region units
    // and the repair rounds; "longest" is the longest unit of each kind so far)
    auto dump_stats = [&](const char* what, uint64_t Kn) -> int {
        if (!dstats) return DMX_OK;
        uint32_t hs[16];
        unsigned long long ph[21];
        HIPCHK(hipMemcpyAsync(hs, dstats, 64, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(ph, dstats + 16, sizeof(ph), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const uint64_t K = std::max<uint64_t>(Kn, 1);
        std::fprintf(stderr, "dmx fb [%s]: pdecode header cycles per unit: precode %llu, code lengths %llu, trees %llu, "
                     "tables %llu; longest unit: lane-parallel %llu, serial %llu, serial after a block %llu, weak %llu\n",
                     what, ph[10] / K, ph[11] / K, ph[12] / K, ph[13] / K, ph[14] >> 24, ph[15] >> 24, ph[16] >> 24,
                     ph[17] >> 24);
        std::fprintf(stderr, "dmx fb [%s]: longest lane-parallel unit: %llu settle rounds, %llu attempts; "
                     "settle re-decodes %llu cycles per unit\n",
                     what, (ph[14] >> 4) & 4095, ph[14] & 15, ph[20] / K);
        std::fprintf(stderr, "dmx fb [%s]: pdecode cycles per unit: stage %llu, header %llu, tables %llu, first pass %llu, "
                     "settle %llu (%.1f rounds, %.1f lane redos), recount %llu, scans %llu, words %llu\n",
                     what, ph[0] / K, ph[1] / K, ph[2] / K, ph[3] / K, ph[4] / K, (double)ph[8] / K, (double)ph[9] / K,
                     ph[5] / K, ph[6] / K, ph[7] / K);
        std::fprintf(stderr, "dmx fb [%s]: %llu units: %u lane-parallel, %u serial, %u serial after a parallel block, %u weak; "
                     "serial because: header %u, unsettled %u, no end of block %u, bad end %u, capacity %u, "
                     "stream-start copy %u\n",
                     what, (unsigned long long)Kn, hs[0], hs[1], hs[2], hs[3], hs[4], hs[5], hs[6], hs[7], hs[8], hs[9]);
        return DMX_OK;
    };
    if (dump_stats("first pass", K) != DMX_OK) return DMX_ERR_DEVICE;
    uint64_t Ku = K;
    uint64_t rep_used = 0;
    // Sorted list of the starts a repair unit stops at: the scanned ones (a weak start inside a
    // region is superseded by the region's units) and the region units' (soft: inside a block,
    // except the region head E, a block header).
    struct Prim {
        uint64_t pos;
        uint8_t kind;  // 0 strong / region head, 1 weak, 2 soft
    };
    std::vector<Prim> prim;
    struct Reg {
        uint64_t E, T, sb0, nsb;
    };
    std::vector<Reg> regs;  // (kept for the repair units: exact chunk entries inside a region)
    // ---- fixed-code regions ----
    {
        uint64_t nsb = 0;
        for (uint64_t k = 0; k < K; k++) {
            if (!(stops[k] & FB_STOP_REGION)) continue;
            const FbUnit& u = units[k];
            if ((u.flags & (SEGF_ERRORS | SEGF_FINAL)) || u.hdr != FB_AT_HEADER) continue;
            const uint64_t T = std::min(stops[k] & FB_STOP_MASK, nbits);
            if (u.end >= T || T - u.end <= kSuper) continue;  // a repair unit takes the rest
            const uint64_t m = (T - u.end + kSuper - 1) / kSuper;
            regs.push_back({u.end, T, nsb, m});
            nsb += m;
        }
        std::vector<uint8_t> in_region(K, 0);
        if (!regs.empty()) {
            const uint64_t nreg = regs.size();
            if (!c->fbreg.ensure(nreg * 24 + nsb * 4) || !c->fbJ.ensure(nsb * (uint64_t)fb_region_nodes() * 4) ||
                !c->fbvis.ensure((nsb + nreg) * 4) || !c->fbJraw.ensure(nsb * (uint64_t)fb_region_nodes() * 4) ||
                !c->fbJsub.ensure(nsb * (uint64_t)fb_region_nodes() * 8) ||
                !c->fbcbit.ensure(nsb * (uint64_t)fb_region_entries() * 8))
                return DMX_OK;
            std::vector<uint64_t> hreg(3 * nreg);
            std::vector<uint32_t> sbreg(nsb);
            for (uint64_t r = 0; r < nreg; r++) {
                hreg[3 * r] = regs[r].E;
                hreg[3 * r + 1] = regs[r].T;
                hreg[3 * r + 2] = regs[r].sb0;
                for (uint64_t j = 0; j < regs[r].nsb; j++) sbreg[regs[r].sb0 + j] = (uint32_t)r;
            }
            uint64_t* dreg = c->fbreg.as<uint64_t>();
            uint32_t* dsbr = reinterpret_cast<uint32_t*>(dreg + 3 * nreg);
            uint32_t* dvis = c->fbvis.as<uint32_t>();
            HIPCHK(hipMemcpyAsync(dreg, hreg.data(), nreg * 24, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(dsbr, sbreg.data(), nsb * 4, hipMemcpyHostToDevice, st));
            HIPCHK(launch_fb_regions(words, misalign, n, dreg, (uint32_t)nreg, dsbr, nsb, c->fbJ.as<uint32_t>(), dvis,
                                     dvis + nsb, c->fbJraw.as<uint32_t>(), c->fbJsub.as<uint64_t>(),
                                     c->fbcbit.as<uint64_t>(), st));
            dcbit = c->fbcbit.as<uint64_t>();
            std::vector<uint32_t> vis(nsb + nreg);
            HIPCHK(hipMemcpyAsync(vis.data(), dvis, (nsb + nreg) * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            const uint64_t ch = fb_region_chunk_bits(), k0 = Ku;
            for (uint64_t r = 0; r < nreg; r++) {
                const uint32_t rs = vis[nsb + r];
                if (fb_debug)
                    std::fprintf(stderr, "dmx fb: region %llu: bits %llu..%llu, %llu super blocks, walk %s\n",
                                 (unsigned long long)r, (unsigned long long)regs[r].E, (unsigned long long)regs[r].T,
                                 (unsigned long long)regs[r].nsb,
                                 rs == FB_REGION_END ? "end" : rs == FB_REGION_LINK ? "link" : "fail (cut there)");
                // A failed walk (the map met a dynamic header that was not a listed start, a
                // stored block past T, ...): the super blocks it visited before failing are still
                // on the true path, so they keep their units; the last one decodes on towards T
                // (through the unlisted block, as far as its token space goes) and repair units
                // take the rest -- only that span loses parallelism, not the stream.
                const bool walked = rs == FB_REGION_END || rs == FB_REGION_LINK;
                const uint64_t first = Ku;
                for (uint64_t j = 0; j < regs[r].nsb; j++) {
                    const uint32_t v = vis[regs[r].sb0 + j];
                    if (v == ~0u) continue;
                    if (Ku >= Kcap) return DMX_OK;
                    const bool head = Ku == first;
                    starts[Ku] = regs[r].E + (uint64_t)(v >> 6) * ch + (v & 31u);
                    vmode[Ku] = head ? FB_V_HEADER : FB_V_EXACT;
                    vhdr[Ku] = head ? 0 : (FB_STATE_FIXED | ((v >> 5) & 1u ? FB_STATE_FINAL : 0ull));
                    ucb[Ku] = (uint32_t)((regs[r].sb0 + j) * 64);  // its super block's first chunk
                    Ku++;
                }
                for (uint64_t k = first; k < Ku; k++) {
                    stops[k] = k + 1 < Ku ? (starts[k + 1] | FB_STOP_SOFT) : regs[r].T;
                    const uint64_t w = k + 1 < Ku || walked
                                           ? region_words(std::min(stops[k] & FB_STOP_MASK, nbits) - starts[k])
                                           : std::min(words_of(starts[k], stops[k]), kOpenWords);
                    if (rep_used + w > rep_words) {
                        if (fb_debug)  // (say so instead of a silent serial decode)
                            std::fprintf(stderr, "dmx fb: region token space (%llu words) exhausted at unit %llu: "
                                         "the serial decoder takes the stream\n",
                                         (unsigned long long)rep_words, (unsigned long long)k);
                        return DMX_OK;
                    }
                    tokoff[k + 1] = tokoff[k] + w;
                    rep_used += w;
                    prim.push_back({starts[k], (uint8_t)(k == first ? 0 : 2)});
                }
                // weak starts inside the region: superseded
                for (uint64_t k = (uint64_t)(std::upper_bound(starts.begin(), starts.begin() + K, regs[r].E) - starts.begin());
                     k < K && starts[k] < regs[r].T; k++)
                    in_region[k] = 1;
            }
            if (Ku > k0 && (upload(k0, Ku - k0) != DMX_OK || decode(k0, Ku - k0) != DMX_OK)) return DMX_ERR_DEVICE;
            if (fb_debug && dump_stats("region units", Ku) != DMX_OK) return DMX_ERR_DEVICE;
        }
        for (uint64_t k = 0; k < K; k++)
            if (!in_region[k]) prim.push_back({starts[k], (uint8_t)(strong[k] ? 0 : 1)});
        std::sort(prim.begin(), prim.end(), [](const Prim& a, const Prim& b) { return a.pos < b.pos; });
    }
    // the stop of a repair unit at pos: a soft stop at the next region unit, else the next
    // strong start (or region head)
    auto stop_of = [&](uint64_t pos) -> uint64_t {
        auto it = std::upper_bound(prim.begin(), prim.end(), pos, [](uint64_t p, const Prim& q) { return p < q.pos; });
        if (it != prim.end() && it->kind == 2) return it->pos | FB_STOP_SOFT;
        for (; it != prim.end(); ++it)
            if (it->kind != 1) return it->pos;
        return FB_STOP_MASK;
    };
    // the code state a unit assumes at its start: FB_AT_HEADER, or the code in force
    auto expects = [&](uint64_t k) -> uint64_t { return vmode[k] == FB_V_HEADER ? FB_AT_HEADER : vhdr[k]; };
    // chain from bit 0: each unit must end exactly where the next one on the chain starts, in
    // the code state that one assumes (a block header, or the code in force and its BFINAL bit).
    // Every break -- an end where no such unit starts -- gets a repair unit that starts exactly
    // there in that state; the walk goes on optimistically past a break (from the next unit in
    // start order), so one round repairs all the breaks it can see.
    std::vector<uint32_t> chain;
    std::vector<uint64_t> coffs, csizes;
    uint64_t total = 0;
    auto chain_break = [&](const char* why, uint64_t k) {
        if (fb_debug)
            std::fprintf(stderr, "dmx fb: chain breaks at unit %llu of %llu (%s): start %llu end %llu size %llu flags %u\n",
                         (unsigned long long)k, (unsigned long long)Ku, why, (unsigned long long)units[k].start,
                         (unsigned long long)units[k].end, (unsigned long long)units[k].size, units[k].flags);
        return DMX_OK;
    };
    std::vector<std::pair<uint64_t, uint64_t>> repaired;  // (end bit, state) already given a repair unit
    // A unit that starts on the chain (at bit 0, or exactly where the chain's last unit ended, in
    // the code state it ended in) decodes the stream's own blocks from there, so an over-read or
    // an undecodable code it reports is the error realDecompress meets (inflate.hpp:277-322):
    // the stream ends with that error at once instead of a serial re-decode from bit 0 to find
    // it again (a truncated 1 GiB stream took ~75 s on the serial decoder).  Only
    // pure stream errors count; token space, staging or exotic-layout flags are this decoder's
    // own limits and still go to the serial decoder.
    auto stream_error = [&](const FbUnit& u) -> int {
        constexpr uint32_t kStreamErr = SEGF_OVERREAD | SEGF_ERR_DATA;
        if (!(u.flags & kStreamErr) || (u.flags & ~(kStreamErr | SEGF_CROSSED | SEGF_FINAL))) return DMX_OK;
        return (u.flags & SEGF_OVERREAD) ? DMX_ERR_OVERREAD : DMX_ERR_DATA;  // as k_inflate_serial maps it
    };
    auto chain_error = [&](int rc, uint64_t k) {
        if (fb_debug)
            std::fprintf(stderr, "dmx fb: the chain meets a stream error at unit %llu (start %llu): %s\n",
                         (unsigned long long)k, (unsigned long long)units[k].start, dmx_strerror(rc));
        *handled = true;
        *total_out = 0;
        c->stats.segments = chain.size();
        return rc;
    };
    for (int round = 0;; round++) {
        std::vector<std::pair<uint64_t, uint32_t>> by, bad;  // (start, unit) decoded without / with an error
        by.reserve(Ku);
        for (uint64_t k = 0; k < Ku; k++)
            (units[k].flags & SEGF_ERRORS ? bad : by).emplace_back(units[k].start, (uint32_t)k);
        std::sort(by.begin(), by.end());
        std::sort(bad.begin(), bad.end());
        chain.clear();
        coffs.clear();
        csizes.clear();
        total = 0;
        std::vector<std::pair<uint64_t, uint64_t>> breaks;  // (end bit, code state)
        bool fin = false;
        if (units[0].flags & SEGF_ERRORS) {
            if (const int rc = stream_error(units[0])) return chain_error(rc, 0);
            return chain_break("unit error", 0);
        }
        uint64_t k = 0;
        for (;;) {
            const FbUnit& u = units[k];
            chain.push_back((uint32_t)k);
            coffs.push_back(total);
            csizes.push_back(u.size);
            total += u.size;
            if (u.flags & SEGF_FINAL) {
                fin = true;
                break;
            }
            const uint64_t state = u.hdr;
            // (several units may start there in that state -- a scanned one, a region unit, a
            // repair: all decode the same tokens, the one that reaches farthest is taken)
            uint64_t best = ~0ull;
            for (auto it = std::lower_bound(by.begin(), by.end(), std::make_pair(u.end, 0u));
                 it != by.end() && it->first == u.end; ++it)
                if (it->second != k && expects(it->second) == state &&
                    (best == ~0ull || units[it->second].end >= units[best].end))
                    best = it->second;
            if (best != ~0ull) {
                k = best;
                continue;
            }
            if (breaks.empty()) {  // the first break: everything before it is the stream's true path
                for (auto it = std::lower_bound(bad.begin(), bad.end(), std::make_pair(u.end, 0u));
                     it != bad.end() && it->first == u.end; ++it)
                    if (expects(it->second) == state)
                        if (const int rc = stream_error(units[it->second])) return chain_error(rc, it->second);
            }
            breaks.emplace_back(u.end, state);
            // (optimistic: on with the unit after this one in start order)
            auto self = std::lower_bound(by.begin(), by.end(), std::make_pair(u.start, (uint32_t)k));
            if (self == by.end() || self->second != k || ++self == by.end()) break;
            k = self->second;
        }
        if (fin && breaks.empty()) break;
        if (breaks.empty() || round == kRepairRounds || Ku + breaks.size() > Kcap)
            return chain_break(fin ? "repairs exhausted" : "no final block", chain.back());
        std::sort(breaks.begin(), breaks.end());
        breaks.erase(std::unique(breaks.begin(), breaks.end()), breaks.end());
        // repair units, appended at [Ku, Ku + breaks)
        const uint64_t k0 = Ku;
        for (const auto& br : breaks) {
            // a repair that was already made there failed: the serial decoder reports why
            if (std::binary_search(repaired.begin(), repaired.end(), br))
                return chain_break("repair failed", chain.back());
            const uint64_t e = br.first;
            starts[Ku] = e;
            vmode[Ku] = br.second == FB_AT_HEADER ? FB_V_HEADER : FB_V_EXACT;
            vhdr[Ku] = br.second == FB_AT_HEADER ? 0 : br.second;
            stops[Ku] = stop_of(e);
            // inside a fixed-code region (after a stored block there, say): the true path's
            // chunk entries are known, so the repair unit's ranges start exactly on them too
            // Off (DMX_FB_REPAIR_EXACT, developer A/B): measured Z_FIXED 64 MiB text 4.7 -> 4.2 ms
            // but 32 MiB mixed 8.7 -> 13.4 ms (a repair unit after a stored block then ends
            // serially), also with soft stops only.
            ucb[Ku] = ~0u;
            if (DMX_FB_REPAIR_EXACT && dcbit && (stops[Ku] & FB_STOP_SOFT)) {
                auto rg = std::upper_bound(regs.begin(), regs.end(), e, [](uint64_t v, const Reg& g) { return v < g.E; });
                if (rg != regs.begin() && e < (--rg)->T)
                    ucb[Ku] = (uint32_t)((rg->sb0 + (e - rg->E) / kSuper) * 64);
            }
            const uint64_t w = (stops[Ku] & FB_STOP_SOFT) ? region_words((stops[Ku] & FB_STOP_MASK) - std::min(e, nbits))
                                                          : std::min(words_of(e, stops[Ku]), kOpenWords);
            if (rep_used + w > rep_words) return chain_break("repair token space", chain.back());
            tokoff[Ku + 1] = tokoff[Ku] + w;
            rep_used += w;
            Ku++;
        }
        repaired.insert(repaired.end(), breaks.begin(), breaks.end());
        std::sort(repaired.begin(), repaired.end());
        if (upload(k0, Ku - k0) != DMX_OK || decode(k0, Ku - k0) != DMX_OK) return DMX_ERR_DEVICE;
        if (fb_debug) {
            std::fprintf(stderr, "dmx fb: repair round %d: %llu units\n", round, (unsigned long long)(Ku - k0));
            if (dump_stats("after repair round", Ku) != DMX_OK) return DMX_ERR_DEVICE;
        }
    }
    // the path's own scratch first: when it does not fit, the stream still decodes on the
    // serial decoder, which needs only the output
    const uint64_t nch = chain.size();
    if (!c->fbch.ensure(nch * 4) || !c->fbco.ensure(nch * 8) || !c->fbcs.ensure(nch * 8) ||
        !c->fbimg.ensure(total * 2 + 16))
        return DMX_OK;
    *handled = true;
    *total_out = total;
    uint8_t* out = fixed_out;
    if (!out) {
        if (!c->out.ensure(total ? total : 1)) return DMX_ERR_NOMEM;
        out = c->out.as<uint8_t>();
    } else if (total > cap) {
        return DMX_ERR_CAPACITY;
    }
    hmark(5);
    c->pin_off = 0;  // (the chain walk followed a stream sync)
    HIPCHK(pin_h2d(c, c->fbch.p, chain.data(), nch * 4, st));
    HIPCHK(pin_h2d(c, c->fbco.p, coffs.data(), nch * 8, st));
    HIPCHK(pin_h2d(c, c->fbcs.p, csizes.data(), nch * 8, st));
    HIPCHK(hipMemsetAsync(&ds->fb_err, 0, 4, st));
    // the parallel window hand-off when its scratch fits (nch * 128 KiB), else the serial one
    uint32_t *win = nullptr, *open = nullptr;
    const uint64_t went = fb_window_entries(nch);
    if (went && !fb_serial_only(c) && c->fbwin.ensure(went * 4) && c->fbopen.ensure(fb_window_rounds(nch) * 4)) {
        win = c->fbwin.as<uint32_t>();
        open = c->fbopen.as<uint32_t>();
    }
    unsigned long long* uph = nullptr;
    if ((c->diag & DIAG_FB) && c->fbph.ensure(256)) {
        uph = c->fbph.as<unsigned long long>();
        HIPCHK(hipMemsetAsync(uph, 0, 64, st));
    }
    HIPCHK(launch_fb_resolve(d_in, c->fbs.as<uint64_t>(), c->fbch.as<uint32_t>(), c->fbco.as<uint64_t>(),
                             c->fbcs.as<uint64_t>(), nch, c->fbt.as<uint64_t>(), c->fbk.as<uint32_t>(),
                             c->fbu.as<FbUnit>(), c->fbimg.as<uint16_t>(), total, out, &ds->fb_err, win, open,
                             !fb_serial_only(c), uph, st));
    if (uph) {
        unsigned long long ph[5];
        HIPCHK(hipMemcpyAsync(ph, uph, sizeof(ph), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::fprintf(stderr, "dmx fb: k_fb_units cycles per unit: batches %llu, expansion %llu, jumping %llu (%llu rounds "
                     "in all), write-out %llu\n", ph[0] / nch, ph[1] / nch, ph[2] / nch, ph[4], ph[3] / nch);
    }
    hmark(6);
    if (c->diag & DIAG_FBT) {
        auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(ht[b] - ht[a]).count(); };
        std::fprintf(stderr, "dmx fb: host us: scan+check+starts %.1f, unit setup %.1f, upload %.1f, pass-1 decode "
                     "(launch to records) %.1f, chain walk %.1f, chain upload + launches %.1f\n", us(0, 1), us(1, 2),
                     us(2, 3), us(3, 4), us(4, 5), us(5, 6));
    }
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    uint32_t ferr = 0;
    HIPCHK(hipMemcpyAsync(&ferr, &ds->fb_err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ferr) {
        *handled = false;
        *total_out = 0;
        return DMX_OK;
    }
    c->stats.segments = nch;
    c->last_end = (units[chain.back()].end + 7) / 8;
    if (dev_out) *dev_out = out;
    return DMX_OK;
}

// Shared inflate driver.  fixed_out != nullptr: decode into the caller's device buffer of
// `cap` bytes.  Otherwise decode into c->out, grown as needed (*dev_out receives it).
// iflags: DMX_IFLAG_PIECE for one piece of a larger stream (dmx_inflate_piece_device).
int inflate_device_locked(dmx_ctx* c, const uint8_t* d_in, size_t n, uint8_t* fixed_out,
                          size_t cap, size_t* total_out, uint8_t** dev_out, hipStream_t st,
                          uint32_t iflags = 0) {
    // an asynchronous inflate still running uses the same scratch
    if (c->inf_pending) HIPCHK(hipStreamWaitEvent(st, c->ev_inf, 0));
    begin_timing(c, st);
    *total_out = 0;
    if (n == 0) return DMX_ERR_OVERREAD;  // the reference throws (or faults) on empty input
    if (!c->scal.ensure(sizeof(Scal))) return DMX_ERR_NOMEM;
    Scal* ds = c->scal.as<Scal>();
    const uint64_t misalign = (uintptr_t)d_in & 3;
    const uint32_t* words = reinterpret_cast<const uint32_t*>(d_in - misalign);

    // candidate segment starts
    const uint64_t ntiles = marker_tiles(n, misalign);
    if (!c->tiles.ensure(ntiles * 4) || !c->tileoffs.ensure(scan_words(ntiles) * 8)) return DMX_ERR_NOMEM;
    HIPCHK(launch_marker_count(words, misalign, n, c->tiles.as<uint32_t>(), ntiles, st));
    HIPCHK(launch_scan_u32(c->tiles.as<uint32_t>(), c->tileoffs.as<uint64_t>(), ntiles, &ds->nmarkers, st));
    uint64_t nmarkers = 0;
    HIPCHK(hipMemcpyAsync(&nmarkers, &ds->nmarkers, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t ncand = nmarkers + 1;
    if (!c->cands.ensure(ncand * 8) || !c->recs.ensure(ncand * sizeof(SegRecord)) ||
        !c->status.ensure(ncand * 8))
        return DMX_ERR_NOMEM;
    HIPCHK(launch_marker_write(words, misalign, n, c->tileoffs.as<uint64_t>(), ntiles,
                               c->cands.as<uint64_t>(), ~0ull, st));

    uint8_t* out = fixed_out;
    // The segment-parallel passes place candidate j at j * 32 KiB.  Every 00 00 FF FF inside
    // stored data is a candidate too, so a marker-dense stream can ask for more HBM than exists:
    // then the parallel plan is skipped and the serial decoder (sized by its count pass) runs.
    bool parallel_ok = true;
    if (!out) {
        size_t freeb = 0, totb = 0;
        if (hipMemGetInfo(&freeb, &totb) != hipSuccess) freeb = 0;
        const size_t want = ncand * (size_t)std::max<uint32_t>(kSegCap, c->seg);
        if ((want <= c->out.cap || want <= freeb / 2) && c->out.ensure(want)) {
            out = c->out.as<uint8_t>();
            cap = c->out.cap;
        } else {
            parallel_ok = false;
            if (!c->out.ensure(1)) return DMX_ERR_NOMEM;
            out = c->out.as<uint8_t>();
            cap = 0;
        }
    }
    InflateArgs A;
    A.in_words = words;
    A.misalign = misalign;
    A.n = n;
    A.cands = c->cands.as<uint64_t>();
    A.ncand = ncand;
    A.out = out;
    A.cap = cap;
    A.recs = c->recs.as<SegRecord>();
    A.status = c->status.as<unsigned long long>();
    A.ticket = &ds->ticket;
    A.flags = c->flags | iflags;
    A.dbg = phase_buf(c, ncand);
    InflateResult r{};
    // Plan: the lane decoder (one lane per segment decodes tokens, one wave per segment
    // resolves them; segment j lands at j * seg) with a patch pass of the exact wave decoder
    // for the candidates it declines; then the older workgroup-per-segment decoder with both
    // segment sizes; then the wave-per-segment decoder, which places segments of any size
    // <= 32 KiB by look-back.  Each pass runs only if the previous one reported status 1 (a
    // segment outside its layout or sizes not uniform); status 2 goes to the serial decoder.
    const int path_env = c->inflate_pass;  // developer A/B (dmx_config.dev_inflate_pass)
    // Heavy candidates (mode 6): a lane decodes about one symbol per 1000 cycles, so the lane
    // decoder takes as long as the serial decode of the densest segment in a wave (a 24 MiB
    // bitmap: 6 ms for ~10K symbols).  Candidates spanning more than heavy_bytes compressed
    // bytes go to the workgroup decoder instead (k_inflate_pj: the segment's bits split over 512
    // lanes, ~0.17 ms per dense segment on one CU): always up to 2048 candidates, beyond that
    // when the device-side count finds at most 32 per CU (32 rounds of workgroups, ~5.5 ms;
    // more dense segments than that keep the lanes' throughput: 1 GiB of text).
    // A stream of at most one candidate per CU takes one round of workgroups, which beats the
    // lanes' ~0.3 ms floor (a wave's header, table and token phases) from 256 bytes up.
    const bool heavy_env = c->heavy_bytes != 0;
    const uint32_t heavy_bytes = heavy_env ? c->heavy_bytes : 2048u;
    const bool few_bits = n / ncand < 4096;
    uint32_t plan[8][2];
    int np = 0;
    r.status = 2;
    uint32_t heavy = 0, heavy_limit = 0;
    if (path_env == -1 || path_env == 4) {
        // k_lane_caps: min(8 bits, slot / 2 + 2) + 16 words per candidate, in groups of four
        const uint64_t per = (std::max<uint64_t>(LN_OUT_CAP_BYTES, c->seg) / 2 + 2 + 16 + 3) & ~3ull;
        const uint64_t words = std::min<uint64_t>(ncand * per, 8ull * n + 20ull * ncand);
        auto lane_bufs = [&]() {
            return c->ltok.ensure(words * 4) && c->ltokoff.ensure(scan_words(ncand) * 8) &&
                   c->lntok.ensure(ncand * 4) && c->lcaps.ensure(ncand * 4) && c->lsplit.ensure(ncand * 4 + 8);
        };
        // short of device memory: drop the scratch this call does not use (the deflate's token
        // words and slots, path 5's token space and images, chain-repair scratch) and try again
        // before the plan goes past the lane decoder
        bool lanes_ok = lane_bufs();
        if (!lanes_ok) {
            for (DevBuf* b : {&c->dtok, &c->slots, &c->rtmp, &c->fbt, &c->fbimg, &c->fbwin, &c->fbopen, &c->fbk,
                              &c->fbu, &c->fbJ, &c->fbJraw, &c->fbJsub})
                b->release();
            lanes_ok = lane_bufs();
        }
        if (lanes_ok) {
            plan[np][0] = 4, plan[np][1] = c->seg, np++;
            // (the workgroup decoder of the heavy route takes segments of <= 32 KiB)
            if (heavy_bytes && c->seg <= 32768 && ncand < 0xFFFFFFF0ull && c->lheavy.ensure((ncand + 2) * 4)) {
                if (c->ncu <= 0 && hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
                    c->ncu = 256;
                heavy = (!heavy_env && ncand <= (uint64_t)c->ncu) ? 256u : heavy_bytes;
                heavy_limit = ncand <= 2048 ? 0xFFFFFFFFu : 32u * (uint32_t)std::max(c->ncu, 1);
                plan[np][0] = 6, plan[np][1] = c->seg, np++;  // the heavy candidates
            }
            plan[np][0] = 3, plan[np][1] = c->seg, np++;  // patch the declined candidates
        }
    }
    if (path_env == 0 || path_env == 1) {
        plan[np][0] = (uint32_t)path_env, plan[np][1] = 0, np++;
    } else if (path_env == 4) {
    } else if (few_bits && path_env != 2) {
        plan[np][0] = 0, plan[np][1] = 0, np++;
    } else if (c->seg <= 32768) {  // (the workgroup decoder's slots are 16 or 32 KiB)
        plan[np][0] = 2, plan[np][1] = c->seg, np++;
        plan[np][0] = 3, plan[np][1] = c->seg, np++;
        plan[np][0] = 2, plan[np][1] = c->seg == 32768 ? 16384u : 32768u, np++;
        plan[np][0] = 3, plan[np][1] = c->seg == 32768 ? 16384u : 32768u, np++;
    }
    if (path_env != 1 && path_env != 4) plan[np][0] = 1, plan[np][1] = 0, np++;
    uint32_t lead_mode = 0;
    if (!parallel_ok) np = 0;
    // no marker in a large stream: not libdmx's segment layout, the block-parallel path next
    if (ncand == 1 && n > 65536 && path_env == -1) np = 0;
    if (path_env == 5 || path_env == 7) np = 0;  // 7: the serial decoder alone
    // the plan's passes into A.out / A.cap; returns the last validation result
    auto run_plan = [&](InflateResult& r) -> int {
        r.status = 2;
        for (int pi = 0; pi < np; pi++) {
            const uint32_t mode = plan[pi][0];
            if (mode == 3 && (r.exotic == 0 || r.exotic > ncand / 8)) continue;  // nothing / too many
            if (mode == 6 && r.exotic == 0) continue;
            A.mode = mode;
            A.slot = plan[pi][1];
            // main-kernel window: from the first pass's launch to the end of the last pass run
            hipEvent_t e0 = (c->timing && pi == 0) ? c->ev[1] : nullptr, e1 = c->timing ? c->ev[2] : nullptr;
            if (mode != 3 && mode != 6) lead_mode = mode;
            if (mode == 4) {
                HIPCHK(launch_inflate_lanes(A, c->ltok.as<uint32_t>(), c->ltokoff.as<uint64_t>(),
                                            c->lntok.as<uint32_t>(), c->lcaps.as<uint32_t>(), heavy,
                                            heavy_limit, c->lheavy.as<uint32_t>(), c->lsplit.as<uint32_t>(), st, e0,
                                            e1));
            } else if (mode == 6) {
                const uint32_t grid = (uint32_t)std::min<uint64_t>(r.exotic, (uint64_t)std::max(c->ncu, 1));
                HIPCHK(launch_inflate_pj_list(A, A.slot, c->lheavy.as<uint32_t>(), grid, st, e1));
            } else if (mode == 2) {
                HIPCHK(launch_inflate_pj(A, A.slot, st, e0, e1));
            } else {
                HIPCHK(hipMemsetAsync(A.status, 0, ncand * 8, st));
                HIPCHK(hipMemsetAsync(&ds->ticket, 0, 4, st));
                HIPCHK(launch_inflate_segments(A, st, e0, e1));
            }
            HIPCHK(launch_inflate_validate(A, &ds->vw, &ds->res, st));
            if (A.dbg) phase_dump(c, "inflate", ncand, st);
            HIPCHK(hipMemcpyAsync(&r, &ds->res, sizeof r, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (c->diag & DIAG_RECS) {  // developer aid: per-candidate outcome of this pass
                std::vector<SegRecord> h(ncand);
                (void)hipMemcpy(h.data(), A.recs, ncand * sizeof(SegRecord), hipMemcpyDeviceToHost);
                uint64_t fl[8] = {0}, shown = 0;
                for (uint64_t i = 0; i < ncand; i++) {
                    for (int b = 0; b < 8; b++) fl[b] += (h[i].flags >> b) & 1;
                    if ((h[i].flags & ~1u) && shown++ < 8)
                        std::fprintf(stderr, "dmx: mode %u cand %llu flags %u size %u end %llu\n", mode,
                                     (unsigned long long)i, h[i].flags, h[i].out_size,
                                     (unsigned long long)h[i].end_byte);
                }
                std::fprintf(stderr, "dmx: mode %u ncand %llu status %u flags fin %llu data %llu over %llu ovf %llu xref %llu tmo %llu exo %llu\n",
                             mode, (unsigned long long)ncand, r.status, (unsigned long long)fl[0], (unsigned long long)fl[1],
                             (unsigned long long)fl[2], (unsigned long long)fl[3], (unsigned long long)fl[4],
                             (unsigned long long)fl[5], (unsigned long long)fl[6]);
            }
            if (r.status != 1) break;  // 1: not this layout
            // the lane pass decoded every candidate but the segment sizes are not uniform (a
            // shard ending on a short segment, 16 KiB segments): the chain repair below
            // places them, the other passes would only decode everything again
            if (lead_mode == 4 && r.exotic == 0 && (mode == 4 || mode == 6 || mode == 3)) break;
        }
        return DMX_OK;
    };
    {
        const int rc = run_plan(r);
        if (rc != DMX_OK) return rc;
    }
    c->stats.segments = ncand;
    c->stats.in_bytes = n;
    if (r.status == 0) {
        end_timing(c, st);
        c->last_end = r.end_byte;
        c->stats.path = lead_mode == 4 ? 4 : lead_mode >= 2 ? 3 : lead_mode;
        c->stats.out_bytes = r.total;
        *total_out = r.total;
        if (dev_out) *dev_out = out;
        return r.total > cap ? DMX_ERR_CAPACITY : DMX_OK;
    }
    // Chain repair.  A "00 00 FF FF" inside stored data (random data: once per ~4 GiB) is a
    // candidate no segment starts at, so the candidate chain skips it and every later segment
    // sits one slot too far; the whole stream used to go to the serial decoder (hours at
    // multi-GiB sizes).  Segments of other sizes than the slot (a short segment in the middle,
    // 16 KiB segments) are placed the same way.  The records say where each segment ends: the host walks the chain
    // from candidate 0 (each segment's end must be a candidate start, up to the first BFINAL),
    // the segments are decoded into a scratch buffer at their slots if the first decode did
    // not hold every slot, and one kernel moves the chain's segments to their offsets.
    if (r.status != 0 && lead_mode == 4 && parallel_ok && ncand > 1) {
        std::vector<SegRecord> h(ncand);
        std::vector<uint64_t> hc(ncand);
        HIPCHK(hipMemcpyAsync(h.data(), A.recs, ncand * sizeof(SegRecord), hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(hc.data(), A.cands, ncand * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::vector<uint64_t> chain, coffs;
        std::vector<uint32_t> csz;
        uint64_t tot = 0, k = 0;
        bool ok = false;
        for (;;) {
            const SegRecord& s = h[k];
            if (s.flags & ~SEGF_FINAL) break;
            chain.push_back(k);
            coffs.push_back(tot);
            csz.push_back(s.out_size);
            tot += s.out_size;
            if (s.flags & SEGF_FINAL) { ok = true; break; }
            const auto it = std::lower_bound(hc.begin() + k + 1, hc.end(), s.end_byte);
            if (it == hc.end() || *it != s.end_byte) break;
            k = (uint64_t)(it - hc.begin());
        }
        uint64_t slot = A.slot ? A.slot : c->seg;
        // (when the repair's own scratch does not fit, the stream still decodes on path 5 or the
        // serial decoder, which need only the output: ADVICE r3)
        uint8_t* const a_out = A.out;
        const uint64_t a_cap = A.cap;
        do {
            if (!ok) break;
            if (fixed_out && tot > cap) return DMX_ERR_CAPACITY;
            uint8_t* dst = fixed_out ? fixed_out : out;
            const uint64_t need = (chain.back() + 1) * slot;
            const uint32_t maxsz = *std::max_element(csz.begin(), csz.end());
            const uint8_t* src = out;
            uint8_t* place = dst;  // where the kernel writes; then copied to dst if scratch
            if (need > A.cap || maxsz > slot) {
                // slots past the buffer were not written, or segments larger than the slot
                // overlapped: decode again into scratch with 32 KiB slots, place into dst
                if (maxsz > slot) {
                    slot = LN_OUT_CAP_BYTES;
                    for (int pi = 0; pi < np; pi++)
                        if (plan[pi][0] == 4 || plan[pi][0] == 6 || plan[pi][0] == 3) plan[pi][1] = (uint32_t)slot;
                }
                if (!c->rtmp.ensure(ncand * slot)) break;
                A.out = c->rtmp.as<uint8_t>();
                A.cap = ncand * slot;
                InflateResult r2{};
                const int rc = run_plan(r2);
                if (rc != DMX_OK) return rc;
                src = A.out;
            } else {  // every slot is in `out` (== dst): place into scratch, copy back
                if (!c->rtmp.ensure(tot ? tot : 1)) break;
                place = c->rtmp.as<uint8_t>();
            }
            const uint64_t nch = chain.size();
            if (!c->rchain.ensure(nch * 20)) break;
            uint64_t* dch = c->rchain.as<uint64_t>();
            uint64_t* doffs = dch + nch;
            uint32_t* dsz = reinterpret_cast<uint32_t*>(doffs + nch);
            HIPCHK(hipMemcpyAsync(dch, chain.data(), nch * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(doffs, coffs.data(), nch * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(dsz, csz.data(), nch * 4, hipMemcpyHostToDevice, st));
            HIPCHK(launch_place_segments(src, (uint32_t)slot, dch, doffs, dsz, nch, place, st));
            if (place != dst && tot) HIPCHK(hipMemcpyAsync(dst, place, tot, hipMemcpyDeviceToDevice, st));
            if (c->timing) (void)hipEventRecord(c->ev[2], st);
            HIPCHK(hipStreamSynchronize(st));
            end_timing(c, st);
            c->last_end = h[chain.back()].end_byte;
            c->stats.path = 4;
            c->stats.out_bytes = tot;
            *total_out = tot;
            if (dev_out) *dev_out = dst;
            return DMX_OK;
        } while (0);
        A.out = a_out;  // not repaired: the later paths decode into the caller's buffer
        A.cap = a_cap;
    }

    if (path_env == -1 || path_env == 5) {
        bool handled = false;
        const int rc = inflate_fb_locked(c, d_in, n, fixed_out, cap, total_out, dev_out, st, &handled, iflags);
        if (handled) {
            end_timing(c, st);
            c->stats.path = 5;
            c->stats.in_bytes = n;
            c->stats.out_bytes = *total_out;
            return rc;
        }
    }
    // serial path: one pass into the caller's buffer, or into c->out sized generously (bytes
    // past the capacity are counted, not written); a second pass only when that did not fit
    c->stats.path = 2;
    if (c->timing) (void)hipEventRecord(c->ev[1], st);
    uint64_t dummy_dbg = 0;
    A.dbg = (c->diag & DIAG_FB) ? &dummy_dbg : nullptr;  // (a flag for the kernel: count phases)
    if (!fixed_out) {
        size_t freeb = 0, totb = 0;
        if (hipMemGetInfo(&freeb, &totb) != hipSuccess) freeb = 0;
        // a generous first buffer saves the second pass on high-ratio streams, but it is kept
        // by the context: bounded by 4 GiB (64 n alone held ~72 GiB for a 1 GiB
        // stream); a larger output is counted by the first pass and decoded by a second
        const uint64_t guess = std::min<uint64_t>({64ull * n + (16ull << 20), 4ull << 30, freeb / 4});
        if (c->out.cap < guess && !c->out.ensure(guess)) (void)c->out.ensure(1);
        A.out = c->out.as<uint8_t>();
        A.cap = c->out.p ? c->out.cap : 0;
    } else {
        A.out = fixed_out;
        A.cap = cap;
    }
    HIPCHK(launch_inflate_serial(A, 0, &ds->res, st));
    if (c->timing) (void)hipEventRecord(c->ev[2], st);
    HIPCHK(hipMemcpyAsync(&r, &ds->res, sizeof r, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (r.status != 0) return r.status;
    if (r.total > A.cap) {
        if (fixed_out) return DMX_ERR_CAPACITY;
        if (!c->out.ensure(r.total)) return DMX_ERR_NOMEM;
        A.out = c->out.as<uint8_t>();
        A.cap = c->out.cap;
        HIPCHK(launch_inflate_serial(A, 0, &ds->res, st));
        if (c->timing) (void)hipEventRecord(c->ev[2], st);
        HIPCHK(hipMemcpyAsync(&r, &ds->res, sizeof r, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    end_timing(c, st);
    if (c->diag & DIAG_FB)
        std::fprintf(stderr, "dmx serial: cycles %llu %llu %llu %llu %llu, regions %llu; walk phases %llu %llu %llu %llu %llu, "
                     "rounds %llu (k_inflate_serial_wg: doubling, members+scan+cuts, parallel writes, wave-0 copies + "
                     "flush, decode + walks; walks: first pass, rounds, output sums, writes, dependent copies)\n",
                     (unsigned long long)r.cycles[0], (unsigned long long)r.cycles[1], (unsigned long long)r.cycles[2],
                     (unsigned long long)r.cycles[3], (unsigned long long)r.cycles[4], (unsigned long long)r.cycles[5],
                     (unsigned long long)r.cycles[6], (unsigned long long)r.cycles[7], (unsigned long long)r.cycles[8],
                     (unsigned long long)r.cycles[9], (unsigned long long)r.cycles[10], (unsigned long long)r.cycles[11]);
    *total_out = r.total;
    c->last_end = r.end_byte;
    c->stats.out_bytes = r.total;
    if (dev_out) *dev_out = A.out;
    return r.status;
}

// dmx_inflate_device_async: the lane path (path 4) of a libdmx-layout stream with no host
// synchronisation.  The candidate count stays on the device: the scratch is provisioned for
// cap / segment + 64 candidates (a libdmx stream has one per segment), the grids are sized for
// that many and every kernel stops at the device-side count.  No heavy route, no patch pass,
// no chain repair: any stream the lanes do not decode whole -- another layout, a declined
// segment, more candidates than provisioned, output beyond cap -- ends with status 1 in
// d_result[1], and the caller decodes it with dmx_inflate_device.
int inflate_device_async_locked(dmx_ctx* c, const uint8_t* d_in, size_t n, uint8_t* d_out, size_t cap,
                                uint64_t* d_result, hipStream_t st, uint32_t iflags) {
    static const uint64_t fail[2] = {0, 1};
    if (c->inf_pending) HIPCHK(hipStreamWaitEvent(st, c->ev_inf, 0));
    if (n == 0) {
        HIPCHK(hipMemcpyAsync(d_result, fail, 16, hipMemcpyHostToDevice, st));
        return DMX_OK;
    }
    if (!c->scal.ensure(sizeof(Scal))) return DMX_ERR_NOMEM;
    Scal* ds = c->scal.as<Scal>();
    const uint64_t misalign = (uintptr_t)d_in & 3;
    const uint32_t* words = reinterpret_cast<const uint32_t*>(d_in - misalign);
    const uint64_t slot = c->seg;
    const uint64_t ncap = cap / slot + 64;
    const uint64_t ntiles = marker_tiles(n, misalign);
    const uint64_t per = (std::max<uint64_t>(LN_OUT_CAP_BYTES, slot) / 2 + 2 + 16 + 3) & ~3ull;
    const uint64_t words_tok = std::min<uint64_t>(ncap * per, 8ull * n + 20ull * ncap);
    if (!c->tiles.ensure(ntiles * 4) || !c->tileoffs.ensure(scan_words(ntiles) * 8) || !c->cands.ensure(ncap * 8) ||
        !c->recs.ensure(ncap * sizeof(SegRecord)) || !c->status.ensure(ncap * 8) || !c->ltok.ensure(words_tok * 4) ||
        !c->ltokoff.ensure(scan_words(ncap) * 8) || !c->lntok.ensure(ncap * 4) || !c->lcaps.ensure(ncap * 4) ||
        !c->lsplit.ensure(ncap * 4 + 8))
        return DMX_ERR_NOMEM;
    HIPCHK(launch_marker_count(words, misalign, n, c->tiles.as<uint32_t>(), ntiles, st));
    HIPCHK(launch_scan_u32(c->tiles.as<uint32_t>(), c->tileoffs.as<uint64_t>(), ntiles, &ds->nmarkers, st));
    HIPCHK(launch_async_prep(&ds->nmarkers, &ds->ncand, st));
    HIPCHK(launch_marker_write(words, misalign, n, c->tileoffs.as<uint64_t>(), ntiles, c->cands.as<uint64_t>(), ncap,
                               st));
    InflateArgs A;
    A.in_words = words;
    A.misalign = misalign;
    A.n = n;
    A.cands = c->cands.as<uint64_t>();
    A.ncand = ncap;
    A.ncand_dev = &ds->ncand;
    A.out = d_out;
    A.cap = cap;
    A.recs = c->recs.as<SegRecord>();
    A.status = c->status.as<unsigned long long>();
    A.ticket = &ds->ticket;
    A.flags = c->flags | iflags;
    A.mode = 4;
    A.slot = (uint32_t)slot;
    A.dbg = nullptr;
    HIPCHK(launch_inflate_lanes(A, c->ltok.as<uint32_t>(), c->ltokoff.as<uint64_t>(), c->lntok.as<uint32_t>(),
                                c->lcaps.as<uint32_t>(), 0, 0, nullptr, c->lsplit.as<uint32_t>(), st, nullptr, nullptr));
    HIPCHK(launch_inflate_validate(A, &ds->vw, &ds->res, st));
    HIPCHK(launch_async_result(&ds->res, &ds->ncand, ncap, cap, d_result, st));
    HIPCHK(hipEventRecord(c->ev_inf, st));
    c->inf_pending = true;
    return DMX_OK;
}

// Adler-32 / CRC-32 of a device buffer, computed on the GPU (checksum.hip); the value is
// returned to the host (the call synchronizes the stream).
int checksum_locked(dmx_ctx* c, bool crc, const uint8_t* d, size_t n, uint32_t init, uint32_t* out,
                    hipStream_t st) {
    if (!c->ck.ensure(256 + checksum_scratch_bytes(n))) return DMX_ERR_NOMEM;
    uint32_t* d_res = c->ck.as<uint32_t>();
    void* scratch = c->ck.as<uint8_t>() + 256;
    if (crc) HIPCHK(launch_crc32_raw(d, n, scratch, d_res, st));
    else HIPCHK(launch_adler32(d, n, init, scratch, d_res, st));
    uint32_t v = 0;
    HIPCHK(hipMemcpyAsync(&v, d_res, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *out = crc ? crc32_finish(v, n, init) : v;
    return DMX_OK;
}

// zlib (RFC 1950) / gzip (RFC 1952) framing around libdmx's raw stream; the checksum of the
// input is computed on the GPU from the device copy the deflate reads.
int deflate_framed(dmx_ctx* c, bool gz, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                   size_t* out_len) {
    const size_t head = gz ? 10 : 2, tail = gz ? 8 : 4;
    *out_len = 0;
    const size_t bound = dmx_deflate_bound(n);
    if (!c->in.ensure(n + 16) || !c->out.ensure(bound)) return DMX_ERR_NOMEM;
    if (n) HIPCHK(hipMemcpyAsync(c->in.p, in, n, hipMemcpyHostToDevice, c->stream));
    size_t total = 0;
    int rc = deflate_device_locked(c, c->in.as<uint8_t>(), n, level, 0, c->out.as<uint8_t>(), c->out.cap,
                                   &total, c->stream);
    if (rc != DMX_OK) return rc;
    uint32_t ck = 0;
    rc = checksum_locked(c, gz, c->in.as<uint8_t>(), n, gz ? 0u : 1u, &ck, c->stream);
    if (rc != DMX_OK) return rc;
    *out_len = head + total + tail;
    if (head + total + tail > cap) return DMX_ERR_CAPACITY;
    const int lv = (level < 0 || level > 3) ? 1 : level;
    if (gz) {
        const uint8_t h[10] = {0x1F, 0x8B, 8, 0, 0, 0, 0, 0, (uint8_t)(lv == 3 ? 2 : lv <= 1 ? 4 : 0), 255};
        std::memcpy(out, h, 10);
    } else {
        const uint32_t flevel = lv <= 1 ? 0 : lv == 2 ? 1 : 3;  // RFC 1950 FLEVEL
        const uint32_t cmf = 0x78, flg0 = flevel << 6;
        const uint32_t flg = flg0 + (31 - (cmf * 256 + flg0) % 31) % 31;
        out[0] = (uint8_t)cmf;
        out[1] = (uint8_t)flg;
    }
    if (total) HIPCHK(hipMemcpyAsync(out + head, c->out.p, total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    uint8_t* t = out + head + total;
    if (gz) {
        for (int b = 0; b < 4; b++) t[b] = (uint8_t)(ck >> (8 * b));
        for (int b = 0; b < 4; b++) t[4 + b] = (uint8_t)((uint64_t)n >> (8 * b));
    } else {
        for (int b = 0; b < 4; b++) t[b] = (uint8_t)(ck >> (24 - 8 * b));
    }
    return DMX_OK;
}

// Restores the calling thread's current HIP device on scope exit: an entry point switches to
// its context's device, and a caller driving several GPUs from one thread must not see its
// current device move.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = prev == dev || hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---- n_gpus > 1: the host-buffer API over several devices ---------------------
// Deflate: contiguous segment-aligned shards, one per sub-context, each deflated NOT_FINAL except
// the last non-empty one; one host thread per shard (the pageable H2D / D2H copies of different
// devices then overlap), sizes first, then every shard's bytes straight to its offset in `out`.
// Segments are independent (the reference resets its window per chunk, deflate.hpp:689-697), so
// the bytes equal the one-device stream.
template <class F>
void run_parallel(size_t G, F&& f) {
    std::vector<std::thread> th;
    for (size_t g = 1; g < G; g++) th.emplace_back(f, g);
    f((size_t)0);
    for (auto& t : th) t.join();
}

int deflate_multi(dmx_ctx* c, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                  size_t* out_len) {
    const size_t G = c->subs.size(), seg = c->seg;
    size_t per = (n + G - 1) / G;
    per = (per + seg - 1) / seg * seg;
    std::vector<size_t> b(G), e(G), len(G, 0);
    std::vector<int> rc(G, DMX_OK);
    size_t last = 0, used = 0;
    for (size_t g = 0; g < G; g++) {
        b[g] = std::min(n, g * per);
        e[g] = std::min(n, b[g] + per);
        if (e[g] > b[g]) last = g, used++;
    }
    run_parallel(G, [&](size_t g) {
        if (e[g] == b[g]) return;
        dmx_ctx* s = c->subs[g];
        std::lock_guard<std::mutex> lk(s->mu);
        DeviceGuard dg(s->device);
        const size_t m = e[g] - b[g];
        if (!dg.ok) rc[g] = DMX_ERR_DEVICE;
        else if (!s->in.ensure(m + 16) || !s->out.ensure(dmx_deflate_bound(m))) rc[g] = DMX_ERR_NOMEM;
        else if (hipMemcpyAsync(s->in.p, in + b[g], m, hipMemcpyHostToDevice, s->stream) != hipSuccess) rc[g] = DMX_ERR_DEVICE;
        else rc[g] = deflate_device_locked(s, s->in.as<uint8_t>(), m, level, g == last ? 0u : DMX_DEFLATE_NOT_FINAL,
                                           s->out.as<uint8_t>(), s->out.cap, &len[g], s->stream);
    });
    size_t total = 0;
    for (size_t g = 0; g < G; g++) {
        if (rc[g] != DMX_OK) return rc[g];
        total += len[g];
    }
    *out_len = total;
    if (total > cap) return DMX_ERR_CAPACITY;
    std::vector<size_t> off(G, 0);
    for (size_t g = 1; g < G; g++) off[g] = off[g - 1] + len[g - 1];
    run_parallel(G, [&](size_t g) {
        if (!len[g]) return;
        dmx_ctx* s = c->subs[g];
        DeviceGuard dg(s->device);
        if (hipMemcpyAsync(out + off[g], s->out.p, len[g], hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess)
            rc[g] = DMX_ERR_DEVICE;
    });
    for (size_t g = 0; g < G; g++)
        if (rc[g] != DMX_OK) return rc[g];
    c->stats = dmx_stats{};
    c->stats.in_bytes = n;
    c->stats.out_bytes = total;
    c->stats.shards = (uint32_t)used;
    return DMX_OK;
}

// Inflate: sub-context 0 indexes the candidate segment starts (the bytes after every 00 00 FF FF)
// and proves cuts near equal shares of them with a piece-mode decode of the segment there (it must
// end on another candidate: a marker inside stored data is no cut); every sub-context decodes its
// piece (closed with an empty final block; pieces after the first in piece mode, where a
// reference before the piece is an error), then the outputs land at their offsets: in `out`
// (at most cap bytes, *written) or in a malloc'd buffer (*alloc).  Returns 1 when the stream does
// not split (fewer than G proven cuts' worth of candidates, or a piece fails): the caller then
// decodes it on one device, so the result never depends on the split.
int inflate_multi(dmx_ctx* c, const uint8_t* in, size_t n, uint8_t* out, size_t cap, uint8_t** alloc,
                  size_t* written, size_t* total_out) {
    const size_t G = c->subs.size();
    dmx_ctx* s0 = c->subs[0];
    std::vector<uint64_t> starts;
    {
        DeviceGuard dg(s0->device);
        if (!dg.ok) return 1;
        {
            std::lock_guard<std::mutex> lk(s0->mu);
            if (!s0->in.ensure(n + 16) || hipMemcpyAsync(s0->in.p, in, n, hipMemcpyHostToDevice, s0->stream) != hipSuccess)
                return 1;
        }
        size_t cnt = 0;
        if (dmx_segment_starts_device(s0, s0->in.p, n, nullptr, 0, &cnt, nullptr) != DMX_OK || cnt + 1 < 2 * G) return 1;
        starts.resize(cnt);
        if (dmx_segment_starts_device(s0, s0->in.p, n, starts.data(), cnt, &cnt, nullptr) != DMX_OK) return 1;
        // cut candidates: up to 8 around each target, proven in one batched check
        std::vector<uint64_t> near;
        for (size_t r = 1; r < G; r++) {
            const size_t t = r * starts.size() / G;
            for (size_t j = (t >= 4 ? t - 4 : 0); j < std::min(starts.size(), t + 4); j++)
                if (starts[j] < n) near.push_back(starts[j]);
        }
        std::sort(near.begin(), near.end());
        near.erase(std::unique(near.begin(), near.end()), near.end());
        std::vector<uint64_t> ends(near.size());
        if (dmx_segment_check_device(s0, s0->in.p, n, near.data(), near.size(), ends.data(), nullptr) != DMX_OK) return 1;
        std::vector<uint64_t> ok;
        for (size_t i = 0; i < near.size(); i++)
            if (ends[i] != UINT64_MAX && ends[i] > near[i] &&
                (ends[i] == n || std::binary_search(starts.begin(), starts.end(), ends[i])))
                ok.push_back(near[i]);
        std::vector<uint64_t> cut{0};
        for (size_t r = 1; r < G; r++) {
            const uint64_t target = starts[r * starts.size() / G];
            uint64_t best = 0, bd = UINT64_MAX;
            for (uint64_t x : ok)
                if (x > cut.back() && (x > target ? x - target : target - x) < bd) best = x, bd = x > target ? x - target : target - x;
            if (!best) return 1;
            cut.push_back(best);
        }
        cut.push_back(n);
        starts = cut;
    }
    std::vector<size_t> len(G, 0);
    std::vector<int> rc(G, DMX_OK);
    std::vector<uint8_t*> dev(G, nullptr);
    run_parallel(G, [&](size_t g) {
        dmx_ctx* s = c->subs[g];
        std::lock_guard<std::mutex> lk(s->mu);
        DeviceGuard dg(s->device);
        const size_t a = starts[g], m = starts[g + 1] - a;
        static const uint8_t close[2] = {0x03, 0x00};  // an empty final block ends the piece
        const bool closes = g + 1 < G;
        if (!dg.ok || !s->in.ensure(m + 16) ||
            hipMemcpyAsync(s->in.p, in + a, m, hipMemcpyHostToDevice, s->stream) != hipSuccess ||
            (closes && hipMemcpyAsync(s->in.as<uint8_t>() + m, close, 2, hipMemcpyHostToDevice, s->stream) != hipSuccess)) {
            rc[g] = DMX_ERR_DEVICE;
            return;
        }
        s->last_end = 0;
        rc[g] = inflate_device_locked(s, s->in.as<uint8_t>(), m + (closes ? 2 : 0), nullptr, 0, &len[g], &dev[g],
                                      s->stream, g ? DMX_IFLAG_PIECE : 0u);
        // a piece must end at its appended empty final block: a BFINAL block before it (two
        // streams concatenated: the reference stops at the first) would drop the piece's rest
        if (rc[g] == DMX_OK && closes && s->last_end != m + 2) rc[g] = DMX_ERR_DATA;
    });
    for (size_t g = 0; g < G; g++)
        if (rc[g] != DMX_OK) return 1;
    size_t total = 0;
    std::vector<size_t> off(G, 0);
    for (size_t g = 0; g < G; g++) {
        off[g] = total;
        total += len[g];
    }
    uint8_t* dst = out;
    size_t lim = cap;
    if (alloc) {
        dst = static_cast<uint8_t*>(std::malloc(total ? total : 1));
        if (!dst) return DMX_ERR_NOMEM;
        lim = total;
    }
    run_parallel(G, [&](size_t g) {
        const size_t w = off[g] >= lim ? 0 : std::min(len[g], lim - off[g]);
        if (!w) return;
        dmx_ctx* s = c->subs[g];
        DeviceGuard dg(s->device);
        if (hipMemcpyAsync(dst + off[g], dev[g], w, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess)
            rc[g] = DMX_ERR_DEVICE;
    });
    for (size_t g = 0; g < G; g++)
        if (rc[g] != DMX_OK) {
            if (alloc) std::free(dst);
            return DMX_ERR_DEVICE;
        }
    if (alloc) *alloc = dst;
    if (written) *written = std::min(total, lim);
    *total_out = total;
    c->stats = dmx_stats{};
    c->stats.in_bytes = n;
    c->stats.out_bytes = total;
    c->stats.path = 4;
    c->stats.shards = (uint32_t)G;
    return DMX_OK;
}

bool is_gfx950(int dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
    return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace

extern "C" {

void dmx_config_default(dmx_config* cfg) {
    cfg->device = -1;
    cfg->segment_bytes = 32768;
    cfg->flags = 0;
    cfg->n_gpus = 1;
    cfg->dev_inflate_pass = 0;
    cfg->dev_heavy_bytes = 0;
}

int dmx_create(dmx_ctx** out, const dmx_config* cfg) {
    if (!out) return DMX_ERR_ARG;
    *out = nullptr;
    dmx_config d;
    dmx_config_default(&d);
    if (!cfg) cfg = &d;
    if (cfg->segment_bytes != 16384 && cfg->segment_bytes != 32768 && cfg->segment_bytes != 65536) return DMX_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DMX_ERR_DEVICE;
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return DMX_ERR_DEVICE;
    if (dev >= ndev || !is_gfx950(dev)) return DMX_ERR_DEVICE;
    // n_gpus: at most 8 shards per visible device (a stale or garbage value -- a caller built
    // against an older dmx_config -- would otherwise create contexts without bound)
    if (cfg->n_gpus > 8u * (uint32_t)ndev) return DMX_ERR_ARG;
    DeviceGuard dg(dev);
    if (!dg.ok) return DMX_ERR_DEVICE;
    dmx_ctx* c = new (std::nothrow) dmx_ctx();
    if (!c) return DMX_ERR_NOMEM;
    c->device = dev;
    c->seg = cfg->segment_bytes;
    c->flags = cfg->flags;
    c->inflate_pass = (int)cfg->dev_inflate_pass - 1;
    c->heavy_bytes = cfg->dev_heavy_bytes;
    c->diag = diag_env().bits;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return DMX_ERR_DEVICE;
    }
    for (auto& e : c->ev) (void)hipEventCreate(&e);
    if (hipEventCreateWithFlags(&c->ev_df, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_inf, hipEventDisableTiming) != hipSuccess) {
        dmx_destroy(c);
        return DMX_ERR_DEVICE;
    }
    if (cfg->n_gpus > 1) {  // one context per shard, round-robin over the visible devices
        dmx_config sc = *cfg;
        sc.n_gpus = 1;
        for (uint32_t i = 0; i < cfg->n_gpus; i++) {
            sc.device = (dev + (int)i) % ndev;
            dmx_ctx* s = nullptr;
            const int rc = is_gfx950(sc.device) ? dmx_create(&s, &sc) : DMX_ERR_DEVICE;
            if (rc != DMX_OK) {
                dmx_destroy(c);
                return rc;
            }
            c->subs.push_back(s);
        }
    }
    *out = c;
    return DMX_OK;
}

void dmx_destroy(dmx_ctx* c) {
    if (!c) return;
    for (dmx_ctx* s : c->subs) dmx_destroy(s);
    c->subs.clear();
    DeviceGuard dg(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (DevBuf* b : {&c->in, &c->out, &c->slots, &c->sizes, &c->offs, &c->scal, &c->cands,
                      &c->tiles, &c->tileoffs, &c->recs, &c->status, &c->dbg, &c->ltok,
                      &c->ltokoff, &c->lntok, &c->lcaps, &c->lheavy, &c->rtmp, &c->rchain, &c->fbc, &c->fbh, &c->fbo, &c->fbl,
                      &c->fbs, &c->fbt, &c->fbk, &c->fbu, &c->fbch, &c->fbco, &c->fbcs, &c->fbimg, &c->fbstop, &c->fbwin, &c->fbopen, &c->fbvm, &c->fbvh,
                      &c->fbreg, &c->fbJ, &c->fbvis, &c->fbph,
                      &c->ck})
        b->release();
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_df) (void)hipEventDestroy(c->ev_df);
    if (c->ev_inf) (void)hipEventDestroy(c->ev_inf);
    if (c->fbkeep_h) (void)hipHostFree(c->fbkeep_h);
    if (c->pin) (void)hipHostFree(c->pin);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

static std::mutex g_default_mu;
static dmx_config g_default_cfg;
static bool g_default_set = false, g_default_made = false;

int dmx_set_default_config(const dmx_config* cfg) {
    if (!cfg) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(g_default_mu);
    if (g_default_made) return DMX_ERR_ARG;
    g_default_cfg = *cfg;
    g_default_set = true;
    return DMX_OK;
}

dmx_ctx* dmx_default_ctx(void) {
    static std::once_flag once;
    static dmx_ctx* ctx = nullptr;
    std::call_once(once, [] {
        std::lock_guard<std::mutex> g(g_default_mu);
        g_default_made = true;
        if (dmx_create(&ctx, g_default_set ? &g_default_cfg : nullptr) != DMX_OK) ctx = nullptr;
    });
    return ctx;
}

size_t dmx_deflate_bound(size_t n) { return n + 10 * ((n + 16383) / 16384) + 16; }

int dmx_deflate_device(dmx_ctx* c, const void* d_in, size_t n, int level, uint32_t flags,
                       void* d_out, size_t cap, size_t* out_len, void* stream) {
    if (!c || (!d_in && n) || !d_out || !out_len) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return deflate_device_locked(c, (const uint8_t*)d_in, n, level, flags, (uint8_t*)d_out, cap,
                                 out_len, st);
}

int dmx_deflate_device_async(dmx_ctx* c, const void* d_in, size_t n, int level, uint32_t flags,
                             void* d_out, size_t cap, uint64_t* d_out_len, void* stream) {
    if (!c || (!d_in && n) || !d_out || !d_out_len) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return deflate_device_locked(c, (const uint8_t*)d_in, n, level, flags, (uint8_t*)d_out, cap,
                                 nullptr, st, d_out_len);
}

int dmx_inflate_device(dmx_ctx* c, const void* d_in, size_t n, void* d_out, size_t cap,
                       size_t* out_len, void* stream) {
    if (!c || (!d_in && n) || !d_out || !out_len) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return inflate_device_locked(c, (const uint8_t*)d_in, n, (uint8_t*)d_out, cap, out_len,
                                 nullptr, st);
}

int dmx_inflate_device_async(dmx_ctx* c, const void* d_in, size_t n, void* d_out, size_t cap,
                             uint64_t* d_result, uint32_t flags, void* stream) {
    if (!c || (!d_in && n) || !d_out || !d_result || (flags & ~DMX_INFLATE_PIECE)) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return inflate_device_async_locked(c, (const uint8_t*)d_in, n, (uint8_t*)d_out, cap, d_result, st,
                                       (flags & DMX_INFLATE_PIECE) ? DMX_IFLAG_PIECE : 0u);
}

int dmx_inflate_piece_device(dmx_ctx* c, const void* d_in, size_t n, void* d_out, size_t cap,
                             size_t* out_len, void* stream) {
    if (!c || (!d_in && n) || !d_out || !out_len) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return inflate_device_locked(c, (const uint8_t*)d_in, n, (uint8_t*)d_out, cap, out_len, nullptr, st,
                                 DMX_IFLAG_PIECE);
}

int dmx_deflate(dmx_ctx* c, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                size_t* out_len) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || !out_len || (!out && cap)) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->subs.size() > 1 && n >= 2 * c->subs.size() * (size_t)c->seg)
        return deflate_multi(c, in, n, level, out, cap, out_len);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    const size_t bound = dmx_deflate_bound(n);
    if (!c->in.ensure(n + 16) || !c->out.ensure(bound)) return DMX_ERR_NOMEM;
    if (n) HIPCHK(hipMemcpyAsync(c->in.p, in, n, hipMemcpyHostToDevice, c->stream));
    size_t total = 0;
    int rc = deflate_device_locked(c, c->in.as<uint8_t>(), n, level, 0, c->out.as<uint8_t>(),
                                   c->out.cap, &total, c->stream);
    *out_len = total;
    if (rc != DMX_OK) return rc;
    if (total > cap) return DMX_ERR_CAPACITY;
    if (total) HIPCHK(hipMemcpyAsync(out, c->out.p, total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DMX_OK;
}

static int inflate_host(dmx_ctx* c, const uint8_t* in, size_t n, uint8_t** dev, size_t* total) {
    if (!c->in.ensure(n + 16)) return DMX_ERR_NOMEM;
    if (n) HIPCHK(hipMemcpyAsync(c->in.p, in, n, hipMemcpyHostToDevice, c->stream));
    return inflate_device_locked(c, c->in.as<uint8_t>(), n, nullptr, 0, total, dev, c->stream);
}

int dmx_inflate(dmx_ctx* c, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                size_t* written, size_t* total) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || (!out && cap) || !written) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    uint8_t* dev = nullptr;
    size_t tot = 0;
    *written = 0;
    if (total) *total = 0;
    if (c->subs.size() > 1 && n >= 4 * c->subs.size() * (size_t)c->seg) {
        const int mr = inflate_multi(c, in, n, out, cap, nullptr, written, &tot);
        if (mr != 1) {
            if (total) *total = tot;
            return mr;
        }
    }
    int rc = inflate_host(c, in, n, &dev, &tot);
    if (rc != DMX_OK) return rc;
    const size_t w = tot < cap ? tot : cap;
    if (w) HIPCHK(hipMemcpyAsync(out, dev, w, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *written = w;
    if (total) *total = tot;
    return DMX_OK;
}

int dmx_inflate_alloc(dmx_ctx* c, const uint8_t* in, size_t n, uint8_t** out, size_t* len) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || !out || !len) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    *out = nullptr;
    *len = 0;
    uint8_t* dev = nullptr;
    size_t tot = 0;
    if (c->subs.size() > 1 && n >= 4 * c->subs.size() * (size_t)c->seg) {
        const int mr = inflate_multi(c, in, n, nullptr, 0, out, nullptr, &tot);
        if (mr != 1) {
            if (mr == DMX_OK) *len = tot;
            return mr;
        }
    }
    int rc = inflate_host(c, in, n, &dev, &tot);
    if (rc != DMX_OK) return rc;
    uint8_t* h = static_cast<uint8_t*>(std::malloc(tot ? tot : 1));
    if (!h) return DMX_ERR_NOMEM;
    if (tot && hipMemcpyAsync(h, dev, tot, hipMemcpyDeviceToHost, c->stream) != hipSuccess) {
        std::free(h);
        return DMX_ERR_DEVICE;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(h);
        return DMX_ERR_DEVICE;
    }
    *out = h;
    *len = tot;
    return DMX_OK;
}

// ---- segment index for multi-GPU inflate ------------------------------------
int dmx_segment_starts_device(dmx_ctx* c, const void* d_in, size_t n, uint64_t* starts, size_t cap,
                              size_t* count, void* stream) {
    if (!c || (!d_in && n) || !count || (!starts && cap)) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    *count = 0;
    if (n == 0) return DMX_OK;
    if (!c->scal.ensure(sizeof(Scal))) return DMX_ERR_NOMEM;
    Scal* ds = c->scal.as<Scal>();
    const uint8_t* in = static_cast<const uint8_t*>(d_in);
    const uint64_t misalign = (uintptr_t)in & 3;
    const uint32_t* words = reinterpret_cast<const uint32_t*>(in - misalign);
    const uint64_t ntiles = marker_tiles(n, misalign);
    if (!c->tiles.ensure(ntiles * 4) || !c->tileoffs.ensure(scan_words(ntiles) * 8)) return DMX_ERR_NOMEM;
    HIPCHK(launch_marker_count(words, misalign, n, c->tiles.as<uint32_t>(), ntiles, st));
    HIPCHK(launch_scan_u32(c->tiles.as<uint32_t>(), c->tileoffs.as<uint64_t>(), ntiles, &ds->nmarkers, st));
    uint64_t nm = 0;
    HIPCHK(hipMemcpyAsync(&nm, &ds->nmarkers, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (!c->cands.ensure((nm + 1) * 8)) return DMX_ERR_NOMEM;
    HIPCHK(launch_marker_write(words, misalign, n, c->tileoffs.as<uint64_t>(), ntiles, c->cands.as<uint64_t>(),
                               ~0ull, st));
    // cands[0] is the stream start; markers follow
    const size_t k = std::min<size_t>(cap, nm);
    if (k) HIPCHK(hipMemcpyAsync(starts, c->cands.as<uint64_t>() + 1, k * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *count = nm;
    return DMX_OK;
}

int dmx_segment_check_device(dmx_ctx* c, const void* d_in, size_t n, const uint64_t* starts, size_t k,
                             uint64_t* ends, void* stream) {
    if (!c || (!d_in && n) || (k && (!starts || !ends))) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (k == 0) return DMX_OK;
    if (!c->cands.ensure(2 * k * 8)) return DMX_ERR_NOMEM;
    uint64_t* d_starts = c->cands.as<uint64_t>();
    uint64_t* d_ends = d_starts + k;
    HIPCHK(hipMemcpyAsync(d_starts, starts, k * 8, hipMemcpyHostToDevice, st));
    const uint8_t* in = static_cast<const uint8_t*>(d_in);
    InflateArgs A{};
    A.misalign = (uintptr_t)in & 3;
    A.in_words = reinterpret_cast<const uint32_t*>(in - A.misalign);
    A.n = n;
    A.flags = c->flags | DMX_IFLAG_PIECE;
    HIPCHK(launch_segment_check(A, d_starts, k, d_ends, st));
    HIPCHK(hipMemcpyAsync(ends, d_ends, k * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return DMX_OK;
}

// ---- checksums and zlib / gzip containers ------------------------------
int dmx_adler32_device(dmx_ctx* c, const void* d, size_t n, uint32_t init, uint32_t* out, void* stream) {
    if (!c || (!d && n) || !out) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    return checksum_locked(c, false, (const uint8_t*)d, n, init, out, stream ? (hipStream_t)stream : c->stream);
}

int dmx_crc32_device(dmx_ctx* c, const void* d, size_t n, uint32_t init, uint32_t* out, void* stream) {
    if (!c || (!d && n) || !out) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    return checksum_locked(c, true, (const uint8_t*)d, n, init, out, stream ? (hipStream_t)stream : c->stream);
}

static int checksum_host(dmx_ctx* c, bool crc, const uint8_t* in, size_t n, uint32_t init, uint32_t* out) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || !out) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    if (!c->in.ensure(n + 16)) return DMX_ERR_NOMEM;
    if (n) HIPCHK(hipMemcpyAsync(c->in.p, in, n, hipMemcpyHostToDevice, c->stream));
    return checksum_locked(c, crc, c->in.as<uint8_t>(), n, init, out, c->stream);
}

int dmx_adler32(dmx_ctx* c, const uint8_t* in, size_t n, uint32_t init, uint32_t* out) {
    return checksum_host(c, false, in, n, init, out);
}

int dmx_crc32(dmx_ctx* c, const uint8_t* in, size_t n, uint32_t init, uint32_t* out) {
    return checksum_host(c, true, in, n, init, out);
}

size_t dmx_framed_bound(size_t n) { return dmx_deflate_bound(n) + 18; }

static int deflate_framed_entry(dmx_ctx* c, bool gz, const uint8_t* in, size_t n, int level, uint8_t* out,
                                size_t cap, size_t* out_len) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || !out_len || !out) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    return deflate_framed(c, gz, in, n, level, out, cap, out_len);
}

int dmx_deflate_zlib(dmx_ctx* c, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                     size_t* out_len) {
    return deflate_framed_entry(c, false, in, n, level, out, cap, out_len);
}

int dmx_deflate_gzip(dmx_ctx* c, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                     size_t* out_len) {
    return deflate_framed_entry(c, true, in, n, level, out, cap, out_len);
}

// Parses the container header, inflates the raw stream on the GPU and (DMX_VERIFY) checks the
// trailer against the GPU checksum of the decoded bytes.  The trailer is taken from the last
// 4 (zlib) / 8 (gzip) bytes of the input.
static int inflate_framed(dmx_ctx* c, bool gz, const uint8_t* in, size_t n, uint32_t flags, uint8_t** out,
                          size_t* len) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if ((!in && n) || !out || !len) return DMX_ERR_ARG;
    *out = nullptr;
    *len = 0;
    size_t head = 0;
    if (gz) {
        if (n < 18) return DMX_ERR_OVERREAD;
        if (in[0] != 0x1F || in[1] != 0x8B || in[2] != 8) return DMX_ERR_DATA;
        const uint8_t flg = in[3];
        head = 10;
        if (flg & 4) {  // FEXTRA
            if (head + 2 > n) return DMX_ERR_OVERREAD;
            head += 2 + (size_t)(in[head] | (in[head + 1] << 8));
        }
        for (int z = 0; z < 2; z++) {  // FNAME, FCOMMENT: zero-terminated
            if (flg & (8 << z)) {
                while (head < n && in[head]) head++;
                head++;
            }
        }
        if (flg & 2) head += 2;  // FHCRC
        if (head + 8 > n) return DMX_ERR_OVERREAD;
    } else {
        if (n < 6) return DMX_ERR_OVERREAD;
        const uint32_t cmf = in[0], flg = in[1];
        if ((cmf & 15) != 8 || (cmf >> 4) > 7 || (cmf * 256 + flg) % 31 != 0) return DMX_ERR_DATA;
        if (flg & 0x20) return DMX_ERR_DATA;  // preset dictionary: not supported
        head = 2;
    }
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    uint8_t* dev = nullptr;
    size_t tot = 0;
    int rc = inflate_host(c, in + head, n - head, &dev, &tot);
    if (rc != DMX_OK) return rc;
    if (flags & DMX_VERIFY) {
        uint32_t ck = 0;
        rc = checksum_locked(c, gz, dev, tot, gz ? 0u : 1u, &ck, c->stream);
        if (rc != DMX_OK) return rc;
        const uint8_t* t = in + n - (gz ? 8 : 4);
        uint32_t want = 0;
        if (gz) {
            want = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
            const uint32_t isize = (uint32_t)t[4] | ((uint32_t)t[5] << 8) | ((uint32_t)t[6] << 16) |
                                   ((uint32_t)t[7] << 24);
            if (isize != (uint32_t)tot) return DMX_ERR_CHECKSUM;
        } else {
            want = ((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | (uint32_t)t[3];
        }
        if (ck != want) return DMX_ERR_CHECKSUM;
    }
    uint8_t* h = static_cast<uint8_t*>(std::malloc(tot ? tot : 1));
    if (!h) return DMX_ERR_NOMEM;
    if (tot && hipMemcpyAsync(h, dev, tot, hipMemcpyDeviceToHost, c->stream) != hipSuccess) {
        std::free(h);
        return DMX_ERR_DEVICE;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
        std::free(h);
        return DMX_ERR_DEVICE;
    }
    *out = h;
    *len = tot;
    return DMX_OK;
}

int dmx_inflate_zlib(dmx_ctx* c, const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* len) {
    return inflate_framed(c, false, in, n, flags, out, len);
}

int dmx_inflate_gzip(dmx_ctx* c, const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* len) {
    return inflate_framed(c, true, in, n, flags, out, len);
}

// ---- file-path overloads with streaming I/O ----------------------------
namespace {

struct Pinned {
    void* p = nullptr;
    explicit Pinned(size_t n) {
        if (hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault) != hipSuccess) p = nullptr;
    }
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

struct File {
    FILE* f = nullptr;
    File(const char* path, const char* mode) : f(std::fopen(path, mode)) {}
    ~File() {
        if (f) std::fclose(f);
    }
};

// A reader thread fills two pinned buffers in turn from a file (chunk k into buffer k % 2);
// the consumer takes chunk k, and releases its buffer once the H2D copy from it has finished.
struct ChunkReader {
    FILE* f;
    size_t chunk, total, nchunks;
    uint8_t* buf[2];
    size_t len[2] = {0, 0};
    bool ready[2] = {false, false};
    bool failed = false, stop = false;
    std::mutex m;
    std::condition_variable cv;
    std::thread th;
    ChunkReader(FILE* f_, size_t total_, size_t chunk_, uint8_t* b0, uint8_t* b1)
        : f(f_), chunk(chunk_), total(total_), nchunks((total_ + chunk_ - 1) / chunk_), buf{b0, b1} {
        th = std::thread([this] { run(); });
    }
    ~ChunkReader() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void run() {
        for (size_t k = 0; k < nchunks; k++) {
            const int b = (int)(k & 1);
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return !ready[b] || stop; });
                if (stop) return;
            }
            const size_t want = std::min(chunk, total - k * chunk);
            const size_t got = std::fread(buf[b], 1, want, f);
            std::lock_guard<std::mutex> g(m);
            len[b] = want;
            ready[b] = true;
            if (got != want) failed = true;
            cv.notify_all();
        }
    }
    // waits for chunk k; returns its buffer and length (nullptr on a read error)
    uint8_t* take(size_t k, size_t* n) {
        const int b = (int)(k & 1);
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return ready[b] || failed; });
        if (failed) return nullptr;
        *n = len[b];
        return buf[b];
    }
    void release(size_t k) {
        std::lock_guard<std::mutex> g(m);
        ready[k & 1] = false;
        cv.notify_all();
    }
};

// A writer thread takes the compressed chunks in order: chunk k's D2H into pinned buffer
// k % 2 was recorded on an event by the producer; the writer waits for the event and writes
// the bytes, then frees the buffer for chunk k + 2.  The producer meanwhile compresses the
// next chunk, so the D2H and the file write of chunk k overlap the compression of k + 1.
struct ChunkWriter {
    FILE* f;
    uint8_t* buf[2];
    hipEvent_t ev[2];
    size_t len[2] = {0, 0};
    bool full[2] = {false, false};
    bool failed = false, stop = false;
    size_t next = 0, queued = 0;  // next chunk to write, chunks handed over
    std::mutex m;
    std::condition_variable cv;
    std::thread th;
    ChunkWriter(FILE* f_, uint8_t* b0, uint8_t* b1, hipEvent_t e0, hipEvent_t e1)
        : f(f_), buf{b0, b1}, ev{e0, e1} {
        th = std::thread([this] { run(); });
    }
    ~ChunkWriter() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void run() {
        for (;;) {
            size_t k, n;
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return full[next & 1] || stop; });
                if (!full[next & 1]) return;  // stop with nothing queued
                k = next;
                n = len[k & 1];
            }
            bool ok = hipEventSynchronize(ev[k & 1]) == hipSuccess;
            ok = ok && (n == 0 || std::fwrite(buf[k & 1], 1, n, f) == n);
            std::lock_guard<std::mutex> g(m);
            if (!ok) failed = true;
            full[k & 1] = false;
            next++;
            cv.notify_all();
        }
    }
    // waits until buffer k % 2 is free (chunk k - 2 written); false after a write error
    bool acquire(size_t k) {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return !full[k & 1] || failed; });
        return !failed;
    }
    void hand_over(size_t k, size_t n) {
        std::lock_guard<std::mutex> g(m);
        len[k & 1] = n;
        full[k & 1] = true;
        queued = k + 1;
        cv.notify_all();
    }
    bool drain() {  // all handed-over chunks written
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return next == queued || failed; });
        return !failed;
    }
};

int64_t file_size(FILE* f) {
    if (std::fseek(f, 0, SEEK_END) != 0) return -1;
    const long long n = ftello(f);
    if (std::fseek(f, 0, SEEK_SET) != 0) return -1;
    return n;
}

constexpr size_t kFileChunk = 64ull << 20;  // bytes per streamed chunk (a multiple of 32 KiB)

}  // namespace

int dmx_deflate_file(dmx_ctx* c, const char* in_path, const char* out_path, int level, size_t* in_bytes,
                     size_t* out_bytes) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if (!in_path || !out_path) return DMX_ERR_ARG;
    File fi(in_path, "rb");
    if (!fi.f) return DMX_ERR_ARG;
    const int64_t N = file_size(fi.f);
    if (N < 0) return DMX_ERR_ARG;
    File fo(out_path, "wb");
    if (!fo.f) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    const size_t K = kFileChunk;
    const size_t bound = dmx_deflate_bound(K);
    Pinned hin0(K), hin1(K), hout0(bound), hout1(bound);
    DevBuf din[2], dout[2];
    auto release_all = [&] {
        for (auto& d : din) d.release();
        for (auto& d : dout) d.release();
    };
    if (!hin0.p || !hin1.p || !hout0.p || !hout1.p || !din[0].ensure(K) || !din[1].ensure(K) ||
        !dout[0].ensure(bound) || !dout[1].ensure(bound)) {
        release_all();
        return DMX_ERR_NOMEM;
    }
    hipStream_t cs = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr}, evo[2] = {nullptr, nullptr};
    int rc = DMX_OK;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) rc = DMX_ERR_DEVICE;
    for (auto* e : {&ev[0], &ev[1], &evo[0], &evo[1]})
        if (rc == DMX_OK && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) rc = DMX_ERR_DEVICE;
    size_t written = 0;
    if (rc == DMX_OK && N == 0) {  // empty file: one empty final block, as dmx_deflate
        size_t len = 0;
        rc = deflate_device_locked(c, nullptr, 0, level, 0, dout[0].as<uint8_t>(), bound, &len, c->stream);
        if (rc == DMX_OK && hipMemcpy(hout0.p, dout[0].p, len, hipMemcpyDeviceToHost) != hipSuccess) rc = DMX_ERR_DEVICE;
        if (rc == DMX_OK && std::fwrite(hout0.p, 1, len, fo.f) != len) rc = DMX_ERR_ARG;
        written = len;
    } else if (rc == DMX_OK) {
        ChunkReader rd(fi.f, (size_t)N, K, hin0.u8(), hin1.u8());
        ChunkWriter wr(fo.f, hout0.u8(), hout1.u8(), evo[0], evo[1]);
        const size_t nch = rd.nchunks;
        // copy chunk k + 1 in on the copy stream while chunk k compresses on the context stream
        auto h2d = [&](size_t k) -> int {
            size_t n = 0;
            uint8_t* h = rd.take(k, &n);
            if (!h) return DMX_ERR_ARG;
            if (hipMemcpyAsync(din[k & 1].p, h, n, hipMemcpyHostToDevice, cs) != hipSuccess) return DMX_ERR_DEVICE;
            if (hipEventRecord(ev[k & 1], cs) != hipSuccess) return DMX_ERR_DEVICE;
            return DMX_OK;
        };
        rc = h2d(0);
        for (size_t k = 0; k < nch && rc == DMX_OK; k++) {
            if (k + 1 < nch && (rc = h2d(k + 1)) != DMX_OK) break;
            if (hipStreamWaitEvent(c->stream, ev[k & 1], 0) != hipSuccess) { rc = DMX_ERR_DEVICE; break; }
            const size_t n = std::min(K, (size_t)N - k * K);
            size_t len = 0;
            // output buffers k % 2 are free once chunk k - 2 is written (its D2H is done then)
            if (!wr.acquire(k)) { rc = DMX_ERR_ARG; break; }
            rc = deflate_device_locked(c, din[k & 1].as<uint8_t>(), n, level, k + 1 < nch ? DMX_DEFLATE_NOT_FINAL : 0,
                                       dout[k & 1].as<uint8_t>(), bound, &len, c->stream);
            if (rc != DMX_OK) break;
            rd.release(k);  // the H2D of chunk k is complete (the deflate waited for it)
            // D2H on the copy stream (after the deflate, which synchronized), written by the
            // writer thread while chunk k + 1 compresses
            if ((len && hipMemcpyAsync(k & 1 ? hout1.p : hout0.p, dout[k & 1].p, len, hipMemcpyDeviceToHost, cs) != hipSuccess) ||
                hipEventRecord(evo[k & 1], cs) != hipSuccess) { rc = DMX_ERR_DEVICE; break; }
            wr.hand_over(k, len);
            written += len;
        }
        if (!wr.drain() && rc == DMX_OK) rc = DMX_ERR_ARG;
        (void)hipStreamSynchronize(cs);
    }
    for (auto* e : {ev[0], ev[1], evo[0], evo[1]})
        if (e) (void)hipEventDestroy(e);
    if (cs) (void)hipStreamDestroy(cs);
    release_all();
    if (in_bytes) *in_bytes = (size_t)N;
    if (out_bytes) *out_bytes = written;
    return rc;
}

int dmx_inflate_file(dmx_ctx* c, const char* in_path, const char* out_path, size_t* out_bytes) {
    if (!c) c = dmx_default_ctx();
    if (!c) return DMX_ERR_DEVICE;
    if (!in_path || !out_path) return DMX_ERR_ARG;
    if (out_bytes) *out_bytes = 0;
    File fi(in_path, "rb");
    if (!fi.f) return DMX_ERR_ARG;
    const int64_t C = file_size(fi.f);
    if (C < 0) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    DeviceGuard dg(c->device);
    if (!dg.ok) return DMX_ERR_DEVICE;
    const size_t K = kFileChunk;
    if (!c->in.ensure((size_t)C + 16)) return DMX_ERR_NOMEM;
    Pinned hb0(K), hb1(K);
    if (!hb0.p || !hb1.p) return DMX_ERR_NOMEM;
    int rc = DMX_OK;
    {   // stream the compressed file in: disk reads overlap the H2D copies of earlier chunks
        ChunkReader rd(fi.f, (size_t)C, K, hb0.u8(), hb1.u8());
        for (size_t k = 0; k < rd.nchunks && rc == DMX_OK; k++) {
            size_t n = 0;
            uint8_t* h = rd.take(k, &n);
            if (!h) { rc = DMX_ERR_ARG; break; }
            if (hipMemcpyAsync(c->in.as<uint8_t>() + k * K, h, n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
                hipStreamSynchronize(c->stream) != hipSuccess) { rc = DMX_ERR_DEVICE; break; }
            rd.release(k);
        }
    }
    if (rc != DMX_OK) return rc;
    uint8_t* dev = nullptr;
    size_t tot = 0;
    rc = inflate_device_locked(c, c->in.as<uint8_t>(), (size_t)C, nullptr, 0, &tot, &dev, c->stream);
    if (rc != DMX_OK) return rc;
    File fo(out_path, "wb");
    if (!fo.f) return DMX_ERR_ARG;
    // stream the output back: the D2H of chunk k + 1 overlaps the file write of chunk k
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (auto& e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = DMX_ERR_DEVICE;
    uint8_t* hb[2] = {hb0.u8(), hb1.u8()};
    const size_t nch = (tot + K - 1) / K;
    auto d2h = [&](size_t k) -> bool {
        const size_t n = std::min(K, tot - k * K);
        return hipMemcpyAsync(hb[k & 1], dev + k * K, n, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
               hipEventRecord(ev[k & 1], c->stream) == hipSuccess;
    };
    if (rc == DMX_OK && nch && !d2h(0)) rc = DMX_ERR_DEVICE;
    for (size_t k = 0; k < nch && rc == DMX_OK; k++) {
        if (hipEventSynchronize(ev[k & 1]) != hipSuccess) { rc = DMX_ERR_DEVICE; break; }
        if (k + 1 < nch && !d2h(k + 1)) { rc = DMX_ERR_DEVICE; break; }
        const size_t n = std::min(K, tot - k * K);
        if (std::fwrite(hb[k & 1], 1, n, fo.f) != n) rc = DMX_ERR_ARG;
    }
    (void)hipStreamSynchronize(c->stream);
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    if (out_bytes && rc == DMX_OK) *out_bytes = tot;
    return rc;
}

void dmx_free(void* p) { std::free(p); }

const char* dmx_strerror(int code) {
    switch (code) {
        case DMX_OK: return "ok";
        case DMX_ERR_ARG: return "invalid argument";
        case DMX_ERR_NOMEM: return "out of memory";
        case DMX_ERR_DEVICE: return "HIP device error (no usable gfx950 device?)";
        case DMX_ERR_DATA: return "invalid deflate stream";
        case DMX_ERR_OVERREAD: return "Reading bits beyond the alloted buffer size!";
        case DMX_ERR_CAPACITY: return "output buffer too small";
        case DMX_ERR_INTERNAL: return "internal error";
        case DMX_ERR_CHECKSUM: return "container checksum or length mismatch";
        default: return "unknown error";
    }
}

int dmx_set_timing(dmx_ctx* c, int enable) {
    if (!c) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->timing = enable != 0;
    return DMX_OK;
}

int dmx_last_stats(dmx_ctx* c, dmx_stats* st) {
    if (!c || !st) return DMX_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    *st = c->stats;
    return DMX_OK;
}

}  // extern "C"
