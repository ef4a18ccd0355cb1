/* dmx.h -- C-ABI of the MI355X-native DEFLATE/INFLATE engine (libdmx.so).
 *
 * This is the drop-in boundary for HyperBitGore/deflate.hpp's hot path.  The reference has no
 * C ABI of its own (header-only static methods); each entry point below states the reference
 * interface it replaces (file:line under the reference's include/).  include/deflate.hpp and
 * include/inflate.hpp re-expose the reference's class API on top of these functions, and
 * INTEGRATION.md shows the ctypes / C++ bindings a caller adds.
 *
 * Plain pointers and sizes only; no torch or HIP types in any signature (streams are passed as
 * an opaque void* that is a hipStream_t).  All functions are thread-safe per context; the
 * default context (dmx_default_ctx) is created lazily under a once-flag.
 */
#ifndef DMX_H
#define DMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define DMX_OK 0
#define DMX_ERR_ARG (-1)      /* bad argument (null pointer, unsupported option)              */
#define DMX_ERR_NOMEM (-2)    /* host or device allocation failed                               */
#define DMX_ERR_DEVICE (-3)   /* HIP runtime error or no usable gfx950 device                   */
#define DMX_ERR_DATA (-4)     /* stream cannot be decoded (no Huffman code matches, bad table) */
#define DMX_ERR_OVERREAD (-5) /* stream ends before its final block: the reference throws
                                 "Reading bits beyond the alloted buffer size!"
                                 (inflate.hpp:81-82, 97-99, 106-108)                          */
#define DMX_ERR_CAPACITY (-6) /* caller's output buffer too small (device API only)           */
#define DMX_ERR_INTERNAL (-7)
#define DMX_ERR_CHECKSUM (-8) /* zlib Adler-32 / gzip CRC-32 or ISIZE mismatch (DMX_VERIFY)      */

/* ---- context --------------------------------------------------------------------------- */
typedef struct dmx_ctx dmx_ctx;

typedef struct dmx_config {
    int device;             /* HIP device ordinal, -1 = the calling thread's current device  */
    uint32_t segment_bytes; /* independent deflate segment: 16384, 32768 (default) or 65536.
                               32768 mirrors the reference's per-chunk LZ77 reset
                               (deflate.hpp:689-697).  65536 (SURVEY 8(d) config C4's
                               64 KiB blocks): one DEFLATE block per 64 KiB of input, its
                               two 32 KiB halves matched independently under one Huffman
                               code; inflate then places 64 KiB per segment.  Inflate takes
                               any stream with any setting; the lane decoder's slot follows
                               this size.                                                      */
    uint32_t flags;         /* DMX_CFG_*                                                        */
    uint32_t n_gpus;        /* 0 or 1: one device.  N > 1: the host-buffer API (dmx_deflate,
                               dmx_inflate, dmx_inflate_alloc, hence deflate::compress and
                               inflate::decompress) splits each large call over N devices,
                               `device`, device + 1, ... (mod the visible count: fewer GPUs than N
                               run several shards each; more than 8 per visible GPU is
                               DMX_ERR_ARG).  Deflate: contiguous segment-aligned
                               shards, NOT_FINAL except the last -- segments are independent
                               (deflate.hpp:689-697), so the bytes equal the one-device stream.
                               Inflate: cuts at segment starts proven by a piece-mode decode
                               (dmx_segment_check_device), one piece per device, the outputs
                               concatenated; a stream that does not split decodes on one.
                               The split assumes the stream's first BFINAL block lies in its
                               last piece (every stream libdmx, zlib or the reference writes);
                               bytes after an early BFINAL that still decode as marker-delimited
                               segments would be inflated too, where one device stops.          */
    /* developer controls for A/B runs; dmx_config_default sets both to 0 = the product plan */
    uint32_t dev_inflate_pass; /* k + 1 forces inflate pass k of the segmented plan
                                  (0 wave, 1 workgroup, 2 look-back, 4 lanes, 5 block-parallel,
                                  7 the serial decoder alone) */
    uint32_t dev_heavy_bytes;  /* lane decoder: candidates spanning more compressed bytes go to
                                  the workgroup decoder; 0 = the built-in 2048 and CU rule      */
} dmx_config;

/* Inflate code-length RLE per RFC 1951 (repeat may span HLIT/HDIST, code 16 repeats the
 * previous length) instead of the reference's behaviour (SURVEY A-11/A-12, inflate.hpp:166-224).
 * Default off: output is bit-exact to the reference. */
#define DMX_CFG_RFC_STRICT 1u
/* Developer A/B: the block-parallel path decodes every unit with one wavefront. */
#define DMX_CFG_FB_SERIAL 2u

void dmx_config_default(dmx_config* cfg);
int dmx_create(dmx_ctx** ctx, const dmx_config* cfg);
void dmx_destroy(dmx_ctx* ctx);
/* process-wide context (never destroyed), created on first use with the config set by
 * dmx_set_default_config, else the default config on the current device.  This is the context
 * include/deflate.hpp and include/inflate.hpp use: a caller of the reference's class API turns
 * on the whole node with one call, e.g. cfg.n_gpus = 8, before its first compress. */
dmx_ctx* dmx_default_ctx(void);
/* DMX_ERR_ARG once the default context exists (the config is read at its creation). */
int dmx_set_default_config(const dmx_config* cfg);

/* ---- host-buffer API (what include/deflate.hpp / inflate.hpp call) ---------------------- */

/* Upper bound of dmx_deflate's output for n input bytes, any segment size / level. */
size_t dmx_deflate_bound(size_t n);

/* Replaces deflate::compress(char*, size_t, int)             deflate.hpp:779-796
 *          deflate::compress(std::vector<uint8_t>&, int)      deflate.hpp:798-815
 * Raw DEFLATE (RFC 1951, no zlib/gzip wrapper).  level 0 = stored, 1 = Huffman only,
 * 2 = fast (greedy hash), 3 = slow (lazy, deeper search); any other value behaves like 1,
 * as the reference's switch without default does (deflate.hpp:699-717).  Output is a valid
 * stream the reference inflate::decompress round-trips exactly (the reference's own levels
 * 2/3 are not; SURVEY A-1..A-3).  *out_len receives the stream length. */
int dmx_deflate(dmx_ctx* ctx, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                size_t* out_len);

/* Replaces inflate::decompress(void*, size_t, void*, size_t)   inflate.hpp:338-350
 * Decodes the whole stream, copies min(total, cap) bytes to out.  *written = bytes copied
 * (the reference's return value), *total = full decoded size (may be NULL). */
int dmx_inflate(dmx_ctx* ctx, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                size_t* written, size_t* total);

/* Replaces inflate::decompress(void*, size_t)                  inflate.hpp:363-374
 *          inflate::decompress(std::vector<uint8_t>)           inflate.hpp:376-387
 * *out is allocated by the library; release it with dmx_free. */
int dmx_inflate_alloc(dmx_ctx* ctx, const uint8_t* in, size_t n, uint8_t** out, size_t* len);

void dmx_free(void* p);

/* Replaces deflate::compress(std::string, std::string, int)      deflate.hpp:755-777
 *          inflate::decompress(std::string, std::string)          inflate.hpp:390-408
 * Streaming file I/O in 64 MiB chunks.  Deflate: a reader thread fills two pinned buffers,
 * the H2D of chunk k + 1 and the D2H + file write of chunk k - 1 (a writer thread) overlap the
 * compression of chunk k; each chunk is a NOT_FINAL shard, the last one final, so the file is
 * one stream; device memory is bounded (2 x 64 MiB in, 2 x bound out).  Inflate: the
 * compressed file streams into HBM (disk reads overlapping the H2D copies), decodes as one
 * stream, and the D2H of each output chunk overlaps the file write of the previous one; it
 * holds the whole compressed file and the whole output in HBM (plus the decoder's scratch),
 * so files beyond the device's memory are not supported.  Unlike the reference (correct only
 * for files <= 32 KiB, SURVEY A-8) any size that fits works.  Sizes are reported through the
 * optional out-parameters. */
int dmx_deflate_file(dmx_ctx* ctx, const char* in_path, const char* out_path, int level,
                     size_t* in_bytes, size_t* out_bytes);
int dmx_inflate_file(dmx_ctx* ctx, const char* in_path, const char* out_path, size_t* out_bytes);
const char* dmx_strerror(int code);

/* ---- device-resident API (HBM in, HBM out; used by bench.py and multi-GPU sharding) ------ */

/* Do not set BFINAL on the last block: the output is one shard of a larger stream and ends
 * byte-aligned on an empty stored block, so shards concatenate with plain byte copies. */
#define DMX_DEFLATE_NOT_FINAL 1u

/* d_in/d_out are device pointers on the context's device; stream is a hipStream_t or NULL for
 * the context's own stream.  Returns DMX_ERR_CAPACITY if cap < the produced size. */
int dmx_deflate_device(dmx_ctx* ctx, const void* d_in, size_t n, int level, uint32_t flags,
                       void* d_out, size_t cap, size_t* out_len, void* stream);

/* The same without a host synchronisation: every step is enqueued on `stream` and the stream
 * length lands in *d_out_len (8 bytes of DEVICE memory) when the work completes; the call
 * returns once it is enqueued (graph-capturable, and a multi-GPU caller can keep every device
 * busy from one thread).  A length above cap means the output did not fit: only the segments
 * that fit were written.  Calls on one context are ordered even across streams (the context's
 * scratch is reused). */
int dmx_deflate_device_async(dmx_ctx* ctx, const void* d_in, size_t n, int level, uint32_t flags,
                             void* d_out, size_t cap, uint64_t* d_out_len, void* stream);

/* Device-resident inflate.  Returns DMX_ERR_CAPACITY (and the needed size in *out_len) when
 * the decoded stream does not fit in cap. */
int dmx_inflate_device(dmx_ctx* ctx, const void* d_in, size_t n, void* d_out, size_t cap,
                       size_t* out_len, void* stream);

/* Device-resident inflate without any host synchronisation, for streams in libdmx's segment
 * layout (its own deflate output, or any stream of independent marker-delimited segments of at
 * most segment_bytes each): every step is enqueued on `stream` and the call returns at once
 * (graph-capturable; a multi-GPU caller keeps every device busy from one thread).  When the
 * work completes, d_result (16 bytes of DEVICE memory) holds {decoded bytes, status}: status 0
 * = decoded into d_out; status 1 = this fast path does not take the stream (another layout, a
 * segment it declines, more segments than cap / segment_bytes + 64, output beyond cap) and
 * nothing is promised about d_out -- decode it with dmx_inflate_device, which takes any stream.
 * flags: DMX_INFLATE_PIECE for one piece of a larger stream (a back-reference before the piece
 * is an error, as in dmx_inflate_piece_device).  Calls on one context are ordered even across
 * streams.  Replaces nothing in the reference (whose inflate is synchronous, inflate.hpp:
 * 338-408); it is the asynchronous form of the same decode (multi-GPU pieces). */
#define DMX_INFLATE_PIECE 1u
int dmx_inflate_device_async(dmx_ctx* ctx, const void* d_in, size_t n, void* d_out, size_t cap,
                             uint64_t* d_result, uint32_t flags, void* stream);

/* Byte offsets just past every "00 00 FF FF" (empty stored block) in a device-resident stream:
 * the candidate segment starts of libdmx's layout, in order (at most cap written, *count = all).
 * Multi-GPU inflate splits a stream at these (deflate.hpp_amd/shard.py scatter_inflate); a
 * false candidate inside stored data makes the piece before it fail to decode, and the caller
 * then decodes the stream whole. */
int dmx_segment_starts_device(dmx_ctx* ctx, const void* d_in, size_t n, uint64_t* starts, size_t cap,
                              size_t* count, void* stream);

/* One piece of a larger stream cut at a segment start (multi-GPU inflate, shard.py): exactly
 * dmx_inflate_device, except that a back-reference reaching before the piece's first byte is
 * DMX_ERR_DATA.  At a stream's true start the reference copies nothing for such a distance
 * (inflate.hpp:268-270) and dmx_inflate_device does the same; inside a stream whose window
 * carries across the cut (zlib's sync flush) that rule would drop bytes without an error. */
int dmx_inflate_piece_device(dmx_ctx* ctx, const void* d_in, size_t n, void* d_out, size_t cap,
                             size_t* out_len, void* stream);

/* Cut-point check for multi-GPU inflate: for each of k candidate starts (host array, stream
 * byte offsets, e.g. from dmx_segment_starts_device) the one segment beginning there is decoded
 * by the exact decoder in piece mode; ends[i] (host array) = the byte just past its closing
 * empty stored block "00 00 FF FF" (or past its BFINAL block), or UINT64_MAX when it does not
 * decode (a "00 00 FF FF" inside stored data, more than 32 KiB of output, a reference before
 * the start).  A start whose segment ends on a marker is a block boundary the decoder reaches
 * with an empty window; shard.py cuts only there. */
int dmx_segment_check_device(dmx_ctx* ctx, const void* d_in, size_t n, const uint64_t* starts, size_t k,
                             uint64_t* ends, void* stream);

/* ---- checksums and containers (not in the reference) -------------------
 * The reference's decompressZlib (inflate.hpp:326-361) skips the 2-byte header and ignores the
 * Adler-32 (SURVEY A-9); inflate.hpp's decompressZlib keeps exactly that.  These entry points
 * add what a zlib/gzip user needs on top: framing on the deflate side and a verified inflate,
 * with Adler-32 / CRC-32 computed block-parallel on the GPU (checksum.hip). */

/* zlib's adler32(init, buf, n) / crc32(init, buf, n) of a device buffer (init 1 / 0 to start). */
int dmx_adler32_device(dmx_ctx* ctx, const void* d, size_t n, uint32_t init, uint32_t* out, void* stream);
int dmx_crc32_device(dmx_ctx* ctx, const void* d, size_t n, uint32_t init, uint32_t* out, void* stream);
/* the same for a host buffer (copied to the device first) */
int dmx_adler32(dmx_ctx* ctx, const uint8_t* in, size_t n, uint32_t init, uint32_t* out);
int dmx_crc32(dmx_ctx* ctx, const uint8_t* in, size_t n, uint32_t init, uint32_t* out);

/* Upper bound of a zlib- or gzip-framed stream for n input bytes. */
size_t dmx_framed_bound(size_t n);
/* RFC 1950 zlib stream (CMF 0x78, FLEVEL from the level, Adler-32 trailer) / RFC 1952 gzip
 * member (no name, MTIME 0, OS 255, CRC-32 + ISIZE trailer) around dmx_deflate's raw stream. */
int dmx_deflate_zlib(dmx_ctx* ctx, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                     size_t* out_len);
int dmx_deflate_gzip(dmx_ctx* ctx, const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                     size_t* out_len);

/* Check the container trailer against the decoded bytes (DMX_ERR_CHECKSUM on mismatch). */
#define DMX_VERIFY 1u
/* Inflate of a zlib stream (header checked; preset dictionaries are DMX_ERR_DATA) / a
 * single-member gzip stream (FEXTRA, FNAME, FCOMMENT, FHCRC skipped); the trailer is the last
 * 4 / 8 input bytes.  *out is allocated by the library (dmx_free). */
int dmx_inflate_zlib(dmx_ctx* ctx, const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* len);
int dmx_inflate_gzip(dmx_ctx* ctx, const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* len);

/* ---- instrumentation -------------------------------------------------------------------- */
typedef struct dmx_stats {
    double ms_main_kernel;  /* HIP-event time of the dominant kernel of the last call       */
    double ms_device_total; /* HIP-event time of all device work of the last call          */
    uint64_t segments;      /* segments (deflate) / candidate segments (inflate)            */
    uint64_t in_bytes;
    uint64_t out_bytes;
    uint32_t path;          /* inflate: 0 = segment-parallel (speculative offsets),
                               1 = segment-parallel (look-back offsets), 2 = serial path,
                               3 = workgroup-per-segment decoder (32 KiB slots),
                               4 = lane decoder + wave resolve (the default for libdmx
                                   streams: one lane decodes a segment's tokens, one
                                   wavefront rebuilds its bytes; dense segments of streams
                                   with few of them go to the workgroup decoder instead),
                               5 = block-parallel decoder for streams without segment
                                   markers (zlib's, libdeflate's, the reference's own):
                                   header scan, one wavefront per unit of blocks, window
                                   hand-off                                                  */
    uint32_t shards;        /* host-buffer API with n_gpus > 1: the pieces the call was split
                               into (0 or 1: one device)                                       */
} dmx_stats;

/* Enable (1) / disable (0) per-call HIP-event timing on a context (off by default). */
int dmx_set_timing(dmx_ctx* ctx, int enable);
int dmx_last_stats(dmx_ctx* ctx, dmx_stats* st);

/* ---- synthetic corpora, bytes [offset, offset + n) --------------- */
#define DMX_CORPUS_ZEROS 0
#define DMX_CORPUS_REPEAT 1
#define DMX_CORPUS_RANDOM 2
#define DMX_CORPUS_TEXT 3
#define DMX_CORPUS_MIXED 4
#define DMX_CORPUS_BMP 5
int dmx_corpus_generate(int kind, uint64_t offset, size_t n, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* DMX_H */
