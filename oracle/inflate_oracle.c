/* oracle/inflate_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference INFLATE (HyperBitGore/deflate.hpp,
 * /root/reference/include/inflate.hpp + common.hpp), used by tests/ and bench.py's
 * cpu_baseline leg as the *checker* for the HIP path.  It is never linked into libdmx.
 *
 * Parity is pinned two ways (tests/test_oracle.py): against golden vectors produced by the
 * compiled reference itself (oracle/_ref, see oracle/Makefile + tests/golden/make_golden.py),
 * and against zlib 1.2.11 on valid streams.
 *
 * Semantics restated (each with the reference line it follows):
 *  - Bit reader: LSB-first, one bit at a time for Huffman symbols (inflate.hpp:78-102, 232).
 *    A read at byte offset >= n is an error here; the reference reads data[n] (one byte past
 *    the buffer, garbage) before it throws (inflate.hpp:81,97,106) -- documented divergence.
 *  - Huffman lookup: the reference's bit-trie (common.hpp:68-103, 201-220) is a dictionary
 *    keyed by (k, low k bits of the canonical code); the decoder accumulates bits MSB-first
 *    and takes the first k that hits (inflate.hpp:232-242).  Codes are assigned canonically
 *    over entries sorted by (len, value) (common.hpp:104-145); on a key collision (only in
 *    over-subscribed codes) the later insert -- higher value -- wins (common.hpp:95-100).
 *  - Precode lookup additionally requires the stored code to equal the accumulated bits
 *    (inflate.hpp:175), so overflowed codes of an over-subscribed precode never match.
 *  - Code-length RLE: lit/len and dist lengths are decoded by two separate counted loops
 *    (inflate.hpp:216, 220), a repeat may overshoot its count and the overshoot entries keep
 *    their (out-of-alphabet) symbol values (inflate.hpp:180-194); code 16 repeats the last
 *    *literal* length seen in the current loop, initially 0 (inflate.hpp:170, 181, 198).
 *    With ORACLE_RFC these two become RFC 1951 (one sequence, 16 repeats the previous length).
 *  - Length symbols 286+ and distance symbols 30+ have no table entry (common.hpp:432-439):
 *    length 0 / distance 0, no extra bits.  Copy is byte-serial and overlap-safe; a distance
 *    of 0 or larger than the output so far copies nothing (inflate.hpp:268-270).
 *  - Stored block: align, LEN, NLEN (unchecked), LEN bytes (inflate.hpp:293-303).
 *  - BTYPE 3 is a silent no-op block (inflate.hpp:292 has no case 3).
 *  - Output window is the whole output (inflate.hpp:284); trailing bytes after BFINAL ignored.
 *  - Not reproduced (reference behaviour is undefined there): a lit/len symbol that no code
 *    matches within 15 bits (the reference keeps reading up to 255 more bits, inflate.hpp:228
 *    uint8_t cur_bit), a distance symbol not found within 16 bits (uninitialised `dss`,
 *    inflate.hpp:251-261), symbol values >= 300 (out-of-bounds value_lookup_table write,
 *    common.hpp:100).  All return ORACLE_ERR_DATA.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_OK 0
#define ORACLE_ERR_OVERREAD (-1)
#define ORACLE_ERR_DATA (-2)
#define ORACLE_ERR_NOMEM (-3)

#define ORACLE_RFC 1u
/* Test-side stand-in for dmx_inflate_piece_device: the input is one piece of a larger stream,
 * so a distance reaching before its first byte is an error instead of a no-op. */
#define ORACLE_PIECE 2u

typedef struct {
    const uint8_t* d;
    size_t n;
    size_t off;     /* byte offset */
    unsigned bit;   /* bit offset inside d[off] */
} bitrd;

static int rd_bit(bitrd* b, unsigned* v) {
    if (b->off >= b->n) return ORACLE_ERR_OVERREAD;
    *v = (b->d[b->off] >> b->bit) & 1u;
    if (++b->bit == 8) { b->bit = 0; b->off++; }
    return 0;
}

/* readBits(n): LSB-first value (inflate.hpp:78-102) */
static int rd_bits(bitrd* b, unsigned nbits, uint32_t* v) {
    uint32_t r = 0;
    for (unsigned i = 0; i < nbits; i++) {
        unsigned x;
        int e = rd_bit(b, &x);
        if (e) return e;
        r |= (uint32_t)x << i;
    }
    *v = r;
    return 0;
}

/* dictionary form of FlatHuffmanTree: for each length k a table of 2^k slots holding
 * (symbol+1, full canonical code) of the last inserted code with that key. */
typedef struct {
    uint16_t* sym[16];   /* sym[k][key] = symbol + 1, 0 = no leaf */
    uint32_t* code[16];  /* full (possibly overflowed) canonical code */
    int maxk;
} htree;

static void ht_free(htree* t) {
    for (int k = 0; k < 16; k++) { free(t->sym[k]); free(t->code[k]); t->sym[k] = NULL; t->code[k] = NULL; }
}

/* FlatHuffmanTree::construct (common.hpp:104-145) over (len[v], v) entries, v < nsym */
static int ht_build(htree* t, const uint8_t* len, int nsym) {
    memset(t, 0, sizeof(*t));
    int bl_count[16] = {0};
    for (int v = 0; v < nsym; v++) {
        if (len[v] > 15) return ORACLE_ERR_DATA;
        if (len[v]) {
            if (v >= 300) return ORACLE_ERR_DATA; /* reference: out-of-bounds table write */
            bl_count[len[v]]++;
        }
    }
    uint32_t next_code[16] = {0};
    uint32_t code = 0;
    for (int bits = 1; bits <= 15; bits++) {
        code = (code + (uint32_t)(bits > 1 ? bl_count[bits - 1] : 0)) << 1;
        next_code[bits] = code;
    }
    /* sorted by (len, value): iterate len outer, value inner */
    for (int k = 1; k <= 15; k++) {
        if (!bl_count[k]) continue;
        t->sym[k] = (uint16_t*)calloc((size_t)1 << k, sizeof(uint16_t));
        t->code[k] = (uint32_t*)calloc((size_t)1 << k, sizeof(uint32_t));
        if (!t->sym[k] || !t->code[k]) return ORACLE_ERR_NOMEM;
        t->maxk = k;
        for (int v = 0; v < nsym; v++) {
            if (len[v] != k) continue;
            uint32_t c = next_code[k]++;
            uint32_t key = c & ((1u << k) - 1u);
            t->sym[k][key] = (uint16_t)(v + 1);
            t->code[k][key] = c;
        }
    }
    return 0;
}

/* bit-serial decode: first k (1..kmax) whose key hits; for the precode the stored code must
 * equal the accumulated bits (inflate.hpp:175). */
static int ht_decode(const htree* t, bitrd* b, int kmax, int exact_code, int* sym) {
    uint32_t acc = 0;
    for (int k = 1; k <= kmax; k++) {
        unsigned x;
        int e = rd_bit(b, &x);
        if (e) return e;
        acc = (acc << 1) | x;
        if (k <= t->maxk && t->sym[k]) {
            uint16_t s = t->sym[k][acc];
            if (s && (!exact_code || t->code[k][acc] == acc)) { *sym = s - 1; return 0; }
        }
    }
    return ORACLE_ERR_DATA;
}

typedef struct {
    uint8_t* p;
    size_t n, cap;
} obuf;

static int ob_push(obuf* o, uint8_t c) {
    if (o->n == o->cap) {
        size_t nc = o->cap ? o->cap * 2 : 65536;
        uint8_t* q = (uint8_t*)realloc(o->p, nc);
        if (!q) return ORACLE_ERR_NOMEM;
        o->p = q;
        o->cap = nc;
    }
    o->p[o->n++] = c;
    return 0;
}

/* RangeLookup tables (common.hpp:508-575) */
static const uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                   35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXTRA[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                   3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                   257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
                                   8193, 12289, 16385, 24577};
static const uint8_t DEXTRA[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6,
                                   7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

/* permutation of code-length code lengths (inflate.hpp:137-157) */
static const uint8_t PERM[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* readDynamicTreeCodes (inflate.hpp:166-206): fills lens[] for `iterations` entries starting
 * at index `base`; overshoot entries are written too (up to lens_cap). Returns new count. */
static int read_lengths(bitrd* b, const htree* pre, uint8_t* lens, int lens_cap, int start,
                        int iterations, int* last_len_io, int rfc, int* count_out) {
    int i = start;
    int last = *last_len_io;
    while (i < start + iterations) {
        int s;
        int e = ht_decode(pre, b, 7, 1, &s);
        if (e) return e;
        uint32_t rep;
        int val, cnt;
        if (s == 16) {
            if ((e = rd_bits(b, 2, &rep))) return e;
            cnt = (int)rep + 3;
            if (rfc && i == 0) return ORACLE_ERR_DATA;
            val = last;
        } else if (s == 17) {
            if ((e = rd_bits(b, 3, &rep))) return e;
            cnt = (int)rep + 3;
            val = 0;
        } else if (s == 18) {
            if ((e = rd_bits(b, 7, &rep))) return e;
            cnt = (int)rep + 11;
            val = 0;
        } else {
            cnt = 1;
            val = s;
        }
        for (int j = 0; j < cnt; j++, i++) {
            if (i < lens_cap) {
                lens[i] = (uint8_t)val;
            } else if (val != 0) {
                return ORACLE_ERR_DATA; /* reference: nonzero-length value >= 300 is UB */
            }
        }
        /* reference: last_code tracks literal lengths only; RFC: any previous length */
        if (s < 16 || rfc) last = val;
    }
    if (rfc && i > start + iterations) return ORACLE_ERR_DATA;
    *last_len_io = last;
    *count_out = i < lens_cap ? i : lens_cap;
    return 0;
}

static int decode_dynamic(bitrd* b, htree* lit, htree* dist, int rfc) {
    uint32_t hlit, hdist, hclen;
    int e;
    if ((e = rd_bits(b, 5, &hlit)) || (e = rd_bits(b, 5, &hdist)) || (e = rd_bits(b, 4, &hclen)))
        return e;
    uint8_t plen[19] = {0};
    for (uint32_t i = 0; i < hclen + 4; i++) {
        uint32_t v;
        if ((e = rd_bits(b, 3, &v))) return e;
        plen[PERM[i]] = (uint8_t)v;
    }
    htree pre;
    if ((e = ht_build(&pre, plen, 19))) { ht_free(&pre); return e; }
    uint8_t llen[512], dlen[512];
    memset(llen, 0, sizeof llen);
    memset(dlen, 0, sizeof dlen);
    int nl = 0, nd = 0;
    if (!rfc) {
        int last = 0;
        e = read_lengths(b, &pre, llen, 300, 0, 257 + (int)hlit, &last, 0, &nl);
        if (!e) {
            last = 0; /* fresh last_code per call (inflate.hpp:170) */
            e = read_lengths(b, &pre, dlen, 300, 0, 1 + (int)hdist, &last, 0, &nd);
        }
    } else {
        uint8_t all[600];
        memset(all, 0, sizeof all);
        int last = 0, tot = 0;
        e = read_lengths(b, &pre, all, 600, 0, 258 + (int)hlit + (int)hdist, &last, 1, &tot);
        if (!e) {
            nl = 257 + (int)hlit;
            nd = 1 + (int)hdist;
            memcpy(llen, all, (size_t)nl);
            memcpy(dlen, all + nl, (size_t)nd);
        }
    }
    ht_free(&pre);
    if (e) return e;
    if ((e = ht_build(lit, llen, nl))) return e;
    if ((e = ht_build(dist, dlen, nd))) return e;
    return 0;
}

static void fixed_trees(htree* lit, htree* dist) {
    uint8_t l[288], d[32];
    for (int i = 0; i < 144; i++) l[i] = 8;
    for (int i = 144; i < 256; i++) l[i] = 9;
    for (int i = 256; i < 280; i++) l[i] = 7;
    for (int i = 280; i < 288; i++) l[i] = 8;
    for (int i = 0; i < 32; i++) d[i] = 5;
    ht_build(lit, l, 288);  /* generateFixedCodes (common.hpp:442-482) */
    ht_build(dist, d, 32);  /* generateFixedDistanceCodes (common.hpp:484-495) */
}

/* decompressHuffmanBlock (inflate.hpp:226-275) */
static int huff_block(bitrd* b, obuf* o, const htree* lit, const htree* dist, int piece) {
    for (;;) {
        int s, e;
        if ((e = ht_decode(lit, b, 15, 0, &s))) return e;
        if (s < 256) {
            if ((e = ob_push(o, (uint8_t)s))) return e;
            continue;
        }
        if (s == 256) return 0;
        uint32_t length = 0, extra;
        if (s <= 285) {
            length = LBASE[s - 257];
            if (LEXTRA[s - 257]) {
                if ((e = rd_bits(b, LEXTRA[s - 257], &extra))) return e;
                length += extra;
            }
        }
        int ds;
        if ((e = ht_decode(dist, b, 16, 0, &ds))) return e;
        uint32_t distance = 0;
        if (ds < 30) {
            distance = DBASE[ds];
            if (DEXTRA[ds]) {
                if ((e = rd_bits(b, DEXTRA[ds], &extra))) return e;
                distance += extra;
            }
        }
        if (distance == 0 || length == 0) continue;
        if (distance > o->n) { /* copies nothing (inflate.hpp:268) */
            if (piece) return ORACLE_ERR_DATA;
            continue;
        }
        size_t src = o->n - distance;
        for (uint32_t j = 0; j < length; j++) {
            if ((e = ob_push(o, o->p[src + j]))) return e;
        }
    }
}

/* realDecompress (inflate.hpp:277-322) + decompress(void*, size_t) (inflate.hpp:363-374).
 * flags: ORACLE_RFC, ORACLE_PIECE. On success *out is malloc'd (caller frees with oracle_free). */
int oracle_inflate2(const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* out_len,
                    size_t* consumed);
int oracle_inflate(const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* out_len) {
    return oracle_inflate2(in, n, flags, out, out_len, NULL);
}

/* the same; *consumed (optional) = input bytes up to the end of the final block */
int oracle_inflate2(const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* out_len,
                    size_t* consumed) {
    int rfc = (flags & ORACLE_RFC) != 0, piece = (flags & ORACLE_PIECE) != 0;
    bitrd b = {in, n, 0, 0};
    obuf o = {NULL, 0, 0};
    htree flit, fdist;
    fixed_trees(&flit, &fdist);
    int e = 0;
    for (;;) {
        uint32_t final, type;
        if ((e = rd_bits(&b, 1, &final)) || (e = rd_bits(&b, 2, &type))) break;
        if (type == 0) {
            if (b.bit) { b.bit = 0; b.off++; } /* moveByte(true) */
            uint32_t len, nlen;
            if ((e = rd_bits(&b, 16, &len)) || (e = rd_bits(&b, 16, &nlen))) break;
            if (b.off + len > n) { e = ORACLE_ERR_OVERREAD; break; }
            for (uint32_t i = 0; i < len; i++)
                if ((e = ob_push(&o, in[b.off + i]))) break;
            if (e) break;
            b.off += len;
        } else if (type == 1) {
            if ((e = huff_block(&b, &o, &flit, &fdist, piece))) break;
        } else if (type == 2) {
            htree lit, dist;
            memset(&lit, 0, sizeof lit);
            memset(&dist, 0, sizeof dist);
            e = decode_dynamic(&b, &lit, &dist, rfc);
            if (!e) e = huff_block(&b, &o, &lit, &dist, piece);
            ht_free(&lit);
            ht_free(&dist);
            if (e) break;
        } /* type 3: no-op */
        if (final) break;
    }
    ht_free(&flit);
    ht_free(&fdist);
    if (e) {
        free(o.p);
        *out = NULL;
        *out_len = 0;
        return e;
    }
    *out = o.p ? o.p : (uint8_t*)malloc(1);
    *out_len = o.n;
    if (consumed) *consumed = b.off + (b.bit ? 1 : 0);
    return ORACLE_OK;
}

void oracle_free(void* p) { free(p); }
