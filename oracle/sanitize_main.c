/* oracle/sanitize_main.c -- TEST INFRASTRUCTURE ONLY (never linked into libdmx).
 *
 * Driver for an AddressSanitizer + UndefinedBehaviorSanitizer build of the oracle
 * (`make -C oracle san` -> oracle/_san/oracle_san; tests/test_oracle_sanitizers.py).  argv[1] is
 * a list file, one job per line: "<stream> <out> <flags>".  For each job the oracle inflates the
 * stream; the return code goes to stdout ("<rc> <len>") and, on success, the bytes to <out>.
 * Then every stream is inflated again cut at 16 lengths and with 16 single-bit flips (seeded,
 * deterministic): those runs only have to end without a sanitizer report -- they walk the
 * oracle's error paths (over-reads, bad codes, oversized copies) under ASan/UBSan.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_inflate(const uint8_t* in, size_t n, uint32_t flags, uint8_t** out, size_t* out_len);
void oracle_free(void* p);

static uint8_t* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* p = (uint8_t*)malloc(sz > 0 ? (size_t)sz : 1);
    if (p && sz > 0 && fread(p, 1, (size_t)sz, f) != (size_t)sz) {
        free(p);
        p = NULL;
    }
    fclose(f);
    *n = sz > 0 ? (size_t)sz : 0;
    return p;
}

/* inflate an exact-size heap copy, so that any read past the stream is an ASan report */
static int run(const uint8_t* s, size_t n, uint32_t flags, uint8_t** out, size_t* len) {
    uint8_t* c = (uint8_t*)malloc(n ? n : 1);
    if (n) memcpy(c, s, n);
    int rc = oracle_inflate(c, n, flags, out, len);
    free(c);
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* lf = fopen(argv[1], "r");
    if (!lf) return 2;
    char sp[4096], op[4096];
    unsigned flags;
    uint64_t seed = 0x5EED5A4Eull;
    long jobs = 0, mutants = 0;
    while (fscanf(lf, "%4095s %4095s %u", sp, op, &flags) == 3) {
        size_t n = 0;
        uint8_t* s = read_file(sp, &n);
        if (!s) return 3;
        uint8_t* out = NULL;
        size_t len = 0;
        int rc = run(s, n, flags, &out, &len);
        printf("%d %zu\n", rc, len);
        if (rc == 0) {
            FILE* of = fopen(op, "wb");
            if (!of) return 4;
            if (len && fwrite(out, 1, len, of) != len) return 4;
            fclose(of);
            oracle_free(out);
        }
        jobs++;
        /* error paths: truncations and bit flips (results ignored) */
        for (int k = 0; k < 16 && n; k++) {
            seed = seed * 6364136223846793005ull + 1442695040888963407ull;
            size_t cut = (size_t)((seed >> 33) % n);
            if (run(s, cut, flags, &out, &len) == 0) oracle_free(out);
            uint8_t* m = (uint8_t*)malloc(n);
            memcpy(m, s, n);
            seed = seed * 6364136223846793005ull + 1442695040888963407ull;
            const size_t bit = (size_t)((seed >> 17) % (8 * (uint64_t)n));
            m[bit >> 3] ^= (uint8_t)(1u << (bit & 7));
            if (run(m, n, flags, &out, &len) == 0) oracle_free(out);
            free(m);
            mutants += 2;
        }
        free(s);
    }
    fclose(lf);
    fprintf(stderr, "oracle_san: %ld streams, %ld mutants\n", jobs, mutants);
    return 0;
}
