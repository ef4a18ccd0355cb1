// checksum.hip -- Adler-32 (RFC 1950) and CRC-32 (RFC 1952, ISO-HDLC) of device buffers (gfx950).
//
// The reference has no checksums: decompressZlib skips the 2-byte header and ignores the
// trailer (inflate.hpp:326-361, SURVEY A-9).  These kernels back the zlib / gzip containers
// of SURVEY 8(f) row 4 (dmx_deflate_zlib / _gzip, dmx_inflate_zlib / _gzip).  Both checksums
// are computed block-parallel and combined with their linear structure:
//
//   Adler-32 over bytes x_0..x_{n-1} continuing from (a0, b0):
//     A = a0 + sum x_i,  B = b0 + n a0 + sum (n - i) x_i        (mod 65521)
//   so a block [o, o + m) contributes S1 = sum x and S2' = sum (E - i) x_i with E its virtual
//   end; B adds S2' + (N - E) S1.  One 256-thread workgroup sums 16 KiB (64 B per lane), one
//   workgroup folds all blocks.
//
//   CRC-32 register R (reflected, polynomial 0xEDB88320) is affine in its start value, and the
//   zero-start register of a concatenation is  R0(X || Y) = R0(X) * x^(8|Y|) xor R0(Y)  in
//   GF(2)[x] / P.  Each lane runs the byte-wise table on 64 bytes (zero start), workgroups fold
//   lanes by that rule (x^(8 * 64 * 2^k) from a host-made table of x^(8 * 2^k)), and tree
//   kernels fold 1024 results at a time until one is left; the host applies the start value
//   and the final complement.
//
// Misaligned buffers are read from the 16-byte boundary below them; the bytes before the
// buffer are masked to zero, which leaves both sums unchanged (zero bytes add nothing to S1 and
// S2 is weighted from the end; a zero-start CRC register stays zero over zero bytes).
#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

constexpr uint32_t CK_NT = 256;          // threads per workgroup
constexpr uint32_t CK_RUN = 64;          // bytes per lane
constexpr uint32_t CK_BLK = CK_NT * CK_RUN;  // 16 KiB per workgroup
constexpr uint32_t ADLER_MOD = 65521;

// four 16-byte loads of one lane's run, bytes outside [lead, vend) masked to zero
__device__ __forceinline__ void ck_load_run(const uint8_t* vbase, uint64_t g, uint64_t lead, uint64_t vend,
                                            uint32_t (&w)[16]) {
    const uint64_t b0 = g * CK_RUN;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint64_t qb = b0 + 16 * q;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (qb < vend) v = *reinterpret_cast<const uint4*>(vbase + qb);
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
    if (b0 < lead || b0 + CK_RUN > vend) {  // edge runs only
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint32_t m = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint64_t p = b0 + 4 * k + b;
                if (p >= lead && p < vend) m |= 0xFFu << (8 * b);
            }
            w[k] &= m;
        }
    }
}

// ---- Adler-32 ------------------------------------------------------------------------------
__global__ __launch_bounds__(CK_NT) void k_adler_blocks(const uint8_t* vbase, uint64_t lead, uint64_t vend,
                                                        uint2* part) {
    __shared__ uint64_t s2w[CK_NT / 64];
    __shared__ uint32_t s1w[CK_NT / 64];
    const uint32_t t = threadIdx.x;
    const uint64_t g = (uint64_t)blockIdx.x * CK_NT + t;
    uint32_t w[16];
    ck_load_run(vbase, g, lead, vend, w);
    // s1 = sum x_r, s2 = sum (64 - r) x_r over the run
    uint32_t s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t x = (w[k] >> (8 * b)) & 0xFFu;
            s1 += x;
            s2 += (uint32_t)(CK_RUN - (4 * k + b)) * x;
        }
    }
    // block sums with full 16 KiB weights: S2 = sum_t s2_t + s1_t (CK_BLK - 64 (t + 1))
    uint64_t S2 = (uint64_t)s2 + (uint64_t)s1 * (CK_BLK - CK_RUN * (t + 1));
    uint32_t S1 = s1;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        S1 += (uint32_t)__shfl_xor((int)S1, d, 64);
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)S2, d, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(S2 >> 32), d, 64);
        S2 += ((uint64_t)hi << 32) | lo;
    }
    if ((t & 63) == 0) {
        s1w[t >> 6] = S1;
        s2w[t >> 6] = S2;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t a = 0, b = 0;
#pragma unroll
        for (int i = 0; i < (int)(CK_NT / 64); i++) {
            a += s1w[i];
            b += s2w[i];
        }
        part[blockIdx.x] = make_uint2((uint32_t)(a % ADLER_MOD), (uint32_t)(b % ADLER_MOD));
    }
}

// fold: A = a0 + sum S1_b, B = b0 + n a0 + sum S2_b + (N - E_b) S1_b  (N = vend, E_b = block end)
__global__ __launch_bounds__(1024) void k_adler_fold(const uint2* part, uint64_t nblk, uint64_t vend, uint64_t n,
                                                     uint32_t init, uint32_t* out) {
    __shared__ uint64_t sa[16], sb[16];
    const uint32_t t = threadIdx.x;
    uint64_t a = 0, b = 0;
    for (uint64_t i = t; i < nblk; i += 1024) {
        const uint2 p = part[i];
        const int64_t dist = (int64_t)vend - (int64_t)((i + 1) * CK_BLK);  // < 0 only for the last block
        int64_t f = dist % (int64_t)ADLER_MOD;
        if (f < 0) f += ADLER_MOD;
        a += p.x;
        b += p.y + (uint64_t)f * p.x % ADLER_MOD;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        a += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), d, 64) << 32) |
             (uint32_t)__shfl_xor((int)(uint32_t)a, d, 64);
        b += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(b >> 32), d, 64) << 32) |
             (uint32_t)__shfl_xor((int)(uint32_t)b, d, 64);
    }
    if ((t & 63) == 0) {
        sa[t >> 6] = a;
        sb[t >> 6] = b;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t A = 0, B = 0;
        for (int i = 0; i < 16; i++) {
            A += sa[i] % ADLER_MOD;
            B += sb[i] % ADLER_MOD;
        }
        const uint64_t a0 = init & 0xFFFFu, b0 = init >> 16;
        A = (A + a0) % ADLER_MOD;
        B = (B + b0 + (n % ADLER_MOD) * a0) % ADLER_MOD;
        *out = (uint32_t)((B << 16) | A);
    }
}

// ---- CRC-32 --------------------------------------------------------------------------------
struct CrcPow {
    uint32_t xp[48];  // xp[k] = x^(8 * 2^k) mod P, reflected
};

// a * b mod P in the reflected representation (bit 31 = x^0)
__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll 8
    for (int i = 0; i < 32; i++) {
        r ^= (b & 0x80000000u) ? a : 0u;
        b <<= 1;
        a = (a >> 1) ^ ((a & 1u) ? 0xEDB88320u : 0u);
    }
    return r;
}
// x^(8 L) mod P from the power table
__device__ __forceinline__ uint32_t gf_xpow8(uint64_t L, const CrcPow& X) {
    uint32_t r = 0x80000000u;  // 1
    for (int k = 0; L; k++, L >>= 1)
        if (L & 1) r = gf_mul(r, X.xp[k]);
    return r;
}

// one lane-level value per thread -> tree fold over the workgroup; len[t] = valid bytes.
// Folding pairs (left, right): R = R_left * x^(8 len_right) xor R_right.  A right subtree with
// the full size 2^k * unit takes its power from the table; the one ragged subtree computes it.
template <int NT>
__device__ uint32_t crc_tree_fold(uint32_t R, uint64_t len, uint32_t* sR, uint64_t* sL, int unit_log2,
                                  const CrcPow& X) {
    const uint32_t t = threadIdx.x;
    sR[t] = R;
    sL[t] = len;
    __syncthreads();
    int k = 0;
    for (uint32_t s = 1; s < (uint32_t)NT; s <<= 1, k++) {
        if ((t & (2 * s - 1)) == 0) {
            const uint32_t rr = sR[t + s];
            const uint64_t lr = sL[t + s];
            const uint64_t full = (uint64_t)1 << (unit_log2 + k);
            const uint32_t xp = lr == full ? X.xp[unit_log2 + k] : gf_xpow8(lr, X);
            sR[t] = gf_mul(sR[t], lr ? xp : 0x80000000u) ^ rr;
            sL[t] += lr;
        }
        __syncthreads();
    }
    return sR[0];
}

__global__ __launch_bounds__(CK_NT) void k_crc_blocks(const uint8_t* vbase, uint64_t lead, uint64_t vend,
                                                      CrcPow X, uint32_t* part, uint64_t* plen) {
    __shared__ uint32_t T[256];
    __shared__ uint32_t sR[CK_NT];
    __shared__ uint64_t sL[CK_NT];
    const uint32_t t = threadIdx.x;
    {
        uint32_t c = t;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? 0xEDB88320u : 0u);
        T[t] = c;
    }
    const uint64_t g = (uint64_t)blockIdx.x * CK_NT + t;
    uint32_t w[16];
    ck_load_run(vbase, g, lead, vend, w);
    __syncthreads();
    const uint64_t b0 = g * CK_RUN;
    // valid bytes of the run that lie before the end; leading masked zeros are fed through the
    // zero-start register (it stays zero), trailing bytes past vend are not fed at all
    const uint32_t nfeed = b0 >= vend ? 0u : (uint32_t)min((uint64_t)CK_RUN, vend - b0);
    const uint32_t nlead = b0 >= lead ? 0u : (uint32_t)min((uint64_t)CK_RUN, lead - b0);
    uint32_t R = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
            if ((uint32_t)(4 * k + b) < nfeed) R = T[(R ^ (w[k] >> (8 * b))) & 0xFFu] ^ (R >> 8);
        }
    }
    const uint64_t len = nfeed > nlead ? nfeed - nlead : 0u;  // bytes of the buffer in this run
    // a run holding only leading zeros has R = 0 and length 0: it folds as the identity
    const uint32_t Rb = crc_tree_fold<CK_NT>(nfeed > nlead ? R : 0u, len, sR, sL, 6, X);
    if (t == 0) {
        part[blockIdx.x] = Rb;
        plen[blockIdx.x] = sL[0];
    }
}

// folds 1024 consecutive (R, len) pairs of uniform unit size 2^unit_log2 (the last may be short)
__global__ __launch_bounds__(1024) void k_crc_tree(const uint32_t* inR, const uint64_t* inL, uint64_t nin,
                                                   int unit_log2, CrcPow X, uint32_t* outR, uint64_t* outL) {
    __shared__ uint32_t sR[1024];
    __shared__ uint64_t sL[1024];
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint32_t R = i < nin ? inR[i] : 0u;
    const uint64_t L = i < nin ? inL[i] : 0u;
    const uint32_t Rb = crc_tree_fold<1024>(R, L, sR, sL, unit_log2, X);
    if (threadIdx.x == 0) {
        outR[blockIdx.x] = Rb;
        outL[blockIdx.x] = sL[0];
    }
}

namespace {
uint32_t gf_mul_host(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 32; i++) {
        if (b & 0x80000000u) r ^= a;
        b <<= 1;
        a = (a >> 1) ^ ((a & 1u) ? 0xEDB88320u : 0u);
    }
    return r;
}
CrcPow make_pow() {
    CrcPow X;
    uint32_t p = 0x00800000u;  // x^8 (reflected: bit 31 - 8)
    for (int k = 0; k < 48; k++) {
        X.xp[k] = p;
        p = gf_mul_host(p, p);
    }
    return X;
}
uint32_t xpow8_host(uint64_t L, const CrcPow& X) {
    uint32_t r = 0x80000000u;
    for (int k = 0; L; k++, L >>= 1)
        if (L & 1) r = gf_mul_host(r, X.xp[k]);
    return r;
}
}  // namespace

uint64_t checksum_scratch_bytes(uint64_t n) {
    const uint64_t nblk = (n + 16 + CK_BLK - 1) / CK_BLK + 1;
    return 2 * (nblk * 12 + 64);
}

hipError_t launch_adler32(const uint8_t* d, uint64_t n, uint32_t init, void* scratch, uint32_t* d_out,
                          hipStream_t st) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(d) & ~(uintptr_t)15;
    const uint64_t lead = reinterpret_cast<uintptr_t>(d) - a;
    const uint64_t vend = lead + n;
    const uint64_t nblk = (vend + CK_BLK - 1) / CK_BLK;
    uint2* part = static_cast<uint2*>(scratch);
    if (nblk)
        hipLaunchKernelGGL(k_adler_blocks, dim3((uint32_t)nblk), dim3(CK_NT), 0, st,
                           reinterpret_cast<const uint8_t*>(a), lead, vend, part);
    hipLaunchKernelGGL(k_adler_fold, dim3(1), dim3(1024), 0, st, part, nblk, vend, n, init, d_out);
    return hipGetLastError();
}

// writes the zero-start register of the buffer to *d_out (the host applies start and final xor)
hipError_t launch_crc32_raw(const uint8_t* d, uint64_t n, void* scratch, uint32_t* d_out, hipStream_t st) {
    static const CrcPow X = make_pow();
    const uintptr_t a = reinterpret_cast<uintptr_t>(d) & ~(uintptr_t)15;
    const uint64_t lead = reinterpret_cast<uintptr_t>(d) - a;
    const uint64_t vend = lead + n;
    uint64_t nblk = (vend + CK_BLK - 1) / CK_BLK;
    if (nblk == 0) return hipMemsetAsync(d_out, 0, 4, st);
    const uint64_t half = (nblk + 64) * 12;
    uint32_t* R0 = static_cast<uint32_t*>(scratch);
    uint64_t* L0 = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(scratch) + ((nblk * 4 + 15) & ~15ull));
    uint8_t* s2 = static_cast<uint8_t*>(scratch) + half + 64;
    uint32_t* R1 = reinterpret_cast<uint32_t*>(s2);
    uint64_t* L1 = reinterpret_cast<uint64_t*>(s2 + ((nblk * 4 + 15) & ~15ull));
    hipLaunchKernelGGL(k_crc_blocks, dim3((uint32_t)nblk), dim3(CK_NT), 0, st,
                       reinterpret_cast<const uint8_t*>(a), lead, vend, X, R0, L0);
    int unit = 14;  // log2(CK_BLK)
    while (nblk > 1) {
        const uint64_t nout = (nblk + 1023) / 1024;
        hipLaunchKernelGGL(k_crc_tree, dim3((uint32_t)nout), dim3(1024), 0, st, R0, L0, nblk, unit, X, R1, L1);
        std::swap(R0, R1);
        std::swap(L0, L1);
        nblk = nout;
        unit += 10;
    }
    return hipMemcpyAsync(d_out, R0, 4, hipMemcpyDeviceToDevice, st);
}

uint32_t crc32_finish(uint32_t raw, uint64_t n, uint32_t init) {
    static const CrcPow X = make_pow();
    // register after the buffer from start register ~init: (~init) * x^(8n) xor raw
    const uint32_t reg = gf_mul_host(~init, xpow8_host(n, X)) ^ raw;
    return ~reg;
}

}  // namespace dmx
