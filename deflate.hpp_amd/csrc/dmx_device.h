// dmx_device.h -- device-side helpers shared by the deflate and inflate kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmx {

// RFC 1951 length / distance tables; the same values as the reference's RangeLookup
// (common.hpp:508-575).
__constant__ const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,
                                            15, 17, 19, 23, 27, 31, 35, 43, 51,  59,
                                            67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                            2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ const uint16_t kDistBase[30] = {1,    2,    3,    4,     5,     7,    9,    13,
                                             17,   25,   33,   49,    65,    97,   129,  193,
                                             257,  385,  513,  769,   1025,  1537, 2049, 3073,
                                             4097, 6145, 8193, 12289, 16385, 24577};
__constant__ const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3,  3,  4,  4,  5,  5,  6,
                                             6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
// code-length code order (RFC 1951 3.2.7; reference inflate.hpp:137-157)
__constant__ const uint8_t kPerm[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5,
                                        11, 4,  12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// LDS hand-off between the lanes of ONE wavefront (DS instructions of a wave execute in order;
// this only keeps the compiler from moving LDS accesses across it)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// length 3..258 -> lit/len symbol 257..285
__device__ __forceinline__ uint32_t len_sym(uint32_t L) {
    if (L <= 10) return 254 + L;
    if (L == 258) return 285;
    uint32_t x = L - 3;               // 8..254
    uint32_t k = 31 - __clz(x);       // 3..7
    return 257 + 4 * (k - 1) + ((x >> (k - 2)) & 3);
}
// distance 1..32768 -> distance symbol 0..29
__device__ __forceinline__ uint32_t dist_sym(uint32_t d) {
    if (d <= 4) return d - 1;
    uint32_t x = d - 1;
    uint32_t k = 31 - __clz(x);       // >= 2
    return 2 * k + ((x >> (k - 1)) & 1);
}

// RFC 1951 3.2.5 length / distance code parameters by arithmetic (no table loads in hot loops)
__device__ __forceinline__ uint32_t len_extra(uint32_t s) {  // s in 257..285
    return (s >= 265 && s < 285) ? (s - 261) >> 2 : 0;
}
__device__ __forceinline__ uint32_t len_base(uint32_t s) {
    if (s < 265) return s - 254;
    if (s >= 285) return 258;
    return ((4 + ((s - 265) & 3)) << ((s - 261) >> 2)) + 3;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t d) {  // d in 0..29
    return d < 4 ? 0 : (d >> 1) - 1;
}
__device__ __forceinline__ uint32_t dist_base(uint32_t d) {
    return d < 4 ? d + 1 : ((2 + (d & 1)) << ((d >> 1) - 1)) + 1;
}

__device__ __forceinline__ uint32_t bitrev(uint32_t v, uint32_t n) {
    return n ? (__builtin_bitreverse32(v) >> (32 - n)) : 0;
}

// unaligned 32-bit read from an LDS byte image accessed as words (image padded by >= 8 B)
__device__ __forceinline__ uint32_t ld32u(const uint32_t* w, uint32_t p) {
    uint32_t i = p >> 2, sh = p & 3;
    return __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

// inclusive wave64 scan (sum)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Sorts 512 keys held as k[8] per lane (element index = lane * 8 + r) into descending order
// with a register bitonic network (45 stages; cross-lane stages use ds_bpermute shuffles).
// v from lane (lane ^ M) for a compile-time M: DPP on the VALU for M < 16 (quad_perm for 1/2,
// mirrors composed for 4/8), ds_swizzle for 16, ds_bpermute only for 32.
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
    } else if constexpr (M == 4) {                                                  // ^7 then ^3
        const int h = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);     // row_half_mirror
        return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);         // [3,2,1,0]
    } else if constexpr (M == 8) {                                                  // ^15 then ^7
        const int m = __builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);     // row_mirror
        return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x141, 0xF, 0xF, false);        // row_half_mirror
    } else if constexpr (M == 16) {
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);               // xor_mask 16
    } else {
        return (uint32_t)__shfl_xor((int)v, M, 64);
    }
}

template <int M>
__device__ __forceinline__ void sort512_xstage(uint32_t (&k)[8], int lane, int stride, int size) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int i = lane * 8 + r;
        const uint32_t o = xor_lane<M>(k[r]);
        const bool lower = (i & stride) == 0;
        const bool desc = (i & size) == 0;
        k[r] = (lower == desc) ? max(k[r], o) : min(k[r], o);
    }
}

__device__ __forceinline__ void wave_sort512_desc(uint32_t (&k)[8]) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 512; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 8) {
                switch (stride >> 3) {
                    case 1: sort512_xstage<1>(k, lane, stride, size); break;
                    case 2: sort512_xstage<2>(k, lane, stride, size); break;
                    case 4: sort512_xstage<4>(k, lane, stride, size); break;
                    case 8: sort512_xstage<8>(k, lane, stride, size); break;
                    case 16: sort512_xstage<16>(k, lane, stride, size); break;
                    default: sort512_xstage<32>(k, lane, stride, size); break;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const int p = r ^ stride;
                    if (p > r) {
                        const bool desc = ((lane * 8 + r) & size) == 0;
                        const uint32_t a = k[r], b = k[p];
                        k[r] = desc ? max(a, b) : min(a, b);
                        k[p] = desc ? min(a, b) : max(a, b);
                    }
                }
            }
        }
    }
}

}  // namespace dmx
