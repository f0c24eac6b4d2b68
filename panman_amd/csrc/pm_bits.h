// pm_bits.h -- bit-sliced state arithmetic for 32 alignment sites per 32-bit word.
//
// A Fitch state set (src/fitchSankoff.cpp:30-56 keeps it as `1 << code`, 16 bits) is held
// as 16 one-hot bit-planes: bit b of plane v is set iff code v is in the set of site b.
// A final (single) code is held as 4 code bit-planes.  Intersection / union / emptiness
// over 32 sites are then single VALU ops per plane.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pm {

// 4 code planes -> 16 one-hot planes; `m` masks present sites (absent sites -> empty set).
__device__ __forceinline__ void onehot_from_code(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3,
                                                 uint32_t m, uint32_t* out) {
    const uint32_t n0 = ~b0, n1 = ~b1, n2 = ~b2, n3 = ~b3;
    const uint32_t lo[4] = {n0 & n1, b0 & n1, n0 & b1, b0 & b1};
    const uint32_t hi[4] = {n2 & n3 & m, b2 & n3 & m, n2 & b3 & m, b2 & b3 & m};
#pragma unroll
    for (int v = 0; v < 16; ++v) out[v] = lo[v & 3] & hi[v >> 2];
}

// one-hot planes (at most one bit per site across planes) -> 4 code planes
__device__ __forceinline__ void code_from_onehot(const uint32_t* in, uint32_t& b0, uint32_t& b1,
                                                 uint32_t& b2, uint32_t& b3) {
    const uint32_t p01 = in[1] | in[3], p05 = in[5] | in[7], p09 = in[9] | in[11], p13 = in[13] | in[15];
    b0 = p01 | p05 | p09 | p13;
    const uint32_t q2 = in[2] | in[3], q6 = in[6] | in[7], q10 = in[10] | in[11], q14 = in[14] | in[15];
    b1 = q2 | q6 | q10 | q14;
    b2 = in[4] | in[5] | q6 | in[12] | in[13] | q14;
    b3 = in[8] | in[9] | q10 | in[12] | in[13] | q14;
}

// lowest set code per site (the reference's `currentState <<= 1` scan, :107-113, :118-121)
__device__ __forceinline__ void lowest_code(const uint32_t* s, uint32_t* out) {
    uint32_t seen = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        out[v] = s[v] & ~seen;
        seen |= s[v];
    }
}

// bitwise select, bit by bit: t ? a : b (one v_bfi_b32)
// A 16-B store that streams to memory (non-temporal): replay rows (written once; C5 17 %
// faster than plain stores, r05n) and the post-order's set records (read by the next level's
// launch; N* Fitch post-order 8.2 -> 7.8 ms, Sankoff 10.9 -> 9.9 ms, r05o).
__device__ __forceinline__ void store_stream(uint4* p, const uint4& v) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 nv = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(nv, reinterpret_cast<u32x4*>(p));
}

__device__ __forceinline__ uint32_t bsel(uint32_t t, uint32_t a, uint32_t b) { return (t & a) | (~t & b); }

// Plane c of a 16-plane set, site by site (c in 4 code planes): a 16:1 multiplexer.
__device__ __forceinline__ uint32_t plane_at(const uint32_t* s, const uint32_t* c) {
    uint32_t m8[8], m4[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) m8[k] = bsel(c[0], s[2 * k + 1], s[2 * k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) m4[k] = bsel(c[1], m8[2 * k + 1], m8[2 * k]);
    return bsel(c[3], bsel(c[2], m4[3], m4[2]), bsel(c[2], m4[1], m4[0]));
}

// Lowest code of each site's set in code-plane form (0 for an empty set) by a binary
// search from the top code bit; returns the sites with a non-empty set.
__device__ __forceinline__ uint32_t lowest_code_planes(const uint32_t* s, uint32_t* c) {
    const uint32_t l8 = s[0] | s[1] | s[2] | s[3] | s[4] | s[5] | s[6] | s[7];
    uint32_t h[8], q[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = bsel(l8, s[k], s[8 + k]);
    const uint32_t l4 = h[0] | h[1] | h[2] | h[3];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = bsel(l4, h[k], h[4 + k]);
    const uint32_t l2 = q[0] | q[1];
    const uint32_t r0 = bsel(l2, q[0], q[2]), r1 = bsel(l2, q[1], q[3]);
    const uint32_t any = r0 | r1;
    c[0] = ~r0 & any;
    c[1] = ~l2 & any;
    c[2] = ~l4 & any;
    c[3] = ~l8 & any;
    return any;
}

__device__ __forceinline__ uint32_t any_plane(const uint32_t* s) {
    uint32_t r = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) r |= s[v];
    return r;
}

__device__ __forceinline__ uint32_t code_at(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, int bit) {
    return ((b0 >> bit) & 1u) | (((b1 >> bit) & 1u) << 1) | (((b2 >> bit) & 1u) << 2) |
           (((b3 >> bit) & 1u) << 3);
}

// 64-lane inclusive prefix sum by DPP lane moves (no LDS round trips): shifts of 1, 2, 4, 8
// inside each 16-lane row, then row 0's / rows 0-1's totals broadcast to the rows above
// (row_bcast:15, row_bcast:31 -- the gfx9 family's DPP broadcasts).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    const int lane = threadIdx.x & 63, r = lane & 15;
    uint32_t t;
    t = dpp_mov<0x111>(v); if (r >= 1) v += t;    // row_shr:1
    t = dpp_mov<0x112>(v); if (r >= 2) v += t;    // row_shr:2
    t = dpp_mov<0x114>(v); if (r >= 4) v += t;    // row_shr:4
    t = dpp_mov<0x118>(v); if (r >= 8) v += t;    // row_shr:8
    t = dpp_mov<0x142>(v); if (lane & 16) v += t; // row_bcast:15 -> rows 1, 3
    t = dpp_mov<0x143>(v); if (lane >= 32) v += t; // row_bcast:31 -> rows 2, 3
    return v;
}

// 64-lane exclusive prefix sum; returns the wave total through `total`.  Every lane active.
__device__ __forceinline__ uint32_t wave_exclusive_scan(uint32_t v, uint32_t& total) {
    const uint32_t incl = wave_inclusive_scan(v);
    total = __builtin_amdgcn_readlane(incl, 63);
    return incl - v;
}

// A workgroup barrier that orders LDS only: each wave's LDS accesses are complete (lgkmcnt)
// and visible to the others, while its global stores and loads stay in flight.  __syncthreads()
// is a workgroup release / acquire over global memory too, which on gfx950 waits for every
// outstanding vector memory operation (vmcnt(0)): in the replay (behind a tile's write-out) and the
// post-order sweeps (behind a round's record stores) a full HBM write round trip.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

}  // namespace pm
