// pm_chunk.h -- the packed per-site result chunk every multi-GPU path gathers.
//
// Columns are independent (src/panman.cpp:1381 Fitch, :1568 Sankoff), so ranks own disjoint
// contiguous site ranges.  Each rank contributes ONE fixed-size chunk of `per` u64 entries to
// the all-gather:
//   entry 0         head = site_begin << 32 | count   (count = kChunkFailed: the rank's shard
//                   failed; it still joins the collective so no rank blocks in it)
//   entries 1..count  score (int32, low half) | root code (u8, bits 32-39) of its sites
// `per` = ceil(S / ranks) + 3 holds every shard rule in use: the balanced split r*S/n
// (pm_shard_range) and the MSA driver's even-aligned one (pm_msa.cpp), both at most
// ceil(S / ranks) + 2 sites wide.  The same functions run in the device pack / unpack kernels
// (pm_rccl.hip) and in the host entry points pm_chunk_pack / pm_chunk_unpack, so the CPU tests
// check exactly the layout the GPUs move.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pm {

constexpr uint32_t kChunkFailed = 0xffffffffu;

__host__ __device__ inline int64_t chunk_entries(int64_t total_sites, int ranks) {
    return (total_sites + ranks - 1) / ranks + 3;
}

__host__ __device__ inline uint64_t chunk_head(int64_t site_begin, int64_t count) {
    return ((uint64_t)site_begin << 32) | (uint64_t)(uint32_t)count;
}

__host__ __device__ inline uint64_t chunk_failed_head() { return (uint64_t)kChunkFailed; }

__host__ __device__ inline uint64_t chunk_entry(int32_t score, uint8_t root) {
    return (uint64_t)(uint32_t)score | ((uint64_t)root << 32);
}

__host__ __device__ inline int64_t head_begin(uint64_t head) { return (int64_t)(head >> 32); }
__host__ __device__ inline uint32_t head_count(uint64_t head) { return (uint32_t)(head & 0xffffffffu); }

// Entry g of the gathered buffer (ranks x per entries): write its site's score / root, if it
// is a site entry of a healthy rank inside [0, total).
__host__ __device__ inline void chunk_unpack_one(const uint64_t* all, int64_t per, int64_t g, int64_t total,
                                                 int32_t* score, uint8_t* root) {
    const int64_t r = g / per, i = g - r * per;
    if (i == 0) return;
    const uint64_t head = all[r * per];
    const uint32_t count = head_count(head);
    if (count == kChunkFailed || i > (int64_t)count) return;
    const int64_t site = head_begin(head) + i - 1;
    if (site >= total) return;
    const uint64_t e = all[g];
    score[site] = (int32_t)(uint32_t)e;
    root[site] = (uint8_t)(e >> 32);
}

// Status of a gathered buffer from its heads: 0 = every rank healthy and the ranges tile
// [0, total) exactly; 1 + r = rank r reported a failed shard; -1 = ranges overlap, leave gaps
// or run past `total` (shard rules disagree between ranks).
__host__ __device__ inline int chunk_check(const uint64_t* all, int64_t per, int ranks, int64_t total) {
    int64_t covered = 0;
    for (int r = 0; r < ranks; ++r) {
        const uint64_t h = all[(int64_t)r * per];
        if (head_count(h) == kChunkFailed) return 1 + r;
        const int64_t b = head_begin(h), n = head_count(h);
        if (n > per - 1 || b + n > total) return -1;
        for (int q = 0; q < r; ++q) {   // disjoint from every earlier rank's range
            const uint64_t g = all[(int64_t)q * per];
            const int64_t gb = head_begin(g), gn = head_count(g);
            if (n > 0 && gn > 0 && b < gb + gn && gb < b + n) return -1;
        }
        covered += n;
    }
    return covered == total ? 0 : -1;
}

}  // namespace pm
