// pm_synth.hip -- layout conversion (packed 4-bit codes <-> bit-planes) and the seeded
// on-device column generator used by bench.py and the full-size parity tests.
//
// Generator (SURVEY.md §8d "Synthetic inputs"): root i.i.d. uniform ACGT; per edge and
// site a substitution (mu = 1e-3, uniform to another base) and a gap opening (1e-4,
// geometric length, mean 5); at leaves IUPAC ambiguity (1e-5) and N-runs (start 1e-4,
// mean length 50).  Runs are clipped at global 32-site block boundaries.
// Randomness is counter-based (splitmix64 of seed, node, global site), so every rank and
// the CPU baseline see the same columns for the same global site.
#include "pm_bits.h"
#include "pm_internal.h"

namespace pm {
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t node, uint64_t site, uint64_t salt) {
    return mix64(seed ^ mix64(node * 0xD1B54A32D192ED03ull ^ mix64(site * 0xABC98388FB8FAC03ull + salt)));
}

// probabilities as thresholds on the low 32 bits
constexpr uint32_t kSub = 4294967u;        // 1e-3
constexpr uint32_t kGapOpen = 429497u;     // 1e-4
constexpr uint32_t kGapExtend = 3435973837u;  // 0.8  -> mean length 5
constexpr uint32_t kIupac = 42950u;        // 1e-5
constexpr uint32_t kNOpen = 429497u;       // 1e-4
constexpr uint32_t kNExtend = 4209067950u; // 0.98 -> mean length 50

__device__ __forceinline__ uint32_t base_from(uint32_t r) { return 1u << (r & 3u); }

// Run states (gap, N-run) restart at every global 32-site block and advance on random draws
// alone, so a word that starts mid-block (a shard boundary that is not a multiple of 32)
// first replays the draws of the block's earlier sites: every shard rule sees the same
// columns as one unsharded run.
__device__ uint4 evolve_word(uint4 par, uint64_t seed, uint64_t node, int64_t gsite0, bool leaf) {
    uint32_t b[4] = {0, 0, 0, 0};
    bool in_gap = false, in_n = false;
    for (int64_t gs = gsite0 - (gsite0 & 31); gs < gsite0; ++gs) {
        const uint32_t g = (uint32_t)rnd(seed, node, (uint64_t)gs, 2);
        in_gap = in_gap ? g < kGapExtend : g < kGapOpen;
        if (leaf) {
            const uint32_t nq = (uint32_t)rnd(seed, node, (uint64_t)gs, 4);
            in_n = in_n ? nq < kNExtend : nq < kNOpen;
        }
    }
    for (int k = 0; k < 32; ++k) {
        const uint64_t gs = (uint64_t)(gsite0 + k);
        if ((gs & 31u) == 0) in_gap = in_n = false;
        uint32_t c = code_at(par.x, par.y, par.z, par.w, k);
        const uint64_t r = rnd(seed, node, gs, 1);
        const uint32_t r0 = (uint32_t)r, r1 = (uint32_t)(r >> 32);
        if (c != 0 && r0 < kSub) {
            const uint32_t alt = base_from(r1);
            c = alt == c ? base_from(r1 + 1) : alt;
        }
        const uint32_t g = (uint32_t)rnd(seed, node, gs, 2);
        in_gap = in_gap ? g < kGapExtend : g < kGapOpen;
        if (in_gap) c = 0;
        if (leaf) {
            const uint32_t nq = (uint32_t)rnd(seed, node, gs, 4);
            in_n = in_n ? nq < kNExtend : nq < kNOpen;
            if (c != 0) {
                const uint64_t q = rnd(seed, node, gs, 3);
                if ((uint32_t)q < kIupac) {
                    const uint32_t amb[10] = {3, 5, 6, 7, 9, 10, 11, 12, 13, 14};
                    c = amb[(q >> 32) % 10];
                }
                if (in_n) c = 15;
            }
        }
        b[0] |= (c & 1u) << k;
        b[1] |= ((c >> 1) & 1u) << k;
        b[2] |= ((c >> 2) & 1u) << k;
        b[3] |= ((c >> 3) & 1u) << k;
    }
    return make_uint4(b[0], b[1], b[2], b[3]);
}

__global__ void k_synth_root(uint4* dst, uint64_t seed, int64_t site_begin, int64_t words, int64_t wpad) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= wpad) return;
    uint32_t b[4] = {0, 0, 0, 0};
    if (w < words) {
        for (int k = 0; k < 32; ++k) {
            const uint32_t c = base_from((uint32_t)rnd(seed, ~0ull, (uint64_t)(site_begin + w * 32 + k), 0));
            b[0] |= (c & 1u) << k;
            b[1] |= ((c >> 1) & 1u) << k;
            b[2] |= ((c >> 2) & 1u) << k;
            b[3] |= ((c >> 3) & 1u) << k;
        }
    }
    dst[w] = make_uint4(b[0], b[1], b[2], b[3]);
}

// One thread per (node of this depth, word).  `nodes` are dense internal indices
// (leaf == false, output into finals) or leaf ranks (leaf == true, output into leaf planes).
__global__ void k_synth_level(const int32_t* nodes, int32_t count, const int32_t* parent_of,
                              const int32_t* id_of, uint4* finals, uint4* leaf_planes, bool leaf,
                              uint64_t seed, int64_t site_begin, int64_t words, int64_t wpad) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)count * wpad) return;
    const int32_t i = (int32_t)(t / wpad);
    const int64_t w = t % wpad;
    const int32_t n = nodes[i];
    const uint4 par = finals[(size_t)parent_of[n] * wpad + w];
    uint4 out = make_uint4(0, 0, 0, 0);
    if (w < words) out = evolve_word(par, seed, (uint64_t)id_of[n], site_begin + w * 32, leaf);
    if (leaf) leaf_planes[(size_t)n * wpad + w] = out;
    else finals[(size_t)n * wpad + w] = out;
}

__global__ void k_pack_leaves(const uint8_t* codes4, int64_t row_stride, const int32_t* row_of_leaf,
                              const uint8_t* present, int64_t present_stride, uint4* planes,
                              uint32_t* present_planes, int32_t leaves, int64_t sites, int64_t wpad) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)leaves * wpad) return;
    const int32_t leaf = (int32_t)(t / wpad);
    const int64_t w = t % wpad;
    const int32_t row = row_of_leaf[leaf];
    uint32_t b[4] = {0, 0, 0, 0}, pm = 0;
    if (row >= 0) {
        for (int k = 0; k < 32; ++k) {
            const int64_t s = w * 32 + k;
            if (s >= sites) break;
            const uint8_t byte = codes4[(size_t)row * row_stride + (s >> 1)];
            const uint32_t c = (s & 1) ? (byte >> 4) : (byte & 15u);
            b[0] |= (c & 1u) << k;
            b[1] |= ((c >> 1) & 1u) << k;
            b[2] |= ((c >> 2) & 1u) << k;
            b[3] |= ((c >> 3) & 1u) << k;
            if (present && ((present[(size_t)row * present_stride + (s >> 3)] >> (s & 7)) & 1u)) pm |= 1u << k;
        }
    }
    planes[t] = make_uint4(b[0], b[1], b[2], b[3]);
    if (present_planes) present_planes[t] = pm;
}

__global__ void k_pack_sites(const uint8_t* codes4, uint4* dst, int64_t sites, int64_t wpad) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= wpad) return;
    uint32_t b[4] = {0, 0, 0, 0};
    for (int k = 0; k < 32; ++k) {
        const int64_t s = w * 32 + k;
        if (s >= sites) break;
        const uint8_t byte = codes4[s >> 1];
        const uint32_t c = (s & 1) ? (byte >> 4) : (byte & 15u);
        b[0] |= (c & 1u) << k;
        b[1] |= ((c >> 1) & 1u) << k;
        b[2] |= ((c >> 2) & 1u) << k;
        b[3] |= ((c >> 3) & 1u) << k;
    }
    dst[w] = make_uint4(b[0], b[1], b[2], b[3]);
}

__global__ void k_unpack_leaves(const uint4* planes, const uint8_t* flag, const uint32_t* present,
                                int32_t leaves, int64_t wpad, int64_t s0, int64_t ns, uint8_t* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)leaves * ns) return;
    const int32_t leaf = (int32_t)(t / ns);
    const int64_t s = s0 + t % ns;
    const int64_t w = s >> 5;
    const int k = (int)(s & 31);
    uint8_t c = 0;
    if (flag[leaf] != kLeafAbsent) {
        const uint4 q = planes[(size_t)leaf * wpad + w];
        const bool here = flag[leaf] == kLeafPresent || ((present[(size_t)leaf * wpad + w] >> k) & 1u);
        if (here) c = (uint8_t)code_at(q.x, q.y, q.z, q.w, k);
    }
    out[t] = c;
}

__global__ void k_unpack_sites(const uint4* src, int64_t s0, int64_t ns, uint8_t* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ns) return;
    const int64_t s = s0 + t;
    const uint4 q = src[s >> 5];
    out[t] = (uint8_t)code_at(q.x, q.y, q.z, q.w, (int)(s & 31));
}

inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

hipError_t launch_pack_codes(pm_ctx* c, const uint8_t* d_codes4, int64_t row_stride, const int32_t* d_row_of_leaf,
                             const uint8_t* d_present, int64_t present_stride) {
    const int64_t wpad = (int64_t)((c->words + kWave - 1) / kWave) * kWave;
    const int64_t n = (int64_t)c->dt.num_leaves * wpad;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_leaves, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, d_codes4, row_stride,
                       d_row_of_leaf, d_present, present_stride, c->leaf_planes, d_present ? c->leaf_present : nullptr,
                       c->dt.num_leaves, c->num_sites, wpad);
    return hipGetLastError();
}

hipError_t launch_pack_sites(pm_ctx* c, const uint8_t* d_codes4, uint4* dst) {
    const int64_t wpad = (int64_t)((c->words + kWave - 1) / kWave) * kWave;
    hipLaunchKernelGGL(k_pack_sites, dim3(blocks_for(wpad, 256)), dim3(256), 0, c->stream, d_codes4, dst,
                       c->num_sites, wpad);
    return hipGetLastError();
}

hipError_t launch_synth(pm_ctx* c, int64_t site_begin, uint64_t seed) {
    const HostTree& ht = c->ht;
    const DevTree& dt = c->dt;
    const int64_t wpad = (int64_t)((c->words + kWave - 1) / kWave) * kWave;
    uint4* root_dst = c->finals + (size_t)dt.root_dense * wpad;
    hipLaunchKernelGGL(k_synth_root, dim3(blocks_for(wpad, 256)), dim3(256), 0, c->stream, root_dst, seed,
                       site_begin, (int64_t)c->words, wpad);
    const int D = (int)ht.down_level_off.size() - 1;
    for (int d = 0; d < D; ++d) {
        // internal nodes at depth d (d >= 1), then leaves at depth d
        if (d >= 1) {
            const int32_t cnt = ht.down_level_off[d + 1] - ht.down_level_off[d];
            if (cnt > 0)
                hipLaunchKernelGGL(k_synth_level, dim3(blocks_for((int64_t)cnt * wpad, 256)), dim3(256), 0,
                                   c->stream, dt.down_order + ht.down_level_off[d], cnt, dt.parent_dense,
                                   dt.internal_id, c->finals, c->leaf_planes, false, seed, site_begin,
                                   (int64_t)c->words, wpad);
        }
    }
    const int DL = (int)ht.leaf_level_off.size() - 1;
    for (int d = 0; d < DL; ++d) {
        const int32_t cnt = ht.leaf_level_off[d + 1] - ht.leaf_level_off[d];
        if (cnt > 0)
            hipLaunchKernelGGL(k_synth_level, dim3(blocks_for((int64_t)cnt * wpad, 256)), dim3(256), 0, c->stream,
                               dt.leaf_down + ht.leaf_level_off[d], cnt, dt.leaf_parent, dt.leaf_id, c->finals,
                               c->leaf_planes, true, seed, site_begin, (int64_t)c->words, wpad);
    }
    return hipMemcpyAsync(c->cons, root_dst, sizeof(uint4) * wpad, hipMemcpyDeviceToDevice, c->stream);
}

// S2 / S3 leaf layout (pm_ctx::sub_planes): thread = (S2 / S3 item, word), its three or four
// leaves' words copied side by side (tail descriptors hold the leaves, -1 padded).
__global__ __launch_bounds__(256) void k_sub_planes(const TailDesc* tail, int32_t num_s, const uint4* leaf_planes,
                                                    int64_t wpad, uint4* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)num_s * wpad) return;
    const int32_t item = (int32_t)(i / wpad);
    const int64_t word = i - (int64_t)item * wpad;
    const TailDesc& t = tail[item];
    uint4* o = out + (size_t)i * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = t.vl[j] >= 0 ? leaf_planes[(size_t)t.vl[j] * wpad + word] : make_uint4(0, 0, 0, 0);
}

hipError_t launch_sub_planes(pm_ctx* c) {
    const int64_t wpad = (int64_t)((c->words + kWave - 1) / kWave) * kWave;
    const int64_t n = (int64_t)c->ht.num_tail_s * wpad;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sub_planes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->dt.tail_desc_k,
                       c->ht.num_tail_s, c->leaf_planes, wpad, c->sub_planes);
    return hipGetLastError();
}

hipError_t launch_unpack_leaf_codes(pm_ctx* c, int64_t s0, int64_t ns, uint8_t* d_out) {
    const int64_t wpad = (int64_t)((c->words + kWave - 1) / kWave) * kWave;
    const int64_t n = (int64_t)c->dt.num_leaves * ns;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_leaves, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, c->leaf_planes,
                       c->leaf_flag, c->leaf_present, c->dt.num_leaves, wpad, s0, ns, d_out);
    return hipGetLastError();
}

hipError_t launch_unpack_sites(pm_ctx* c, const uint4* src, int64_t s0, int64_t ns, uint8_t* d_out) {
    if (ns == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_sites, dim3(blocks_for(ns, 256)), dim3(256), 0, c->stream, src, s0, ns, d_out);
    return hipGetLastError();
}

// This file's code object, loaded ahead of its first launch (pm_warmup).
hipError_t warm_synth() {
    hipFuncAttributes at;
    return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_pack_sites));
}

}  // namespace pm
