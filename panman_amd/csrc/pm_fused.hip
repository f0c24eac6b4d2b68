// pm_fused.hip -- Fitch over subtree regions: intermediate state sets live in LDS.
//
// Same algorithm as k_fitch_up / k_down<Fitch> (src/fitchSankoff.cpp:30-171), but the
// tree is cut into connected regions of <= kRegionSlots internal nodes (host:
// build_regions).  One wavefront owns (region, 64-word tile):
//   k_region_up    stages the region's leaf children in LDS, evaluates the region's nodes
//                  in post-order with every set in an LDS slot, and writes only the region
//                  root's set to HBM.
//   k_region_down  re-evaluates the region from its leaves (cheaper than storing every
//                  set), then walks it parents-first: final state per node (kept in the
//                  parent's LDS slot), mutations of the node and its leaf children, and
//                  finals published to HBM only for nodes with children in other regions.
// HBM traffic per site drops from 1.5 L + 7 I bytes (one set write + two set reads per
// internal node) to ~ L + 7 R bytes for R regions.  Lanes only ever touch their own LDS
// words, so no barriers are needed (one wave per workgroup).
#include "pm_kernels.h"

namespace pm {
namespace {

struct FusedArgs {
    const int32_t* order;
    int32_t count;
    const int32_t* node_off;
    const int32_t* node_dense;
    const int32_t* node_pslot;
    const int32_t* node_flags;
    const int32_t* child_off;
    const int32_t* child;
    const int32_t* stage_off;
    const int32_t* stage;
    const uint8_t* leaf_flag;
    const uint4* leaf_planes;
    const uint32_t* leaf_present;
    uint4* sets;
    uint64_t* cmask;
    uint4* finals;
    const uint4* cons;
    const uint4* forced;
    const int32_t* parent_dense;
    const int32_t* internal_id;
    const int32_t* leaf_id;
    int32_t root_dense;
    int32_t tiles;
    int64_t wpad;
    int64_t words;
    int64_t sites;
    pm_mut* recs;
    int64_t shard_cap;
    uint32_t* shard_cnt;
    uint8_t* root_code;
    bool absent_code0;   // always false here (leaf_set16 / leaf_diff contract)
};

struct Lds {
    uint4 slot[kRegionSlots * 4 * kWave];   // [slot][quad][lane]
    uint4 stage[kRegionStage * kWave];      // staged leaf code planes
    uint32_t mask[kRegionStage * kWave];    // staged leaf presence
};

// One region per workgroup (one wave); the device functions address it directly.
__shared__ Lds s;

__device__ __forceinline__ void stage_leaves(const FusedArgs& a, int32_t r, int lane, int64_t word) {
    const int32_t s0 = __builtin_amdgcn_readfirstlane(a.stage_off[r]);
    const int32_t s1 = __builtin_amdgcn_readfirstlane(a.stage_off[r + 1]);
    uint4 v[kRegionStage];
    uint32_t m[kRegionStage];
#pragma unroll
    for (int k = 0; k < kRegionStage; ++k) {
        v[k] = make_uint4(0, 0, 0, 0);
        m[k] = 0;
        if (s0 + k < s1) {
            const int32_t leaf = __builtin_amdgcn_readfirstlane(a.stage[s0 + k]);
            const uint8_t flag = a.leaf_flag[leaf];
            if (flag != kLeafAbsent) {
                v[k] = a.leaf_planes[(size_t)leaf * a.wpad + word];
                m[k] = flag == kLeafPartial ? a.leaf_present[(size_t)leaf * a.wpad + word] : ~0u;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kRegionStage; ++k)
        if (s0 + k < s1) {
            s.stage[k * kWave + lane] = v[k];
            s.mask[k * kWave + lane] = m[k];
        }
}

__device__ __forceinline__ void slot_load(int sl, int lane, uint32_t* x) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = s.slot[(sl * 4 + q) * kWave + lane];
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ void slot_store(int sl, int lane, const uint32_t* x) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s.slot[(sl * 4 + q) * kWave + lane] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
}

// Post-order over the region (src/fitchSankoff.cpp:30-56); the region root's set goes to
// HBM (up pass) or to its slot (down pass).
__device__ __forceinline__ void region_sets(const FusedArgs& a, int32_t r, int tile, int lane, int64_t word, bool root_to_hbm) {
    const int32_t n0 = __builtin_amdgcn_readfirstlane(a.node_off[r]);
    const int32_t n1 = __builtin_amdgcn_readfirstlane(a.node_off[r + 1]);
    for (int32_t e = n0; e < n1; ++e) {
        uint32_t both[16], either[16], x[16];
#pragma unroll
        for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
        const int32_t c0 = __builtin_amdgcn_readfirstlane(a.child_off[e]);
        const int32_t c1 = __builtin_amdgcn_readfirstlane(a.child_off[e + 1]);
        for (int32_t j = c0; j < c1; ++j) {
            const int32_t cc = __builtin_amdgcn_readfirstlane(a.child[j]);
            const int kind = cc & 3, val = cc >> 2;
            if (kind == 0) {
                const uint4 L = s.stage[val * kWave + lane];
                onehot_from_code(L.x, L.y, L.z, L.w, s.mask[val * kWave + lane], x);
            } else if (kind == 1) {
                leaf_set16(a, val, word, x);
            } else if (kind == 2) {
                slot_load(val, lane, x);
            } else {
                load_fitch_set(a.sets, a.cmask, a.cons, val, a.tiles, tile, lane, word, x);
            }
#pragma unroll
            for (int v = 0; v < 16; ++v) { both[v] &= x[v]; either[v] |= x[v]; }
        }
        const uint32_t nz = any_plane(both);
#pragma unroll
        for (int v = 0; v < 16; ++v) x[v] = both[v] | (either[v] & ~nz);
        const int32_t dense = __builtin_amdgcn_readfirstlane(a.node_dense[e]);
        if (dense == a.root_dense && a.forced != nullptr) {   // refState (src/fitchSankoff.cpp:45-47)
            const uint4 F = a.forced[word];
            onehot_from_code(F.x, F.y, F.z, F.w, ~0u, x);
        }
        if (e == n1 - 1 && root_to_hbm) {
            uint64_t mx, ms;   // the region kernels keep full finals, no mask push needed
            store_fitch_set(a.sets, a.cmask, a.cons[word], dense, a.tiles, tile, lane, x, true, mx, ms);
        }
        else slot_store(e - n0, lane, x);
    }
}

__global__ __launch_bounds__(kWave) void k_region_up(FusedArgs a) {
    const int lane = threadIdx.x;
    const int32_t r = __builtin_amdgcn_readfirstlane(a.order[blockIdx.x]);
    const int tile = blockIdx.y;
    const int64_t word = (int64_t)tile * kWave + lane;
    stage_leaves(a, r, lane, word);
    region_sets(a, r, tile, lane, word, true);
}

__device__ __forceinline__ uint32_t staged_diff(int val, int lane, uint32_t valid, const uint32_t* F,
                                                uint4& L) {
    L = s.stage[val * kWave + lane];
    return valid & s.mask[val * kWave + lane] & ((L.x ^ F[0]) | (L.y ^ F[1]) | (L.z ^ F[2]) | (L.w ^ F[3]));
}

// Parent's final codes of region entry e: the region root reads HBM (or the consensus),
// others the parent's slot (quad 0).
__device__ __forceinline__ uint4 parent_codes(const FusedArgs& a, int32_t e, int32_t n1, int32_t dense,
                                              bool is_root, int lane, int64_t word) {
    // read both without selecting between an LDS and a global pointer (gfx950 codegen)
    const int ps = max(__builtin_amdgcn_readfirstlane(a.node_pslot[e]), 0);
    uint4 v = s.slot[(ps * 4) * kWave + lane];
    // pin the LDS load so LLVM cannot merge it with the global one into a flat-pointer phi
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    if (e == n1 - 1) v = is_root ? a.cons[word] : a.finals[(size_t)a.parent_dense[dense] * a.wpad + word];
    return v;
}

// Mutations of region entry e and of its leaf children: count only (EMIT = false) or
// write them at out[pos...] (EMIT = true).  Returns the lane's record count.
template <bool EMIT>
__device__ __forceinline__ uint32_t node_mutations(const FusedArgs& a, int32_t r, int32_t e, int32_t n0,
                                                   int32_t n1, int lane, int64_t word, uint32_t valid, pm_mut* out,
                                                   int64_t pos) {
    const int32_t dense = __builtin_amdgcn_readfirstlane(a.node_dense[e]);
    const uint4 f4 = s.slot[((e - n0) * 4) * kWave + lane];
    const uint32_t pres = s.slot[((e - n0) * 4 + 1) * kWave + lane].x;
    const uint4 q = parent_codes(a, e, n1, dense, dense == a.root_dense, lane, word);
    const uint32_t F[4] = {f4.x, f4.y, f4.z, f4.w};
    const uint32_t pc[4] = {q.x, q.y, q.z, q.w};
    const uint32_t self_diff = pres & valid & ((F[0] ^ pc[0]) | (F[1] ^ pc[1]) | (F[2] ^ pc[2]) | (F[3] ^ pc[3]));
    uint32_t k = 0;
    if (EMIT) k += emit_at(out, pos, a.shard_cap, (uint32_t)a.internal_id[dense], self_diff, word, pc, F[0], F[1], F[2], F[3]);
    else k += __builtin_popcount(self_diff);
    const int32_t c0 = __builtin_amdgcn_readfirstlane(a.child_off[e]);
    const int32_t c1 = __builtin_amdgcn_readfirstlane(a.child_off[e + 1]);
    for (int32_t j = c0; j < c1; ++j) {
        const int32_t cc = __builtin_amdgcn_readfirstlane(a.child[j]);
        const int kind = cc & 3;
        if (kind > 1) continue;
        if (kind == 0) {
            const int sv = cc >> 2;
            const uint4 L = s.stage[sv * kWave + lane];
            const uint32_t d = valid & s.mask[sv * kWave + lane] & ((L.x ^ F[0]) | (L.y ^ F[1]) | (L.z ^ F[2]) | (L.w ^ F[3]));
            if (!EMIT) k += __builtin_popcount(d);
            else if (d) k += emit_at(out, pos + k, a.shard_cap, (uint32_t)a.leaf_id[a.stage[a.stage_off[r] + sv]], d, word, F,
                                  L.x, L.y, L.z, L.w);
        } else {
            uint4 G;
            const uint32_t d = leaf_diff(a, cc >> 2, word, valid, F, G);
            if (!EMIT) k += __builtin_popcount(d);
            else if (d) k += emit_at(out, pos + k, a.shard_cap, (uint32_t)a.leaf_id[cc >> 2], d, word, F, G.x, G.y, G.z, G.w);
        }
    }
    return k;
}

__global__ __launch_bounds__(kWave) void k_region_down(FusedArgs a) {
    const int lane = threadIdx.x;
    const int32_t r = __builtin_amdgcn_readfirstlane(a.order[blockIdx.x]);
    const int tile = blockIdx.y;
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t valid = valid_mask(a, word);
    stage_leaves(a, r, lane, word);
    region_sets(a, r, tile, lane, word, false);

    const int32_t n0 = __builtin_amdgcn_readfirstlane(a.node_off[r]);
    const int32_t n1 = __builtin_amdgcn_readfirstlane(a.node_off[r + 1]);
    // pass 1, parents first: final codes; a node's slot becomes {F, (pres, -, -, -), ...}
    for (int32_t e = n1 - 1; e >= n0; --e) {
        const int32_t dense = __builtin_amdgcn_readfirstlane(a.node_dense[e]);
        const bool is_root = dense == a.root_dense;
        uint32_t own[16], P[16], fin[16];
        slot_load(e - n0, lane, own);
        uint4 q = parent_codes(a, e, n1, dense, is_root, lane, word);
        onehot_from_code(q.x, q.y, q.z, q.w, ~0u, P);
        const uint32_t pres = any_plane(own);
        lowest_code(own, fin);
        if (!is_root) {   // parent & own ? parent : lowest(own)  (src/fitchSankoff.cpp:115-123)
            uint32_t hit = 0;
#pragma unroll
            for (int v = 0; v < 16; ++v) hit |= P[v] & own[v];
#pragma unroll
            for (int v = 0; v < 16; ++v) fin[v] = (P[v] & hit) | (fin[v] & ~hit);
        }
        uint32_t F[4];
        code_from_onehot(fin, F[0], F[1], F[2], F[3]);
        s.slot[((e - n0) * 4) * kWave + lane] = make_uint4(F[0], F[1], F[2], F[3]);
        s.slot[((e - n0) * 4 + 1) * kWave + lane] = make_uint4(pres, 0, 0, 0);
        if (__builtin_amdgcn_readfirstlane(a.node_flags[e]) & 1)
            a.finals[(size_t)dense * a.wpad + word] = make_uint4(F[0], F[1], F[2], F[3]);
        if (is_root) {
            for (int b = 0; b < 32; ++b) {
                const int64_t site = word * 32 + b;
                if (site < a.sites)
                    a.root_code[site] = ((pres >> b) & 1u) ? (uint8_t)code_at(F[0], F[1], F[2], F[3], b) : (uint8_t)255;
            }
        }
    }
    // pass 2: count every mutation of the region (nodes + leaf children), one atomic per wave;
    // pass 3: write them (src/fitchSankoff.cpp:131-171)
    uint32_t count = 0;
    for (int32_t e = n0; e < n1; ++e) count += node_mutations<false>(a, r, e, n0, n1, lane, word, valid, nullptr, 0);
    uint32_t total;
    const uint32_t excl = wave_exclusive_scan(count, total);
    if (total == 0) return;
    const uint32_t shard = (uint32_t)(blockIdx.x + blockIdx.y * 7919u) % kShards;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.shard_cnt[shard], total);
    base = __shfl(base, 0, 64);
    pm_mut* out = a.recs + (size_t)shard * a.shard_cap;
    int64_t pos = (int64_t)base + excl;
    for (int32_t e = n0; e < n1; ++e) pos += node_mutations<true>(a, r, e, n0, n1, lane, word, valid, out, pos);
}

}  // namespace

hipError_t launch_fitch_fused(pm_ctx* c) {
    const HostTree& ht = c->ht;
    const DevTree& dt = c->dt;
    const int32_t tiles = (c->words + kWave - 1) / kWave;
    FusedArgs a{};
    a.node_off = dt.rg_node_off;
    a.node_dense = dt.rg_node_dense;
    a.node_pslot = dt.rg_node_pslot;
    a.node_flags = dt.rg_node_flags;
    a.child_off = dt.rg_child_off;
    a.child = dt.rg_child;
    a.stage_off = dt.rg_stage_off;
    a.stage = dt.rg_stage;
    a.leaf_flag = c->leaf_flag;
    a.leaf_planes = c->leaf_planes;
    a.leaf_present = c->leaf_present;
    a.sets = reinterpret_cast<uint4*>(c->sets);
    a.cmask = c->cmask;
    a.finals = c->finals;
    a.cons = c->cons;
    a.forced = c->has_forced ? c->forced : nullptr;
    a.parent_dense = dt.parent_dense;
    a.internal_id = dt.internal_id;
    a.leaf_id = dt.leaf_id;
    a.root_dense = dt.root_dense;
    a.tiles = tiles;
    a.wpad = (int64_t)tiles * kWave;
    a.words = c->words;
    a.sites = c->num_sites;
    a.recs = c->recs;
    a.shard_cap = c->shard_cap;
    a.shard_cnt = c->shard_cnt;
    a.root_code = c->root_code;
    a.absent_code0 = false;
    const int H = (int)ht.rg_up_level_off.size() - 1;
    for (int h = 0; h < H; ++h) {
        a.order = dt.rg_up_order + ht.rg_up_level_off[h];
        a.count = ht.rg_up_level_off[h + 1] - ht.rg_up_level_off[h];
        timer_begin(c, 0);
        hipLaunchKernelGGL(k_region_up, dim3(a.count, tiles), dim3(kWave), 0, c->stream, a);
        timer_end(c, 0);
    }
    hipError_t e = hipMemsetAsync(c->shard_cnt, 0, sizeof(uint32_t) * kShards, c->stream);
    if (e != hipSuccess) return e;
    const int D = (int)ht.rg_down_level_off.size() - 1;
    for (int d = 0; d < D; ++d) {
        a.order = dt.rg_down_order + ht.rg_down_level_off[d];
        a.count = ht.rg_down_level_off[d + 1] - ht.rg_down_level_off[d];
        timer_begin(c, 1);
        hipLaunchKernelGGL(k_region_down, dim3(a.count, tiles), dim3(kWave), 0, c->stream, a);
        timer_end(c, 1);
    }
    return hipGetLastError();
}

}  // namespace pm
