// pm_fitch.hip -- Fitch small parsimony over every alignment column at once (gfx950).
//
// Restates, for all sites together, the per-column recursion of the reference:
//   post-order  Tree::nucFitchForwardPass      src/fitchSankoff.cpp:30-56      -> k_fitch_up
//   pre-order   Tree::nucFitchBackwardPass     src/fitchSankoff.cpp:96-129     -> k_fitch_down
//   assignment  Tree::nucFitchAssignMutations  src/fitchSankoff.cpp:131-171    -> k_fitch_down
//   score       (edges with a change; the gather target of SURVEY.md §8e)        -> k_site_score
//
// Work decomposition: one wavefront = one tree node x one tile of 64 words (2048 sites);
// lane = one 32-site word.  The node (and therefore its child list) is wave-uniform, so
// child loads are scalar and there is no divergence; every lane streams 64 B (Fitch set)
// or 16 B (leaf / final codes) through fully coalesced 1 KiB wave-instructions.  Levels
// (heights for the post-order, depths for the pre-order) are separate launches.
// Integer bit-set work only: no MFMA (SURVEY.md §8d roofline is HBM bandwidth).
#include "pm_bits.h"
#include "pm_internal.h"

namespace pm {
namespace {

struct UpArgs {
    const int32_t* order;
    int32_t count;
    const int32_t* child_off;
    const int32_t* child_enc;
    const uint8_t* leaf_flag;
    const uint4* leaf_planes;
    const uint32_t* leaf_present;
    uint4* sets;
    const uint4* forced;   // nullable
    int32_t root_dense;
    int32_t tiles;
    int64_t wpad;
};

__device__ __forceinline__ void load_set16(const uint4* sets, int64_t node, int32_t tiles, int tile,
                                           int lane, uint32_t* s) {
    const uint4* p = sets + ((size_t)node * tiles + tile) * 256 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = p[q * 64];
        s[4 * q + 0] = v.x;
        s[4 * q + 1] = v.y;
        s[4 * q + 2] = v.z;
        s[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ void store_set16(uint4* sets, int64_t node, int32_t tiles, int tile,
                                            int lane, const uint32_t* s) {
    uint4* p = sets + ((size_t)node * tiles + tile) * 256 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q * 64] = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}

// Leaf child as a one-hot set: src/fitchSankoff.cpp:32-38 (absent leaf -> 0).
__device__ __forceinline__ void leaf_set16(const UpArgs& a, int32_t leaf, int64_t word, uint32_t* s) {
    const uint8_t flag = a.leaf_flag[leaf];
    if (flag == kLeafAbsent) {
#pragma unroll
        for (int v = 0; v < 16; ++v) s[v] = 0;
        return;
    }
    const uint4 L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    const uint32_t m = flag == kLeafPartial ? a.leaf_present[(size_t)leaf * a.wpad + word] : ~0u;
    onehot_from_code(L.x, L.y, L.z, L.w, m, s);
}

__global__ __launch_bounds__(kBlock) void k_fitch_up(UpArgs a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t item = blockIdx.x * kWavesPerBlock + wave;
    if (item >= a.count) return;
    const int32_t n = __builtin_amdgcn_readfirstlane(a.order[item]);
    const int tile = blockIdx.y;
    const int64_t word = (int64_t)tile * kWave + lane;

    uint32_t both[16], either[16], s[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
    const int32_t e0 = __builtin_amdgcn_readfirstlane(a.child_off[n]);
    const int32_t e1 = __builtin_amdgcn_readfirstlane(a.child_off[n + 1]);
    for (int32_t e = e0; e < e1; ++e) {
        const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        if (c >= 0) load_set16(a.sets, c, a.tiles, tile, lane, s);
        else leaf_set16(a, -c - 1, word, s);
#pragma unroll
        for (int v = 0; v < 16; ++v) { both[v] &= s[v]; either[v] |= s[v]; }
    }
    // AND if non-empty, else OR (src/fitchSankoff.cpp:48-55)
    const uint32_t nz = any_plane(both);
#pragma unroll
    for (int v = 0; v < 16; ++v) s[v] = both[v] | (either[v] & ~nz);
    if (n == a.root_dense && a.forced != nullptr) {
        // refState replaces the root's set (src/fitchSankoff.cpp:45-47)
        const uint4 F = a.forced[word];
        onehot_from_code(F.x, F.y, F.z, F.w, ~0u, s);
    }
    store_set16(a.sets, n, a.tiles, tile, lane, s);
}

struct DownArgs {
    const int32_t* order;
    int32_t count;
    const int32_t* child_off;
    const int32_t* child_enc;
    const int32_t* parent_dense;
    const int32_t* internal_id;
    const int32_t* leaf_id;
    const uint8_t* leaf_flag;
    const uint4* leaf_planes;
    const uint32_t* leaf_present;
    const uint4* sets;
    uint4* finals;
    const uint4* cons;
    int32_t root_dense;
    int32_t tiles;
    int64_t wpad;
    int64_t words;
    int64_t sites;
    pm_mut* recs;
    int64_t shard_cap;
    uint32_t* shard_cnt;
    uint8_t* root_code;
};

__device__ __forceinline__ uint32_t valid_mask(const DownArgs& a, int64_t word) {
    if (word >= a.words) return 0u;
    const int64_t left = a.sites - word * 32;
    return left >= 32 ? ~0u : ((1u << left) - 1u);
}

// Leaf mutation mask against the parent's final codes F (leaf final = own code).
__device__ __forceinline__ uint32_t leaf_diff(const DownArgs& a, int32_t leaf, int64_t word, uint32_t valid,
                                              const uint32_t* F, uint4& L) {
    const uint8_t flag = a.leaf_flag[leaf];
    if (flag == kLeafAbsent) return 0u;
    L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    uint32_t m = valid;
    if (flag == kLeafPartial) m &= a.leaf_present[(size_t)leaf * a.wpad + word];
    return m & ((L.x ^ F[0]) | (L.y ^ F[1]) | (L.z ^ F[2]) | (L.w ^ F[3]));
}

// One record per changed site (src/fitchSankoff.cpp:140-166): parent gap -> NI,
// child gap -> ND (char '-', code 0), else NS; NI/NS carry the child's code.
__device__ __forceinline__ uint32_t emit(pm_mut* out, int64_t pos, int64_t cap, uint32_t node, uint32_t diff,
                                         int64_t word, const uint32_t* pc, uint32_t c0, uint32_t c1,
                                         uint32_t c2, uint32_t c3) {
    uint32_t k = 0;
    while (diff) {
        const int b = __builtin_ctz(diff);
        diff &= diff - 1;
        const uint32_t p = code_at(pc[0], pc[1], pc[2], pc[3], b);
        const uint32_t c = code_at(c0, c1, c2, c3, b);
        const uint32_t type = p == 0 ? PM_MUT_NI : (c == 0 ? PM_MUT_ND : PM_MUT_NS);
        const uint32_t site = (uint32_t)(word * 32 + b);
        if (pos + k < cap) out[pos + k] = pm_mut{node, (site << 8) | (type << 4) | (type == PM_MUT_ND ? 0u : c)};
        ++k;
    }
    return k;
}

__global__ __launch_bounds__(kBlock) void k_fitch_down(DownArgs a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t item = blockIdx.x * kWavesPerBlock + wave;
    if (item >= a.count) return;   // whole wave leaves together
    const int32_t n = __builtin_amdgcn_readfirstlane(a.order[item]);
    const int tile = blockIdx.y;
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t valid = valid_mask(a, word);

    uint32_t own[16], P[16], fin[16], pc[4];
    load_set16(a.sets, n, a.tiles, tile, lane, own);
    const bool is_root = n == a.root_dense;
    {
        uint4 q = is_root ? a.cons[word] : a.finals[(size_t)a.parent_dense[n] * a.wpad + word];
        pc[0] = q.x; pc[1] = q.y; pc[2] = q.z; pc[3] = q.w;
    }
    onehot_from_code(pc[0], pc[1], pc[2], pc[3], ~0u, P);
    const uint32_t pres = any_plane(own);   // state 0: subtree absent, skipped (:101-103, :136-138)
    lowest_code(own, fin);
    if (!is_root) {
        // parent & own ? parent : lowest(own)   (src/fitchSankoff.cpp:115-123)
        uint32_t hit = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) hit |= P[v] & own[v];
#pragma unroll
        for (int v = 0; v < 16; ++v) fin[v] = (P[v] & hit) | (fin[v] & ~hit);
    }
    uint32_t F[4];
    code_from_onehot(fin, F[0], F[1], F[2], F[3]);
    a.finals[(size_t)n * a.wpad + word] = make_uint4(F[0], F[1], F[2], F[3]);

    const uint32_t self_diff = pres & valid & ((F[0] ^ pc[0]) | (F[1] ^ pc[1]) | (F[2] ^ pc[2]) | (F[3] ^ pc[3]));
    uint32_t count = __builtin_popcount(self_diff);
    const int32_t e0 = __builtin_amdgcn_readfirstlane(a.child_off[n]);
    const int32_t e1 = __builtin_amdgcn_readfirstlane(a.child_off[n + 1]);
    // The first kCached leaf children keep their planes and masks in registers for the
    // emission pass (binary trees: every leaf child); further ones are reloaded.
    constexpr int kCached = 2;
    uint4 cl[kCached];
    uint32_t cd[kCached];
    int32_t cid[kCached];
    int ncached = 0;
    for (int32_t e = e0; e < e1; ++e) {
        const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        if (c >= 0) continue;
        uint4 L;
        const uint32_t d = leaf_diff(a, -c - 1, word, valid, F, L);
        count += __builtin_popcount(d);
        if (ncached < kCached) {
#pragma unroll
            for (int k = 0; k < kCached; ++k)
                if (k == ncached) { cl[k] = L; cd[k] = d; cid[k] = e; }
            ++ncached;
        }
    }

    if (is_root) {
        for (int b = 0; b < 32; ++b) {
            const int64_t site = word * 32 + b;
            if (site < a.sites)
                a.root_code[site] = ((pres >> b) & 1u) ? (uint8_t)code_at(F[0], F[1], F[2], F[3], b) : (uint8_t)255;
        }
    }

    uint32_t total;
    const uint32_t excl = wave_exclusive_scan(count, total);
    if (total == 0) return;
    const uint32_t shard = (uint32_t)(blockIdx.x * kWavesPerBlock + wave + blockIdx.y * 7919u) % kShards;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.shard_cnt[shard], total);
    base = __shfl(base, 0, 64);
    pm_mut* out = a.recs + (size_t)shard * a.shard_cap;
    int64_t pos = (int64_t)base + excl;

    pos += emit(out, pos, a.shard_cap, (uint32_t)a.internal_id[n], self_diff, word, pc, F[0], F[1], F[2], F[3]);
#pragma unroll
    for (int k = 0; k < kCached; ++k) {
        if (k >= ncached) break;
        const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[cid[k]]);
        if (cd[k]) pos += emit(out, pos, a.shard_cap, (uint32_t)a.leaf_id[-c - 1], cd[k], word, F, cl[k].x, cl[k].y,
                               cl[k].z, cl[k].w);
    }
    if (ncached == kCached) {
        int seen = 0;
        for (int32_t e = e0; e < e1; ++e) {
            const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
            if (c >= 0 || seen++ < kCached) continue;
            uint4 L;
            const uint32_t d = leaf_diff(a, -c - 1, word, valid, F, L);
            if (d) pos += emit(out, pos, a.shard_cap, (uint32_t)a.leaf_id[-c - 1], d, word, F, L.x, L.y, L.z, L.w);
        }
    }
}

// Per-site score = mutated edges below the root.  Records of a shard are histogrammed in
// LDS (sites fit) or straight into global counters.
__global__ __launch_bounds__(kBlock) void k_site_score(const pm_mut* recs, const uint32_t* shard_cnt,
                                                       int64_t shard_cap, uint32_t root_id, int32_t* score,
                                                       int64_t sites, int shards_per_block, bool use_lds) {
    extern __shared__ uint32_t hist[];
    if (use_lds) {
        for (int64_t s = threadIdx.x; s < sites; s += blockDim.x) hist[s] = 0;
        __syncthreads();
    }
    for (int k = 0; k < shards_per_block; ++k) {
        const int shard = blockIdx.x * shards_per_block + k;
        if (shard >= kShards) break;
        const int64_t n = min((int64_t)shard_cnt[shard], shard_cap);
        const pm_mut* r = recs + (size_t)shard * shard_cap;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const pm_mut m = r[i];
            if (m.node == root_id) continue;
            const uint32_t site = m.site_info >> 8;
            if (use_lds) atomicAdd(&hist[site], 1u);
            else atomicAdd(&score[site], 1);
        }
    }
    if (use_lds) {
        __syncthreads();
        for (int64_t s = threadIdx.x; s < sites; s += blockDim.x)
            if (hist[s]) atomicAdd(&score[s], (int32_t)hist[s]);
    }
}

}  // namespace

hipError_t launch_fitch(pm_ctx* c) {
    const HostTree& ht = c->ht;
    const DevTree& dt = c->dt;
    const int32_t tiles = (c->words + kWave - 1) / kWave;
    const int64_t wpad = (int64_t)tiles * kWave;

    UpArgs up{};
    up.child_off = dt.child_off;
    up.child_enc = dt.child_enc;
    up.leaf_flag = c->leaf_flag;
    up.leaf_planes = c->leaf_planes;
    up.leaf_present = c->leaf_present;
    up.sets = reinterpret_cast<uint4*>(c->sets);
    up.forced = c->has_forced ? c->forced : nullptr;
    up.root_dense = dt.root_dense;
    up.tiles = tiles;
    up.wpad = wpad;
    const int H = (int)ht.up_level_off.size() - 1;
    for (int h = 0; h < H; ++h) {
        up.order = dt.up_order + ht.up_level_off[h];
        up.count = ht.up_level_off[h + 1] - ht.up_level_off[h];
        dim3 grid((up.count + kWavesPerBlock - 1) / kWavesPerBlock, tiles);
        timer_begin(c, 0);
        hipLaunchKernelGGL(k_fitch_up, grid, dim3(kBlock), 0, c->stream, up);
        timer_end(c, 0);
    }

    hipError_t e = hipMemsetAsync(c->shard_cnt, 0, sizeof(uint32_t) * kShards, c->stream);
    if (e != hipSuccess) return e;
    DownArgs dn{};
    dn.child_off = dt.child_off;
    dn.child_enc = dt.child_enc;
    dn.parent_dense = dt.parent_dense;
    dn.internal_id = dt.internal_id;
    dn.leaf_id = dt.leaf_id;
    dn.leaf_flag = c->leaf_flag;
    dn.leaf_planes = c->leaf_planes;
    dn.leaf_present = c->leaf_present;
    dn.sets = reinterpret_cast<const uint4*>(c->sets);
    dn.finals = c->finals;
    dn.cons = c->cons;
    dn.root_dense = dt.root_dense;
    dn.tiles = tiles;
    dn.wpad = wpad;
    dn.words = c->words;
    dn.sites = c->num_sites;
    dn.recs = c->recs;
    dn.shard_cap = c->shard_cap;
    dn.shard_cnt = c->shard_cnt;
    dn.root_code = c->root_code;
    const int D = (int)ht.down_level_off.size() - 1;
    for (int d = 0; d < D; ++d) {
        dn.order = dt.down_order + ht.down_level_off[d];
        dn.count = ht.down_level_off[d + 1] - ht.down_level_off[d];
        dim3 grid((dn.count + kWavesPerBlock - 1) / kWavesPerBlock, tiles);
        timer_begin(c, 1);
        hipLaunchKernelGGL(k_fitch_down, grid, dim3(kBlock), 0, c->stream, dn);
        timer_end(c, 1);
    }
    return hipGetLastError();
}

hipError_t launch_score(pm_ctx* c) {
    hipError_t e = hipMemsetAsync(c->score, 0, sizeof(int32_t) * c->num_sites, c->stream);
    if (e != hipSuccess) return e;
    const bool use_lds = c->num_sites * 4 <= 150 * 1024;
    const int spb = 4;
    const int blocks = kShards / spb;
    const size_t lds = use_lds ? (size_t)c->num_sites * 4 : 0;
    timer_begin(c, 2);
    hipLaunchKernelGGL(k_site_score, dim3(blocks), dim3(kBlock), lds, c->stream, c->recs, c->shard_cnt,
                       c->shard_cap, (uint32_t)c->ht.root, c->score, c->num_sites, spb, use_lds);
    timer_end(c, 2);
    return hipGetLastError();
}

}  // namespace pm
