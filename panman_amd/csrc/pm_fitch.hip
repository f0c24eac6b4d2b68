// pm_fitch.hip -- Fitch small parsimony over every alignment column at once (gfx950).
//
// Restates, for all sites together, the per-column recursion of the reference:
//   post-order  Tree::nucFitchForwardPass      src/fitchSankoff.cpp:30-56      -> k_fitch_up
//   pre-order   Tree::nucFitchBackwardPass     src/fitchSankoff.cpp:96-129     -> k_down<Mode::kFitch>
//   assignment  Tree::nucFitchAssignMutations  src/fitchSankoff.cpp:131-171    -> k_down<Mode::kFitch>
//   score       (edges with a change; the gather target of SURVEY.md §8e)        -> k_site_score
//
// Work decomposition: one wavefront = one tree node x one tile of 64 words (2048 sites);
// lane = one 32-site word.  The node (and therefore its child list) is wave-uniform, so
// child loads are scalar and there is no divergence; every lane streams 64 B (Fitch set)
// or 16 B (leaf / final codes) through fully coalesced 1 KiB wave-instructions.  Levels
// (heights for the post-order, depths for the pre-order) are separate launches.
// Integer bit-set work only: no MFMA (SURVEY.md §8d roofline is HBM bandwidth).
#include "pm_kernels.h"

#if PM_NT_LOADS   // (pm_fitch_nt.hip: the same passes, non-temporal set-record loads)
#define launch_fitch launch_fitch_nt
#define warm_fitch warm_fitch_nt
#endif

namespace pm {
namespace {

// One wave = (node, tile).  Children are folded straight into the AND / OR accumulators
// (src/fitchSankoff.cpp:39-55); the first two children's loads are independent and issued
// back to back.
// LEAFY: every child of the level's nodes is a leaf or a virtual leaf-parent (the lowest
// post-order level): no record loads, fewer registers, more waves per SIMD.
#ifndef PM_LEAFY_WAVES
#define PM_LEAFY_WAVES 6
#endif
#ifndef PM_SUB_LEAFY_WAVES
#define PM_SUB_LEAFY_WAVES 4
#endif
#ifndef PM_SUB_UP_WAVES
#define PM_SUB_UP_WAVES 4
#endif
// GROUP: 4 waves per SIMD, where the recomputation spills ~80 B/lane to scratch; 3 waves
// (~150 VGPRs, no scratch) cost C3 2 %.  A spilling build of this kernel once gave wrong sets
// at scale (DESIGN.md, S2 / S3 leaf packing): the at-scale parity tests guard every build.
#ifndef PM_GROUP_UP_WAVES
#define PM_GROUP_UP_WAVES 4
#endif
// SUB: subtree form -- the first two children may also be S2 / S3 subtrees (three or four
// leaves each, evaluated in registers: subtree_set_ap).
// GROUP: the descriptor's pad0 / pad1 (>= 0) name first / second children of this same
// launch, recomputed here (child_recompute) instead of loaded.
// gi: the node's index in the descriptor array (up slots, UpArgs::upm).
// PLAIN (subtree form, grouped order's plain prefix: pm_host.cpp make_groups): binary, neither
// child an S2 / S3 subtree -- the S-subtree code and the polytomy loop compiled out, the child
// sets branch-free (child_set_plain): 79 VGPRs
// instead of 117, so 6 waves per SIMD instead of 4.
template <bool AP, bool LEAFY, bool SUB = false, bool GROUP = false, bool PLAIN = false>
__device__ __forceinline__ void fitch_up_node(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int lane) {
    constexpr bool SS = SUB && !PLAIN;   // S2 / S3 children possible
    const int32_t n = d.node, e0 = d.e0, e1 = d.e1;
    const int64_t word = (int64_t)tile * kWave + lane;
    // subtree form: the children's masks from this node's up slots, its own into its parent's
    UpSlots sl{0, 0, 0, 0};
    if constexpr (SUB && !LEAFY) sl = load_up_slots(a, gi, tile);
    const int32_t ps = SUB ? a.pslot[gi] : -1;

    uint4 cw;   // consensus word for the store; loaded after the children's loads (see below)
    // vd0 / vd1: the first / second child's disagreeing-leaf sites (vd: every child's)
    uint32_t both[16], either[16], vd = 0, vd0 = 0, vd1 = 0;
    bool split = false;
    const int4 vl0 = make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), vl1 = make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]);
    if (GROUP && (d.pad0 >= 0 || d.pad1 >= 0)) {
        static_assert(!GROUP || (AP && !LEAFY), "grouped launches: all leaves present, non-leafy levels");
        fold_first_two<SUB, kUpGroupDepth, kFitchRec>(a, d, gi, tile, lane, word, both, either, vd);
        cw = a.cons[word];
    } else if constexpr (AP) {   // both children's loads in flight together
        ChildFetch f0, f1;
        constexpr bool SLOT = SUB && !LEAFY;
        fetch_child_ap<kFitchRec, LEAFY, SS, SLOT>(a, d.c0, vl0, tile, lane, word, f0, sl.x0, sl.s0);
        if (e1 - e0 > 1) fetch_child_ap<kFitchRec, LEAFY, SS, SLOT>(a, d.c1, vl1, tile, lane, word, f1, sl.x1, sl.s1);
        __builtin_amdgcn_sched_barrier(0);
        // after the children's consensus loads: loaded before them, the compiler reuses it
        // for them through register copies that wait on every outstanding load
        cw = a.cons[word];
        // the accumulators start as the first child's set (no all-ones / zero planes live
        // beside the loads in flight)
        if constexpr (PLAIN) child_set_plain<kCxCompact>(d.c0, vl0, f0, both, vd0);
        else child_set_ap<SS, kCxCompact>(d.c0, vl0, f0, both, vd0);
#pragma unroll
        for (int v = 0; v < 16; ++v) either[v] = both[v];
        if constexpr (PLAIN) {
            if (e1 - e0 > 1) {
                uint32_t y[16];
                child_set_plain<kCxCompact>(d.c1, vl1, f1, y, vd1);
#pragma unroll
                for (int v = 0; v < 16; ++v) { either[v] = both[v] | y[v]; both[v] &= y[v]; }
            }
        } else if (e1 - e0 > 1) {
            fold_child_ap<SS, kCxCompact>(d.c1, vl1, f1, both, either, vd1);
        }
        vd = vd0 | vd1;
        split = true;
    } else {
#pragma unroll
        for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
        fold_child<AP>(a, d.c0, vl0, tile, lane, word, both, either, vd);
        if (e1 - e0 > 1) fold_child<AP>(a, d.c1, vl1, tile, lane, word, both, either, vd);
        cw = a.cons[word];
    }
    for (int32_t e = e0 + 2; !PLAIN && e < e1; ++e) {   // polytomies
        const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        const int4 vl = c >= 0 && (c & kVirtualBit) ? a.vleaf[c & kDenseMask] : make_int4(-1, -1, -1, -1);
        if constexpr (LEAFY) {
            ChildFetch f;
            fetch_child_ap<kFitchRec, true>(a, c, vl, tile, lane, word, f);
            fold_child_ap<false, kCxCompact>(c, vl, f, both, either, vd);
        } else {
            fold_child<AP>(a, c, vl, tile, lane, word, both, either, vd);
        }
    }
    // AND if non-empty, else OR (src/fitchSankoff.cpp:48-55)
    const uint32_t nz = any_plane(both);
#pragma unroll
    for (int v = 0; v < 16; ++v) both[v] |= either[v] & ~nz;
    if (n == a.root_dense && a.forced != nullptr) {
        // refState replaces the root's set (src/fitchSankoff.cpp:45-47)
        const uint4 F = a.forced[word];
        onehot_from_code(F.x, F.y, F.z, F.w, ~0u, both);
    }
    // dirty lanes: complex, or a leaf-parent child's leaves disagree; every lane when some
    // leaf is absent somewhere (an empty leaf set can make a single code by the OR)
    uint64_t mx, ms, md;
    store_fitch_set(a.sets, a.cmask, cw, n, a.tiles, tile, lane, both, !AP || vd != 0u, mx, ms, md);
    push_up_slot(a, ps, tile, lane, mx, ms);
    // The first / second child's own dirty lanes (mask words 6 / 7 for the pre-order
    // descriptor's first / second child; an S2 / S3 child's pushed into its record): this node's complex lanes plus the lanes where that child's
    // leaves disagree.  Elsewhere every site's set is one code c, which all the child's
    // leaves hold, so its finals are c and it has no record (leaf_rule).  (The grouped
    // recomputation keeps one vd: both get the node's dirty lanes.)
    uint64_t md0 = md, md1 = md;
    if (AP && split) {
        md0 = mx | __ballot(vd0 != 0u);
        md1 = mx | __ballot(vd1 != 0u);
    }
    push_children2(a, tile, lane, e0, e1, d.c0, d.c1, mx, ms, md0, md1, n == a.root_dense);
    // (keyed by the pre-order descriptor's children, which omit S2 / S3 ones: pm_host.cpp)
    store_kid_masks(a.cmask, (size_t)n * a.tiles + tile, lane, sub_shaped(d.c0) ? md1 : md0, md1);
}

#ifndef PM_PLAIN_UP_WAVES
#define PM_PLAIN_UP_WAVES 6
#endif
template <bool AP, bool LEAFY, bool SUB = false, bool GROUP = false, bool PLAIN = false>
__global__ __launch_bounds__(kBlock, PLAIN ? PM_PLAIN_UP_WAVES : GROUP ? PM_GROUP_UP_WAVES : SUB ? (LEAFY ? PM_SUB_LEAFY_WAVES : PM_SUB_UP_WAVES) : LEAFY ? PM_LEAFY_WAVES : AP ? 5 : 1) void k_fitch_up(UpArgs a) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#ifdef PM_UP_LDS_PAD   // occupancy experiments only: caps the resident workgroups per CU
    __shared__ uint32_t occ_pad[PM_UP_LDS_PAD / 4];
    if (a.count < 0) {   // never taken; a read keeps the array (and its LDS allocation)
        occ_pad[threadIdx.x] = threadIdx.x;
        __syncthreads();
        a.cmask[threadIdx.x] = occ_pad[(threadIdx.x * 7) % (PM_UP_LDS_PAD / 4)];
    }
#endif
    int32_t item;
    int tile;
    wave_item(wave, a.tiles, item, tile);
    if (item >= a.count) return;
    fitch_up_node<AP, LEAFY, SUB, GROUP, PLAIN>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, lane);
}

// Wide nodes (out-degree > 3): one workgroup per (node, tile), the children dealt
// round-robin to its 4 waves.  Each wave loads 64 child encodings (and virtual children's
// leaves) with one vector load, then fetches two children before folding either, so the
// chain of dependent loads per node shrinks ~8x; the waves' (both, either) accumulators
// are combined through LDS (AND / OR are associative: src/fitchSankoff.cpp:39-55).
struct UpFetch {
    uint32_t w[16];
    bool complex_lane;
    const uint4* p;   // compact records: A in w[0..3], B in w[5..8]; p / mx for cx_decode
    uint64_t mx;
};

template <bool AP>
__device__ __forceinline__ void up_fetch(const UpArgs& a, int32_t c, int4 vl, int tile, int lane, int64_t word,
                                         UpFetch& f) {
    f.complex_lane = false;
    if (c < 0) {
        uint4 L;
        leaf_word<AP>(a, -c - 1, word, L, f.w[4]);
        f.w[0] = L.x; f.w[1] = L.y; f.w[2] = L.z; f.w[3] = L.w;
    } else if (c & kVirtualBit) {
        uint4 L0, L1 = make_uint4(0, 0, 0, 0);
        f.w[9] = 0;
        leaf_word<AP>(a, vl.x, word, L0, f.w[4]);
        if (vl.y >= 0) leaf_word<AP>(a, vl.y, word, L1, f.w[9]);
        f.w[0] = L0.x; f.w[1] = L0.y; f.w[2] = L0.z; f.w[3] = L0.w;
        f.w[5] = L1.x; f.w[6] = L1.y; f.w[7] = L1.z; f.w[8] = L1.w;
    } else {
        const size_t rec = (size_t)c * a.tiles + tile;
        const RecMask mk = rec_mask(a.cmask, rec);
        const uint4* p = a.sets + rec * kFitchRec;
        f.complex_lane = (mk.x >> lane) & 1ull;
        if constexpr (kCxCompact) {
            const uint4 A = rec_code_all<true>(p, mk, lane, a.cons, word), B = cx_b_load(p, mk, lane, a.cons);
            f.w[0] = A.x; f.w[1] = A.y; f.w[2] = A.z; f.w[3] = A.w;
            f.w[5] = B.x; f.w[6] = B.y; f.w[7] = B.z; f.w[8] = B.w;
            f.p = p;
            f.mx = mk.x;
        } else if (f.complex_lane) {
            const uint32_t k = lanes_below(mk.x);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 w = load_rec(p + kWave + q * kWave + k);
                f.w[4 * q] = w.x; f.w[4 * q + 1] = w.y; f.w[4 * q + 2] = w.z; f.w[4 * q + 3] = w.w;
            }
        } else {
            const uint4 w = rec_code(p, mk, lane, a.cons, word);
            f.w[0] = w.x; f.w[1] = w.y; f.w[2] = w.z; f.w[3] = w.w;
        }
    }
}

__device__ __forceinline__ void up_fold(int32_t c, const UpFetch& f, uint32_t* both, uint32_t* either, uint32_t& vd) {
    uint32_t x[16];
    if (kCxCompact && c >= 0 && !(c & kVirtualBit)) {
        onehot_from_code(f.w[0], f.w[1], f.w[2], f.w[3], ~0u, x);
        cx_decode(x, make_uint4(f.w[0], f.w[1], f.w[2], f.w[3]), make_uint4(f.w[5], f.w[6], f.w[7], f.w[8]), f.complex_lane,
                  f.p, f.mx);
    } else if (c >= 0 && !(c & kVirtualBit) && f.complex_lane) {
#pragma unroll
        for (int v = 0; v < 16; ++v) x[v] = f.w[v];
    } else {
        const bool leafish = c < 0 || (c & kVirtualBit);
        const LoHi t = lohi_of(f.w[0], f.w[1], f.w[2], f.w[3], leafish ? f.w[4] : ~0u);
#pragma unroll
        for (int v = 0; v < 16; ++v) x[v] = t.lo[v & 3] & t.hi[v >> 2];
        if (c >= 0 && (c & kVirtualBit)) {
            vd |= f.w[9] & ((f.w[0] ^ f.w[5]) | (f.w[1] ^ f.w[6]) | (f.w[2] ^ f.w[7]) | (f.w[3] ^ f.w[8]));
            const LoHi u = lohi_of(f.w[5], f.w[6], f.w[7], f.w[8], f.w[9]);
#pragma unroll
            for (int v = 0; v < 16; ++v) x[v] |= u.lo[v & 3] & u.hi[v >> 2];
        }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        both[v] &= x[v];
        either[v] |= x[v];
    }
}

// One wave's share of a wide node's children: children e0 + wave, e0 + wave + NW, ... folded
// into (both, either, vd).
template <bool AP, int NW>
__device__ __forceinline__ void wide_fold(const UpArgs& a, int32_t e0, int32_t e1, int wave, int tile, int lane,
                                          int64_t word, uint32_t* both, uint32_t* either, uint32_t& vd) {
#pragma unroll
    for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
    vd = 0;
    for (int32_t base = e0 + wave; base < e1; base += NW * kWave) {
        const int32_t my = base + NW * lane;
        const int32_t enc = my < e1 ? a.child_enc[my] : 0;
        const int4 vl = my < e1 && enc >= 0 && (enc & kVirtualBit) ? a.vleaf[enc & kDenseMask]
                                                                   : make_int4(-1, -1, -1, -1);
        const int cnt = min(kWave, (e1 - base + NW - 1) / NW);
        // AP: every record child's (x, s) masks, one child per lane, loaded once for the whole
        // batch -- a pair's record loads then wait on nothing but themselves
        uint64_t cmx = 0, cms = 0;
        if (AP && my < e1 && materialised(enc)) {
            const uint64_t* q = a.cmask + kMaskWords * ((size_t)enc * a.tiles + tile);
            cmx = q[0];
            cms = q[1];
        }
        for (int k = 0; k < cnt; k += 2) {
            const int32_t c0 = __builtin_amdgcn_readlane(enc, k);
            const int4 v0 = make_int4(__builtin_amdgcn_readlane(vl.x, k), __builtin_amdgcn_readlane(vl.y, k), -1, -1);
            const bool two = k + 1 < cnt;
            const int32_t c1 = two ? __builtin_amdgcn_readlane(enc, k + 1) : 0;
            const int4 v1 = two ? make_int4(__builtin_amdgcn_readlane(vl.x, k + 1), __builtin_amdgcn_readlane(vl.y, k + 1), -1, -1)
                                : make_int4(-1, -1, -1, -1);
            if constexpr (AP) {   // both children's loads in flight together (see k_fitch_up)
                ChildFetch f0, f1;
                fetch_child_ap_m(a, c0, v0, readlane64(cmx, k), readlane64(cms, k), tile, lane, word, f0);
                if (two) fetch_child_ap_m(a, c1, v1, readlane64(cmx, k + 1), readlane64(cms, k + 1), tile, lane, word, f1);
                __builtin_amdgcn_sched_barrier(0);
                fold_child_ap<false, kCxCompact>(c0, v0, f0, both, either, vd);
                if (two) fold_child_ap<false, kCxCompact>(c1, v1, f1, both, either, vd);
            } else {
                UpFetch f0, f1;
                up_fetch<AP>(a, c0, v0, tile, lane, word, f0);
                if (two) up_fetch<AP>(a, c1, v1, tile, lane, word, f1);
                up_fold(c0, f0, both, either, vd);
                if (two) up_fold(c1, f1, both, either, vd);
            }
        }
    }
}

// AND if non-empty else OR, forced root, store and mask pushes of a wide node (one wave).
template <bool AP>
__device__ __forceinline__ void wide_finish(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int lane,
                                            int64_t word, uint32_t* both, const uint32_t* either, uint32_t vd) {
    const uint32_t nz = any_plane(both);
#pragma unroll
    for (int v = 0; v < 16; ++v) both[v] |= either[v] & ~nz;
    if (d.node == a.root_dense && a.forced != nullptr) {
        const uint4 F = a.forced[word];
        onehot_from_code(F.x, F.y, F.z, F.w, ~0u, both);
    }
    uint64_t mx, ms, md;
    store_fitch_set(a.sets, a.cmask, a.cons[word], d.node, a.tiles, tile, lane, both, !AP || vd != 0u, mx, ms, md);
    if (a.upm != nullptr) push_up_slot(a, a.pslot[gi], tile, lane, mx, ms);   // (subtree form)
    push_children(a, tile, lane, d.e0, d.e1, d.c0, d.c1, mx, ms);
    store_kid_masks(a.cmask, (size_t)d.node * a.tiles + tile, lane, md, md);
}

// One workgroup = one wide node x tile.
template <bool AP>
__device__ __forceinline__ void wide_node(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int wave, int lane,
                                          uint32_t (*part)[33][kWave]) {
    const int64_t word = (int64_t)tile * kWave + lane;
    uint32_t both[16], either[16], vd;
    wide_fold<AP, kWavesPerBlock>(a, d.e0, d.e1, wave, tile, lane, word, both, either, vd);
    if (wave > 0) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            part[wave - 1][v][lane] = both[v];
            part[wave - 1][16 + v][lane] = either[v];
        }
        part[wave - 1][32][lane] = vd;
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock - 1; ++w) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            both[v] &= part[w][v][lane];
            either[v] |= part[w][16 + v][lane];
        }
        vd |= part[w][32][lane];
    }
    wide_finish<AP>(a, d, gi, tile, lane, word, both, either, vd);
}

template <bool AP>
__global__ __launch_bounds__(kBlock) void k_fitch_up_wide(UpArgs a) {
    __shared__ uint32_t part[kWavesPerBlock - 1][33][kWave];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    block_item(a.tiles, item, tile);
    wide_node<AP>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, wave, lane, part);
}

// A level holding nodes of both kinds (polytomies, deep trees) in ONE launch instead of two
// dependent ones: blocks [0, narrow_blocks) are k_fitch_up's (a wave per (node, tile) over
// a.desc), the rest k_fitch_up_wide's (a workgroup per (wide node, tile) over wdesc).
static_assert(PM_TILE_FAST, "k_fitch_up_mixed numbers its blocks on one grid axis");
template <bool AP, bool SUB, bool GROUP = false>
__global__ __launch_bounds__(kBlock) void k_fitch_up_mixed(UpArgs a, const NodeDesc* wdesc, int32_t narrow_blocks) {
    __shared__ uint32_t part[kWavesPerBlock - 1][33][kWave];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if ((int32_t)blockIdx.x < narrow_blocks) {
        int32_t item;
        int tile;
        wave_item(wave, a.tiles, item, tile);
        if (item < a.count) fitch_up_node<AP, false, SUB, GROUP>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, lane);
        return;
    }
    const int32_t b = (int32_t)blockIdx.x - narrow_blocks;
    const int32_t item = b / a.tiles;
    wide_node<AP>(a, wdesc[item], (int32_t)(wdesc - a.desc_all) + item, b - item * a.tiles, wave, lane, part);
}

// Narrow levels (PM_OPT_NARROW): a run of consecutive post-order levels with few nodes each
// is walked by ONE launch -- one 1024-thread workgroup per tile, each level's nodes dealt to
// its 16 waves (a wide node's children to all of them, accumulators met by LDS AND / OR
// atomics), a workgroup barrier between levels -- instead of one launch per level, each a
// dependent chain of HBM round trips behind a kernel boundary (deep, ladder-like trees).  A
// tile's records and masks are only touched by the waves of its own workgroup, so the
// barrier's workgroup-scope release / acquire is all the synchronisation the hand-off needs;
// what earlier launches wrote is visible at kernel start.
template <bool AP, bool SUB, bool GROUP = false>
__global__ __launch_bounds__(kBandBlock) void k_fitch_up_band(UpArgs a, const int32_t* class_off, int32_t h0, int32_t h1) {
    __shared__ uint32_t acc[33][kWave];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int tile = blockIdx.x;
    const int64_t word = (int64_t)tile * kWave + lane;
    for (int32_t h = h0; h < h1; ++h) {
        const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1],
                      e = class_off[(h + 1) * kDegreeClasses];
        for (int32_t i = b + wave; i < m; i += kBandWaves) fitch_up_node<AP, false, SUB, GROUP>(a, a.desc[i], i, tile, lane);
        for (int32_t i = m; i < e; ++i) {   // out-degree > 3
            if (wave == 0) {
#pragma unroll
                for (int v = 0; v < 16; ++v) { acc[v][lane] = ~0u; acc[16 + v][lane] = 0u; }
                acc[32][lane] = 0u;
            }
            __syncthreads();
            const NodeDesc& d = a.desc[i];
            uint32_t both[16], either[16], vd;
            wide_fold<AP, kBandWaves>(a, d.e0, d.e1, wave, tile, lane, word, both, either, vd);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                atomicAnd(&acc[v][lane], both[v]);
                atomicOr(&acc[16 + v][lane], either[v]);
            }
            atomicOr(&acc[32][lane], vd);
            __syncthreads();
            if (wave == 0) {
#pragma unroll
                for (int v = 0; v < 16; ++v) { both[v] = acc[v][lane]; either[v] = acc[16 + v][lane]; }
                wide_finish<AP>(a, d, i, tile, lane, word, both, either, acc[32][lane]);
            }
        }
        __syncthreads();
    }
}

// ---- LDS-staged post-order sweeps (PM_OPT_CLUSTER; schedule: pm_cluster.cpp) --------------
// One wave = one (cluster, tile): the cluster's nodes in depth-first post-order, one per step.
// A child of the same cluster comes from its LDS slot (16 planes, 4 KiB per (node, tile));
// every other child as in fitch_up_node (leaf words, a leaf-parent's or S2 / S3 subtree's
// leaves, or an earlier launch's compressed record).  Records and masks go to HBM exactly as
// the level kernels write them (the pre-order pass and the tail read them), without a wait.
// AND if non-empty else OR, forced root, the record + masks to HBM (as fitch_up_node / wide_finish
// write them), the (x, s) masks into the parent's up slot when the parent is in a later band
// (ps = ClArgs::pslot[item]), the set into the node's LDS slot when it is in this cluster.
__device__ __forceinline__ void cluster_finish(const UpArgs& a, const NodeDesc& d, int32_t ps, ClSlots& S, int tile,
                                               int lane, int64_t word, const uint4& cw, uint32_t* both,
                                               const uint32_t* either, uint32_t vd, uint32_t vd0, uint32_t vd1, bool split) {
    const int32_t n = d.node;
    const uint32_t nz = any_plane(both);
#pragma unroll
    for (int v = 0; v < 16; ++v) both[v] |= either[v] & ~nz;
    if (n == a.root_dense && a.forced != nullptr) {   // refState (src/fitchSankoff.cpp:45-47)
        const uint4 F = a.forced[word];
        onehot_from_code(F.x, F.y, F.z, F.w, ~0u, both);
    }
#ifdef PM_CL_NO_OUTPUT   // (timing-only variant: the chain's LDS work alone)
    if (d.parent >= 0) slot_write(S, d.parent, lane, both);
    return;
#endif
    uint64_t mx, ms, md;
    store_fitch_set(a.sets, a.cmask, cw, n, a.tiles, tile, lane, both, vd != 0u, mx, ms, md);
    push_up_slot(a, ps, tile, lane, mx, ms);   // (a parent in a later band)
    uint64_t md0 = md, md1 = md;
    if (split) {
        md0 = mx | __ballot(vd0 != 0u);
        md1 = mx | __ballot(vd1 != 0u);
    }
    push_children2(a, tile, lane, d.e0, d.e1, d.c0, d.c1, mx, ms, md0, md1, n == a.root_dense);
    store_kid_masks(a.cmask, (size_t)n * a.tiles + tile, lane, sub_shaped(d.c0) ? md1 : md0, md1);
    if (d.parent >= 0) slot_write(S, d.parent, lane, both);
}

// A narrow item's first two children that are not in the cluster, from memory in two parts:
// the first load of each (a leaf's word; a leaf-parent's or S2 / S3 subtree's first two leaves;
// an earlier launch's record code word, addressed through the item's up slot) issued one round
// ahead of the item's round, so a round waits on LDS only for the common children; the rest (an
// S2 / S3 subtree's third and fourth leaves, a record's complex lanes) in the round itself.
struct ClFetch {
    uint4 c0, x0, c1, x1;
};

__device__ __forceinline__ void cl_fetch1(const UpArgs& a, int32_t ch, int4 vl, uint64_t mx, uint64_t ms, int tile, int lane,
                                          int64_t word, uint4& cd, uint4& x) {
    if (ch < 0) {
        cd = a.leaf_planes[(size_t)(-ch - 1) * a.wpad + word];
    } else if (ch & kVirtualBit) {
        const int32_t l0 = __builtin_amdgcn_readfirstlane(vl.x), l1 = __builtin_amdgcn_readfirstlane(vl.y);
        cd = a.leaf_planes[(size_t)l0 * a.wpad + word];
        if (l1 >= 0) x = a.leaf_planes[(size_t)l1 * a.wpad + word];
    } else {
        const size_t rec = (size_t)ch * a.tiles + tile;
        const RecMask m{mx, ms, 0, 0, 0};
        cd = rec_code_all<kCxCompact>(a.sets + rec * kFitchRec, m, lane, a.cons, word);
        if constexpr (kCxCompact) x = cx_b_load(a.sets + rec * kFitchRec, m, lane, a.cons);
    }
}

// The child's 16-plane set from its first load (cd, x) and the rest; vd as child_set_ap's.
__device__ __forceinline__ void cl_set1(const UpArgs& a, int32_t ch, int4 vl, uint64_t mx, const uint4& cd, const uint4& x,
                                        int tile, int lane, int64_t word, uint32_t* out, uint32_t& vd) {
    const LoHi t = lohi_of(cd.x, cd.y, cd.z, cd.w, ~0u);
#pragma unroll
    for (int v = 0; v < 16; ++v) out[v] = t.lo[v & 3] & t.hi[v >> 2];
    if (ch >= 0 && (ch & kVirtualBit)) {
        const int shape = (ch >> kShapeShift) & 3;
        if (shape) {   // S2 / S3 (subtree_set_ap): leaves a, b (prefetched), c, d
            ChildFetch f;
            f.code = cd;
            f.v[0] = x;
            const int32_t l2 = __builtin_amdgcn_readfirstlane(vl.z), l3 = __builtin_amdgcn_readfirstlane(vl.w);
            f.v[1] = a.leaf_planes[(size_t)l2 * a.wpad + word];
            if (l3 >= 0) f.v[2] = a.leaf_planes[(size_t)l3 * a.wpad + word];
            subtree_set_ap(shape, f, out, vd);
        } else if (__builtin_amdgcn_readfirstlane(vl.y) >= 0) {   // two leaves: their union
            vd |= code_ne(cd, x);
            const LoHi u = lohi_of(x.x, x.y, x.z, x.w, ~0u);
#pragma unroll
            for (int v = 0; v < 16; ++v) out[v] |= u.lo[v & 3] & u.hi[v >> 2];
        }
    } else if (kCxCompact && ch >= 0) {   // a record (x: its B word)
        cx_decode(out, cd, x, (mx >> lane) & 1ull, a.sets + ((size_t)ch * a.tiles + tile) * kFitchRec, mx);
    } else if (ch >= 0 && mx != 0 && ((mx >> lane) & 1ull)) {   // a record's complex lane
        const uint4* p = a.sets + ((size_t)ch * a.tiles + tile) * kFitchRec + kWave + lanes_below(mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 w = load_rec(p + q * kWave);
            out[4 * q] = w.x; out[4 * q + 1] = w.y; out[4 * q + 2] = w.z; out[4 * q + 3] = w.w;
        }
    }
}

__device__ __forceinline__ void cluster_issue(const UpArgs& a, const NodeDesc& d, const UpSlots& sl, int tile, int lane,
                                              int64_t word, ClFetch& p) {
    if (d.node < 0 || d.e1 - d.e0 > 3) return;
    const int4 vl0 = make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), vl1 = make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]);
    if (d.pad0 < 0) cl_fetch1(a, d.c0, vl0, sl.x0, sl.s0, tile, lane, word, p.c0, p.x0);
    if (d.e1 - d.e0 > 1 && d.pad1 < 0) cl_fetch1(a, d.c1, vl1, sl.x1, sl.s1, tile, lane, word, p.c1, p.x1);
}

// A node of out-degree <= 3 (one wave); its out-of-cluster first two children's first loads in `p`.
__device__ __forceinline__ void cluster_node(const UpArgs& a, const ClArgs& c, const NodeDesc& d, const UpSlots& sl, int32_t ps,
                                             const ClFetch& p, ClSlots& S, int tile, int lane, int64_t word, const uint4& cw) {
    const bool two = d.e1 - d.e0 > 1;
    const int4 vl0 = make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), vl1 = make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]);
    uint32_t both[16], either[16], vd0 = 0, vd1 = 0;
    if (d.pad0 >= 0) slot_read(S, d.pad0, lane, both);
    else cl_set1(a, d.c0, vl0, sl.x0, p.c0, p.x0, tile, lane, word, both, vd0);
#pragma unroll
    for (int v = 0; v < 16; ++v) either[v] = both[v];
    if (two) {
        uint32_t y[16];
        if (d.pad1 >= 0) slot_read(S, d.pad1, lane, y);
        else cl_set1(a, d.c1, vl1, sl.x1, p.c1, p.x1, tile, lane, word, y, vd1);
#pragma unroll
        for (int v = 0; v < 16; ++v) { either[v] |= y[v]; both[v] &= y[v]; }
    }
    uint32_t vd = vd0 | vd1;
    for (int32_t e = d.e0 + 2; e < d.e1; ++e) {   // an out-degree-3 node's third child
        const int32_t ch = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        const int32_t s = materialised(ch) ? __builtin_amdgcn_readfirstlane(c.slot_of[ch]) : -1;
        if (s >= 0) {
            uint32_t y[16];
            slot_read(S, s, lane, y);
#pragma unroll
            for (int v = 0; v < 16; ++v) { either[v] |= y[v]; both[v] &= y[v]; }
        } else {
            const int4 vl = ch >= 0 && (ch & kVirtualBit) ? a.vleaf[ch & kDenseMask] : make_int4(-1, -1, -1, -1);
            fold_child<true>(a, ch, vl, tile, lane, word, both, either, vd);
        }
    }
    cluster_finish(a, d, ps, S, tile, lane, word, cw, both, either, vd, vd0, vd1, true);
}

// A node of out-degree > 3.  Such nodes' children are mostly leaves (T2: 96 %): eight leaf
// words are loaded at a time before any is folded; other children (a leaf-parent's leaves, an
// LDS slot, a record) one at a time.
constexpr int kClWideBatch = 8;
__device__ __forceinline__ void cluster_wide(const UpArgs& a, const ClArgs& c, const NodeDesc& d, int32_t ps, ClSlots& S,
                                             int tile, int lane, int64_t word, const uint4& cw) {
    uint32_t both[16], either[16], vd = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
    for (int32_t base = d.e0; base < d.e1; base += kWave) {
        const int32_t my = base + lane;
        const int32_t enc = my < d.e1 ? a.child_enc[my] : 0;
        const int cnt = min(kWave, d.e1 - base);
        for (int k = 0; k < cnt; k += kClWideBatch) {
            uint4 L[kClWideBatch];
#pragma unroll
            for (int j = 0; j < kClWideBatch; ++j) {
                const int32_t ch = k + j < cnt ? __builtin_amdgcn_readlane(enc, k + j) : 0;
                if (k + j < cnt && ch < 0) L[j] = a.leaf_planes[(size_t)(-ch - 1) * a.wpad + word];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < kClWideBatch; ++j) {
                if (k + j >= cnt) break;
                const int32_t ch = __builtin_amdgcn_readlane(enc, k + j);
                if (ch < 0) {   // a leaf (src/fitchSankoff.cpp:32-38)
                    const LoHi t = lohi_of(L[j].x, L[j].y, L[j].z, L[j].w, ~0u);
#pragma unroll
                    for (int v = 0; v < 16; ++v) {
                        const uint32_t x = t.lo[v & 3] & t.hi[v >> 2];
                        both[v] &= x;
                        either[v] |= x;
                    }
                    continue;
                }
                const int32_t sl = materialised(ch) ? __builtin_amdgcn_readfirstlane(c.slot_of[ch]) : -1;
                if (sl >= 0) {
                    uint32_t y[16];
                    slot_read(S, sl, lane, y);
#pragma unroll
                    for (int v = 0; v < 16; ++v) { either[v] |= y[v]; both[v] &= y[v]; }
                } else {
                    const int4 vl = (ch & kVirtualBit) ? a.vleaf[ch & kDenseMask] : make_int4(-1, -1, -1, -1);
                    fold_child<true>(a, ch, vl, tile, lane, word, both, either, vd);
                }
            }
        }
    }
    cluster_finish(a, d, ps, S, tile, lane, word, cw, both, either, vd, 0, 0, false);
}

__device__ __forceinline__ void cluster_step(const UpArgs& a, const ClArgs& c, const ClMeta& m, const ClFetch& p, ClSlots& S,
                                             int tile, int lane, int64_t word, const uint4& cw) {
    if (m.d.e1 - m.d.e0 > 3) cluster_wide(a, c, m.d, m.ps, S, tile, lane, word, cw);
    else cluster_node(a, c, m.d, m.s, m.ps, p, S, tile, lane, word, cw);
}

#ifndef PM_CL_WAVES   // waves per SIMD (occupancy bound of the sweep kernel)
#define PM_CL_WAVES 3
#endif
__global__ __launch_bounds__(kWave, PM_CL_WAVES) void k_fitch_up_cluster(UpArgs a, ClArgs c) {
    __shared__ ClSlots S;
    const int lane = threadIdx.x;
    const int32_t b = (int32_t)blockIdx.x;
    const int32_t wl = b / a.tiles;
    const int tile = b - wl * a.tiles;
    const int32_t i0 = c.wg_off[c.wg0 + wl], steps = c.wg_off[c.wg0 + wl + 1] - i0;
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint4 cw = a.cons[word];
    // Software pipeline over steps: step r's children loads are issued at the start of step
    // r - 1 (two fetch buffers whose roles alternate: a register copy of a load's destination
    // would wait for the load), its descriptor one step before that.
    ClMeta M0, M1;
    ClFetch fA, fB;
    cl_meta_get(cl_meta_load(a, c, i0, tile, lane), M0);
    cluster_issue(a, M0.d, M0.s, tile, lane, word, fA);
    uint32_t m1 = steps > 1 ? cl_meta_load(a, c, i0 + 1, tile, lane) : 0u;
    for (int32_t r = 0; r < steps; r += 2) {
        // step r (M0, fA); step r + 1's loads into fB; step r + 2's descriptor
        const uint32_t m2 = r + 2 < steps ? cl_meta_load(a, c, i0 + r + 2, tile, lane) : 0u;
        if (r + 1 < steps) {
            cl_meta_get(m1, M1);
            cluster_issue(a, M1.d, M1.s, tile, lane, word, fB);
        }
        cluster_step(a, c, M0, fA, S, tile, lane, word, cw);
        if (r + 1 >= steps) break;
        // step r + 1 (M1, fB); step r + 2's loads into fA; step r + 3's descriptor
        m1 = r + 3 < steps ? cl_meta_load(a, c, i0 + r + 3, tile, lane) : 0u;
        if (r + 2 < steps) {
            cl_meta_get(m2, M0);
            cluster_issue(a, M0.d, M0.s, tile, lane, word, fA);
        }
        cluster_step(a, c, M1, fB, S, tile, lane, word, cw);
    }
}


#if !PM_NT_LOADS   // (the score kernel: once, in pm_fitch.hip)
// Per-site score = mutated edges below the root.  Records of a shard are histogrammed in
// LDS (sites fit) or straight into global counters.  1024-thread workgroups: the LDS
// histogram (4 B per site) admits one workgroup per CU, so the workgroup brings the waves.
constexpr int kScoreBlock = 1024;

__global__ __launch_bounds__(kScoreBlock) void k_site_score(const pm_mut* recs, const uint32_t* shard_cnt,
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
        constexpr int U = 4;   // records in flight per thread
        for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)U * blockDim.x) {
            pm_mut m[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + (int64_t)u * blockDim.x;
                if (i < n) {   // (read once: non-temporal, N* step -0.09 ms)
                    const uint64_t w = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(r + i));
                    m[u] = pm_mut{(uint32_t)w, (uint32_t)(w >> 32)};
                } else {
                    m[u] = pm_mut{root_id, 0};
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (m[u].node == root_id) continue;
                const uint32_t site = m[u].site_info >> 8;
                if (use_lds) atomicAdd(&hist[site], 1u);
                else atomicAdd(&score[site], 1);
            }
        }
    }
    if (use_lds) {
        __syncthreads();
        for (int64_t s = threadIdx.x; s < sites; s += blockDim.x)
            if (hist[s]) atomicAdd(&score[s], (int32_t)hist[s]);
    }
}

#endif

}  // namespace

hipError_t launch_fitch(pm_ctx* c, bool block) {
    const HostTree& ht = c->ht;
    const DevTree& dt = c->dt;
    const int32_t tiles = (c->words + kWave - 1) / kWave;
    const int64_t wpad = (int64_t)tiles * kWave;

    // Fitch (not block Fitch) may skip materialising leaf-parents and, with every leaf
    // present, S2 / S3 subtrees (the subtree form)
    const bool virt = !block && c->virtual_leaf_parents;
    const bool sub = virt && c->subtree_form && c->leaves_all_present && ht.num_sshape > 0;
    const int32_t* child_enc = sub ? dt.child_enc_k : virt ? dt.child_enc_v : dt.child_enc;
    // subtree form: LDS-staged sweeps above the plan's first level (PM_OPT_CLUSTER), the levels
    // below them one launch per height; else grouped post-order launches (PM_OPT_UP_GROUP) or one
    // launch per height
    // (with a sweep plan the grouped order stops below the sweeps: without them, one launch per
    // height)
    const ClusterPlan& cl = ht.cl;
    const bool planned = cl.band_wg.size() > 1;
    const bool clu = sub && c->cluster && planned;
    const bool grp = sub && c->up_group && (clu || !planned);
    const NodeDesc* up_desc = grp ? dt.up_desc_g : sub ? dt.up_desc_k : virt ? dt.up_desc_v : dt.up_desc;
    // PM_OPT_SUB_DOWN: S2 / S3 children stay in their parent's pre-order descriptor (k_down<..,
    // SUB>) and leave the tail
    const bool sub_down = sub && c->sub_down;
    const NodeDesc* down_desc = sub_down ? dt.down_desc_ks : sub ? dt.down_desc_k : virt ? dt.down_desc_v : dt.down_desc;
    const std::vector<int32_t>& up_off = grp ? ht.up_level_off_g : sub ? ht.up_level_off_k : virt ? ht.up_level_off_v : ht.up_level_off;
    const std::vector<int32_t>& down_off = sub ? ht.down_level_off_k : virt ? ht.down_level_off_v : ht.down_level_off;

    const bool ap = c->leaves_all_present;
    UpArgs up{};
    up.child_off = dt.child_off;
    up.child_enc = child_enc;
    up.leaf_flag = c->leaf_flag;
    up.leaf_planes = c->leaf_planes;
    up.leaf_present = c->leaf_present;
    up.sets = reinterpret_cast<uint4*>(c->sets);
    up.cmask = c->cmask;
    up.vleaf = reinterpret_cast<const int4*>(dt.vleaf);
    up.cons = c->cons;
    up.forced = (c->has_forced && !block) ? c->forced : nullptr;   // refState (M1); blocks force in backward
    up.absent_code0 = false;
    up.all_present = c->leaves_all_present;
    up.root_dense = dt.root_dense;
    up.tiles = tiles;
    up.wpad = wpad;
    const std::vector<int32_t>& class_off = grp ? ht.up_class_off_g : sub ? ht.up_class_off_k : virt ? ht.up_class_off_v : ht.up_class_off;
    const int form = sub ? 2 : virt ? 1 : 0;   // pre-order level tables (lvl_down)
    const int up_form = grp ? 3 : form;        // post-order ones (lvl_up)
    up.desc_all = up_desc;
    // up slots: the subtree form's kernels (alloc_work sizes them for its two up orders)
    if (sub && c->upm == nullptr) return hipErrorInvalidValue;
    up.upm = sub ? c->upm : nullptr;
    up.pslot = grp ? (clu ? dt.pslot_gc : dt.pslot_g) : clu ? dt.pslot_kc : dt.pslot_k;
    const int H = clu && !grp ? cl.h0 : (int)up_off.size() - 1;   // (the grouped order holds the levels below h0 only)
    // runs of >= 2 narrow levels (PM_OPT_NARROW): one band launch each
    auto narrow_up = [&](int h) {
        const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1],
                      e = class_off[(h + 1) * kDegreeClasses];
        return (m - b) + 4 * (e - m) <= c->narrow_max;
    };
    for (int h = 0; h < H; ++h) {
        if (c->narrow_max > 0 && narrow_up(h)) {
            int h1 = h + 1;
            while (h1 < H && narrow_up(h1)) ++h1;
            if (h1 - h >= 2) {
                up.desc = up_desc;
                const int32_t* tab = dt.lvl + ht.lvl_up[up_form];
                timer_begin(c, 0);
                if (grp) hipLaunchKernelGGL((k_fitch_up_band<true, true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else if (sub) hipLaunchKernelGGL((k_fitch_up_band<true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else if (ap) hipLaunchKernelGGL((k_fitch_up_band<true, false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else hipLaunchKernelGGL((k_fitch_up_band<false, false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                timer_end(c, 0);
                h = h1 - 1;
                continue;
            }
        }
        // out-degree <= 3: one wave per (node, tile); wider: one workgroup per (node, tile)
        const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1],
                      e = class_off[(h + 1) * kDegreeClasses];
        if (m > b && e > m && (int64_t)(m - b) * tiles <= kMixedMaxWaves) {   // both kinds: one launch
            up.desc = up_desc + b;
            up.count = m - b;
            const int32_t nb = (int32_t)wave_grid(up.count, tiles).x;
            const dim3 grid((unsigned)(nb + (int64_t)(e - m) * tiles));
            timer_begin(c, 0);
            if (grp) hipLaunchKernelGGL((k_fitch_up_mixed<true, true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
            else if (sub) hipLaunchKernelGGL((k_fitch_up_mixed<true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
            else if (ap) hipLaunchKernelGGL((k_fitch_up_mixed<true, false>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
            else hipLaunchKernelGGL((k_fitch_up_mixed<false, false>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
            timer_end(c, 0);
            continue;
        }
        // a level's narrow and wide nodes are independent: the wide launch runs beside the
        // narrow one on the side stream (parallel graph branches) instead of after it
#ifdef PM_NO_SIDE
        const bool fork = false;
#else
        const bool fork = m > b && e > m;
#endif
        if (fork) {
            const hipError_t fe = side_fork(c);
            if (fe != hipSuccess) return fe;
        }
        if (e > m) {
            UpArgs w = up;
            w.desc = up_desc + m;
            w.count = e - m;
            const dim3 grid = block_grid(w.count, tiles);
            hipStream_t s = fork ? c->side : c->stream;
            if (!fork) timer_begin(c, 0);
            if (ap) hipLaunchKernelGGL(k_fitch_up_wide<true>, grid, dim3(kBlock), 0, s, w);
            else hipLaunchKernelGGL(k_fitch_up_wide<false>, grid, dim3(kBlock), 0, s, w);
            if (!fork) timer_end(c, 0);
        }
        if (m > b) {
            const bool leafy = grp ? ht.up_leafy_g[h] : sub ? ht.up_leafy_k[h] : virt && ht.up_leafy_v[h];
            // the grouped order's plain prefix (binary, no S2 / S3 child, nothing recomputed):
            // the lean kernel, then the rest of the class
            int32_t np = grp && !leafy && c->plain_up ? std::min(ht.up_plain_g[h], m - b) : 0;
            if ((int64_t)np * tiles < (c->plain_min_waves > 0 ? c->plain_min_waves : kPlainMinWaves)) np = 0;
            timer_begin(c, 0);
            if (np > 0) {
                up.desc = up_desc + b;
                up.count = np;
                hipLaunchKernelGGL((k_fitch_up<true, false, true, false, true>), wave_grid(np, tiles), dim3(kBlock), 0, c->stream, up);
            }
            up.desc = up_desc + b + np;
            up.count = m - b - np;
            const dim3 grid = wave_grid(up.count, tiles);
            if (up.count == 0) {
                if (fork) {
                    const hipError_t je = side_join(c);
                    if (je != hipSuccess) return je;
                }
                timer_end(c, 0);
                continue;
            }
            if (sub && leafy) hipLaunchKernelGGL((k_fitch_up<true, true, true>), grid, dim3(kBlock), 0, c->stream, up);
            else if (grp && ht.up_recomp_g[h]) hipLaunchKernelGGL((k_fitch_up<true, false, true, true>), grid, dim3(kBlock), 0, c->stream, up);
            else if (sub) hipLaunchKernelGGL((k_fitch_up<true, false, true>), grid, dim3(kBlock), 0, c->stream, up);
            else if (ap && leafy) hipLaunchKernelGGL((k_fitch_up<true, true>), grid, dim3(kBlock), 0, c->stream, up);
            else if (ap) hipLaunchKernelGGL((k_fitch_up<true, false>), grid, dim3(kBlock), 0, c->stream, up);
            else hipLaunchKernelGGL((k_fitch_up<false, false>), grid, dim3(kBlock), 0, c->stream, up);
            if (fork) {
                const hipError_t je = side_join(c);
                if (je != hipSuccess) return je;
            }
            timer_end(c, 0);
        }
    }

    if (clu) {   // the sweeps, band by band
        const ClArgs ca0{dt.cl_items, dt.cl_wg_off, dt.cl_slot_of, dt.cl_pslot, cl.upm_base, 0};
        for (size_t bnd = 0; bnd + 1 < cl.band_wg.size(); ++bnd) {
            ClArgs ca = ca0;
            ca.wg0 = cl.band_wg[bnd];
            const int64_t nwg = cl.band_wg[bnd + 1] - ca.wg0;
            if (nwg == 0) continue;
            timer_begin(c, 0);
            hipLaunchKernelGGL(k_fitch_up_cluster, dim3((unsigned)(nwg * tiles)), dim3(kWave), 0, c->stream, up, ca);
            timer_end(c, 0);
        }
    }

    hipError_t e = hipMemsetAsync(c->shard_cnt, 0, sizeof(uint32_t) * kShards, c->stream);
    if (e != hipSuccess) return e;
    DownArgs dn{};
    dn.child_off = dt.child_off;
    dn.child_enc = child_enc;
    dn.parent_dense = dt.parent_dense;
    dn.internal_id = dt.internal_id;
    dn.leaf_id = dt.leaf_id;
    dn.leaf_flag = c->leaf_flag;
    dn.leaf_planes = c->leaf_planes;
    dn.leaf_present = c->leaf_present;
    dn.sets = reinterpret_cast<uint4*>(c->sets);
    dn.cmask = c->cmask;
    dn.root_final = c->root_final;
    dn.dense_base = -1;
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
    dn.forced = (c->has_forced && block) ? c->forced : nullptr;
    dn.absent_code0 = false;
    dn.all_present = c->leaves_all_present;
    dn.vleaf = reinterpret_cast<const int4*>(dt.vleaf);
    dn.vinner = dt.vinner;
    if (sub_down) {   // the S children's leaf words and node ids (their tail descriptors)
        dn.tail = dt.tail_desc_k;
        dn.num_s = ht.num_tail_s;
        dn.sbase = ht.sbase;
        dn.sub_planes = c->sub_planes;
    }
    // pre-order sweeps over the post-order's clusters (every level swept), the bands top-down
    const bool cld = clu && cl.down && !sub_down;
    if (cld) {
        for (size_t bnd = cl.band_wg.size() - 1; bnd-- > 0;) {
            const ClDownArgs ca{dt.cl_down_items, dt.cl_wg_off, cl.band_wg[bnd]};
            const int64_t nwg = cl.band_wg[bnd + 1] - ca.wg0;
            if (nwg == 0) continue;
            timer_begin(c, 1);
            hipLaunchKernelGGL(k_down_cluster<Mode::kFitch>, dim3((unsigned)(nwg * tiles)), dim3(kWave), 0, c->stream, dn, ca);
            timer_end(c, 1);
        }
    }
    const int D = cld ? 0 : (int)down_off.size() - 1;
    for (int d = 0; d < D; ++d) {
        if (c->narrow_max > 0 && down_off[d + 1] - down_off[d] <= c->narrow_max) {
            int d1 = d + 1;
            while (d1 < D && down_off[d1 + 1] - down_off[d1] <= c->narrow_max) ++d1;
            if (d1 - d >= 2) {
                dn.desc = down_desc;
                const int32_t* tab = dt.lvl + ht.lvl_down[form];
                const int32_t* base = sub ? (ht.down_dense_k ? dt.lvl + ht.lvl_base_k : nullptr)
                                          : (virt && ht.down_dense_v) ? tab : nullptr;
                timer_begin(c, 1);
                // (subtree form: the lean body as in the level kernels, S2 / S3 records in k_tail)
                if (block && ap) hipLaunchKernelGGL((k_down_band<Mode::kBlockFitch, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (block) hipLaunchKernelGGL((k_down_band<Mode::kBlockFitch, false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                // (level groups inside the band when PM_OPT_GROUP_WAVES is on)
                else if (sub_down && c->group_waves > 0) hipLaunchKernelGGL((k_down_band<Mode::kFitch, true, true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (sub_down) hipLaunchKernelGGL((k_down_band<Mode::kFitch, true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (ap && c->group_waves > 0) hipLaunchKernelGGL((k_down_band<Mode::kFitch, true, false, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (ap) hipLaunchKernelGGL((k_down_band<Mode::kFitch, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (c->group_waves > 0) hipLaunchKernelGGL((k_down_band<Mode::kFitch, false, false, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else hipLaunchKernelGGL((k_down_band<Mode::kFitch, false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                timer_end(c, 1);
                d = d1 - 1;
                continue;
            }
        }
        dn.desc = down_desc + down_off[d];
        dn.count = down_off[d + 1] - down_off[d];
        if (dn.count == 0) continue;
        // level d = one range of dense indices: [down_off[d], down_off[d+1]) in the leaf-parent
        // form, from down_dense_base_k[d] in the subtree form
        const bool dense = sub ? ht.down_dense_k : virt && ht.down_dense_v;
        dn.dense_base = !dense ? -1 : sub ? ht.down_dense_base_k[d] : down_off[d];
        // levels d .. d + g - 1 in one launch (PM_OPT_GROUP_*), none of them starting a band
        auto narrow_down = [&](int l) { return c->narrow_max > 0 && down_off[l + 1] - down_off[l] <= c->narrow_max; };
        auto band_at = [&](int l) { return narrow_down(l) && l + 1 < D && narrow_down(l + 1); };
        int g = 1;
        int64_t items = dn.count;
        while (!block && c->group_waves > 0 && g < std::min(c->group_levels, kGroupLevels) && d + g < D) {
            const int32_t ng = down_off[d + g + 1] - down_off[d + g];
            if (ng == 0 || (items + ng) * tiles > c->group_waves || band_at(d + g)) break;
            items += ng;
            ++g;
        }
        if (g > 1) {
            for (int k = 0; k < 4; ++k) {
                const int l = std::min(d + k, d + g - 1);
                if (k > 0) dn.split[k - 1] = k < g ? down_off[d + k] - down_off[d] : (int32_t)items;
                dn.dense_g[k] = !dense ? -1 : sub ? ht.down_dense_base_k[l] : down_off[l];
            }
            dn.count = (int32_t)items;
            const dim3 grid = wave_grid(dn.count, tiles);
            timer_begin(c, 1);
            if (sub_down && dense) hipLaunchKernelGGL((k_down<Mode::kFitch, true, true, true, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else if (sub_down) hipLaunchKernelGGL((k_down<Mode::kFitch, true, false, true, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else if (ap && dense) hipLaunchKernelGGL((k_down<Mode::kFitch, true, true, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else if (ap) hipLaunchKernelGGL((k_down<Mode::kFitch, true, false, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else hipLaunchKernelGGL((k_down<Mode::kFitch, false, false, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            timer_end(c, 1);
            d += g - 1;
            continue;
        }
        const dim3 grid = wave_grid(dn.count, tiles);
        timer_begin(c, 1);
        // (subtree form: the levels' descriptors omit S2 / S3 children, whose records come
        // from the tail launch, so the lean kernels run every level)
        if (block && ap) hipLaunchKernelGGL((k_down<Mode::kBlockFitch, true, false>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (block) hipLaunchKernelGGL((k_down<Mode::kBlockFitch, false, false>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (sub_down && dense) hipLaunchKernelGGL((k_down<Mode::kFitch, true, true, true>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (sub_down) hipLaunchKernelGGL((k_down<Mode::kFitch, true, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (ap && dense) hipLaunchKernelGGL((k_down<Mode::kFitch, true, true>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (ap) hipLaunchKernelGGL((k_down<Mode::kFitch, true, false>), grid, dim3(kBlock), 0, c->stream, dn);
        else hipLaunchKernelGGL((k_down<Mode::kFitch, false, false>), grid, dim3(kBlock), 0, c->stream, dn);
        timer_end(c, 1);
    }
    // The tail (children beyond the second, S2 / S3 subtrees) needs only its parents'
    // finals: one flat launch after the levels.
    // (PM_OPT_SUB_DOWN: the S2 / S3 items, the first num_tail_s, were done by the levels)
    const int32_t tail_skip = sub_down ? ht.num_tail_s : 0;
    const int32_t tail_total = (sub ? ht.num_tail_k : virt ? ht.num_tail_v : ht.num_tail) - tail_skip;
    if (tail_total > 0) {
        DownArgs t = dn;
        t.tail = (sub ? dt.tail_desc_k : virt ? dt.tail_desc_v : dt.tail_desc) + tail_skip;
        t.count = tail_total;
        t.num_s = sub && !sub_down ? ht.num_tail_s : 0;
        t.sbase = ht.sbase;
        t.sub_planes = c->sub_planes;
        const dim3 grid = wave_grid(t.count, tiles);
        timer_begin(c, 5);
        if (sub) hipLaunchKernelGGL((k_tail<Mode::kFitch, true, true>), grid, dim3(kBlock), 0, c->stream, t);
        else if (block && ap) hipLaunchKernelGGL((k_tail<Mode::kBlockFitch, true>), grid, dim3(kBlock), 0, c->stream, t);
        else if (block) hipLaunchKernelGGL((k_tail<Mode::kBlockFitch, false>), grid, dim3(kBlock), 0, c->stream, t);
        else if (ap) hipLaunchKernelGGL((k_tail<Mode::kFitch, true>), grid, dim3(kBlock), 0, c->stream, t);
        else hipLaunchKernelGGL((k_tail<Mode::kFitch, false>), grid, dim3(kBlock), 0, c->stream, t);
        timer_end(c, 5);
    }
    return hipGetLastError();
}

#if !PM_NT_LOADS
hipError_t launch_score(pm_ctx* c) {
    hipError_t e = hipMemsetAsync(c->score, 0, sizeof(int32_t) * c->num_sites, c->stream);
    if (e != hipSuccess) return e;
    const bool use_lds = c->num_sites * 4 <= 150 * 1024;
    const int spb = kShards >= 1024 ? kShards / 256 : 4;   // 256 workgroups
    const int blocks = (kShards + spb - 1) / spb;
    const size_t lds = use_lds ? (size_t)c->num_sites * 4 : 0;
    timer_begin(c, 2);
    hipLaunchKernelGGL(k_site_score, dim3(blocks), dim3(kScoreBlock), lds, c->stream, c->recs, c->shard_cnt,
                       c->shard_cap, (uint32_t)c->ht.root, c->score, c->num_sites, spb, use_lds);
    timer_end(c, 2);
    return hipGetLastError();
}

#endif

// This file's code object, loaded ahead of its first launch (pm_warmup).
hipError_t warm_fitch() {
    hipFuncAttributes at;
    return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_fitch_up_wide<true>));
}

}  // namespace pm

