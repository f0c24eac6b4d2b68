// pm_sankoff.hip -- unit-cost Sankoff over the 16 codes for every column at once (gfx950).
//
// Restates src/fitchSankoff.cpp:359-405 (forward), :487-531 (backward), :676-703
// (assignment), as driven by the low-mem MSA driver (src/panman.cpp:1568-1613).
//
// Exact compression of the reference's 16 x int32 cost vectors: with unit costs a child
// contributes  min_k((i != k) + c[k]) = min(c) + [i not optimal in c]  to its parent, and
// the backward argmin given parent state s only asks whether s is optimal, whether s is
// exactly one above optimal, and which codes are optimal.  So a node keeps two 16-bit sets
// per site: Z0 = optimal codes, Z1 = codes one above optimal (INF <=> Z0 == 0).  Forward:
// count, per code, the finite children that hold it optimal (bit-sliced counters, B bits
// per code); Z0 = codes of maximum count, Z1 = codes of maximum - 1.  B is chosen per
// node by out-degree class so binary nodes pay for 2-bit counters only.
#include "pm_kernels.h"

#if PM_NT_LOADS   // (pm_sankoff_nt.hip: the same passes, non-temporal set-record loads)
#define launch_sankoff launch_sankoff_nt
#define warm_sankoff warm_sankoff_nt
#endif

namespace pm {
namespace {

// Z0 of one child (leaf, virtual leaf-parent or record), as k_sankoff_up reads it.
template <class Args>
__device__ __forceinline__ void child_z0(const Args& a, int32_t c, int32_t l0, int32_t l1, int tile, int lane,
                                         int64_t word, uint32_t* z) {
    if (c >= 0 && (c & kVirtualBit)) {
        uint32_t x[16];
        leaf_set16(a, l0, word, z);
        if (l1 >= 0) {
            leaf_set16(a, l1, word, x);
#pragma unroll
            for (int v = 0; v < 16; ++v) z[v] |= x[v];
        }
    } else if (c >= 0) {
        load_sankoff(a.sets, a.cmask, a.cons, c, a.tiles, tile, lane, word, z, nullptr, false);
    } else {
        leaf_set16(a, -c - 1, word, z);
    }
}

template <int B>
__device__ __forceinline__ void count_child(uint32_t (&cnt)[16][B], uint32_t& finite, const uint32_t* z) {
    finite |= any_plane(z);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        uint32_t x = z[v];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint32_t t = cnt[v][b] & x;
            cnt[v][b] ^= x;
            x = t;
        }
    }
}

// AP: every leaf present -- the first two children's loads are issued together (see
// fetch_child_ap), the third (if any) after.
// SUB: subtree form (every leaf present) -- the first two children may be S2 / S3 subtrees
// of three / four leaves, whose Z0 (= their Fitch set: binary unit-cost Sankoff keeps the
// codes of maximum count, AND if non-empty else OR) comes from subtree_set_ap in registers.
// Their records need the leaves wherever the subtree's leaves disagree (sd: dirty lanes).
// GROUP (grouped post-order launches, subtree form): the descriptor's pad0 / pad1 (>= 0) name
// first / second children of this same launch -- binary, so their Z0 is the AND-else-OR of
// their children's Z0 -- recomputed in registers (fold_first_two) instead of loaded; the
// first two children's counts then follow from their AND (count 2) and OR (count >= 1).
// gi: the node's index in the descriptor array; SUB: up slots (UpArgs::upm), as fitch_up_node.
// PLAIN: the grouped order's plain prefix (binary, no S2 / S3 child, nothing recomputed; see
// fitch_up_node): branch-free child sets, no polytomy loop -- fewer registers, more waves.
template <int B, bool AP, bool SUB = false, bool GROUP = false, bool PLAIN = false>
__device__ __forceinline__ void sankoff_up_node(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int lane) {
    const int32_t n = d.node;
    const int64_t word = (int64_t)tile * kWave + lane;
    UpSlots sl{0, 0, 0, 0};
    if constexpr (SUB) sl = load_up_slots(a, gi, tile);
    const int32_t ps = SUB ? a.pslot[gi] : -1;

    uint32_t cnt[16][B];
#pragma unroll
    for (int v = 0; v < 16; ++v)
#pragma unroll
        for (int b = 0; b < B; ++b) cnt[v][b] = 0;
    uint32_t finite = 0, z[16], sd = 0;
    const int32_t e0 = d.e0, e1 = d.e1;
    int32_t first = e0;
    if (GROUP && (d.pad0 >= 0 || d.pad1 >= 0)) {
        static_assert(!GROUP || (AP && SUB && B >= 2), "grouped launches: subtree form, narrow nodes");
        uint32_t both[16], either[16], vd = 0;
        fold_first_two<SUB, kUpGroupDepth, kSankoffRec>(a, d, gi, tile, lane, word, both, either, vd);
        const bool two = e1 - e0 > 1;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            cnt[v][0] = two ? either[v] & ~both[v] : either[v];
            cnt[v][1] = two ? both[v] : 0u;
        }
        finite = any_plane(either);
        sd = vd;   // (also a cherry's disagreeing leaves: extra dirty lanes, harmless)
        first = e0 + 2;
    } else if constexpr (AP) {
        const int4 vl0 = SUB ? make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]) : make_int4(d.vl0[0], d.vl0[1], -1, -1);
        const int4 vl1 = SUB ? make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]) : make_int4(d.vl1[0], d.vl1[1], -1, -1);
        ChildFetch f0, f1;
        fetch_child_ap<kSankoffRec, false, SUB, SUB>(a, d.c0, vl0, tile, lane, word, f0, sl.x0, sl.s0);
        if (e1 - e0 > 1) fetch_child_ap<kSankoffRec, false, SUB, SUB>(a, d.c1, vl1, tile, lane, word, f1, sl.x1, sl.s1);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t vd = 0;
        if constexpr (PLAIN) child_set_plain(d.c0, vl0, f0, z, vd);
        else child_set_ap<SUB>(d.c0, vl0, f0, z, vd);
        if (SUB && !PLAIN && kid_shape(d.c0)) sd |= vd;
        count_child<B>(cnt, finite, z);
        if (e1 - e0 > 1) {
            vd = 0;
            if constexpr (PLAIN) child_set_plain(d.c1, vl1, f1, z, vd);
            else child_set_ap<SUB>(d.c1, vl1, f1, z, vd);
            if (SUB && !PLAIN && kid_shape(d.c1)) sd |= vd;
            count_child<B>(cnt, finite, z);
        }
        first = e0 + 2;
    }
    for (int32_t e = first; !PLAIN && e < e1; ++e) {   // one or two leaves: Z0 = their codes (:376-402)
        const int32_t c = e == e0 ? d.c0 : (e == e0 + 1 ? d.c1 : __builtin_amdgcn_readfirstlane(a.child_enc[e]));
        const int4 vl = !(c >= 0 && (c & kVirtualBit)) ? make_int4(-1, -1, -1, -1)
                        : e == e0                       ? make_int4(d.vl0[0], d.vl0[1], -1, -1)
                        : e == e0 + 1                   ? make_int4(d.vl1[0], d.vl1[1], -1, -1)
                                                        : a.vleaf[c & kDenseMask];
        child_z0(a, c, __builtin_amdgcn_readfirstlane(vl.x), __builtin_amdgcn_readfirstlane(vl.y), tile, lane, word, z);
        count_child<B>(cnt, finite, z);   // an all-INF child adds nothing (:398-400)
    }
    // maximum count per site, most significant bit first
    uint32_t cand[16], mx[B];
#pragma unroll
    for (int v = 0; v < 16; ++v) cand[v] = ~0u;
#pragma unroll
    for (int b = B - 1; b >= 0; --b) {
        uint32_t hit = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) hit |= cand[v] & cnt[v][b];
        mx[b] = hit;
#pragma unroll
        for (int v = 0; v < 16; ++v) cand[v] &= cnt[v][b] | ~hit;
    }
    // max - 1 (max >= 1 wherever a child is finite)
    uint32_t mm1[B], borrow = ~0u;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        mm1[b] = mx[b] ^ borrow;
        borrow &= ~mx[b];
    }
    uint32_t z0[16], z1[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        uint32_t eq = finite;
#pragma unroll
        for (int b = 0; b < B; ++b) eq &= ~(cnt[v][b] ^ mm1[b]);
        z0[v] = cand[v] & finite;
        z1[v] = eq;
    }
    // dirty lanes: complex ones, and all when a child's code can differ from a single
    // optimal code (three or more children: Z0 = {c}, Z1 = {} still admits a child at
    // count 1 <= max - 2) or a leaf can be absent
    uint64_t rx, rs, rd;
    store_sankoff(a.sets, a.cmask, a.cons, n, a.tiles, tile, lane, word, z0, z1,
                  !a.all_present || e1 - e0 > 2 || sd != 0u, rx, rs, rd);
    push_up_slot(a, ps, tile, lane, rx, rs);
    push_children(a, tile, lane, e0, e1, d.c0, d.c1, rx, rs, rd, n == a.root_dense);
}

#ifndef PM_SK_UP_WAVES
#define PM_SK_UP_WAVES 1
#endif
// the plain kernel at 8 waves per SIMD (64 VGPRs, 8 B spilled): N* Sankoff 19.46 -> 19.34-19.38 ms,
// C3 6.15 -> 6.09-6.11 ms against 7 (r05aj)
#ifndef PM_SK_PLAIN_UP_WAVES
#define PM_SK_PLAIN_UP_WAVES 8
#endif
// GROUP: 4 waves per SIMD (3: no scratch spills, C3 Sankoff 2-3 % slower; see PM_GROUP_UP_WAVES)
#ifndef PM_SK_GROUP_UP_WAVES
#define PM_SK_GROUP_UP_WAVES 4
#endif
template <int B, bool AP, bool SUB = false, bool GROUP = false, bool PLAIN = false>
__global__ __launch_bounds__(kBlock, PLAIN ? PM_SK_PLAIN_UP_WAVES : GROUP ? PM_SK_GROUP_UP_WAVES : PM_SK_UP_WAVES) void k_sankoff_up(UpArgs a) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    wave_item(wave, a.tiles, item, tile);
    if (item >= a.count) return;
    sankoff_up_node<B, AP, SUB, GROUP, PLAIN>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, lane);
}

// Wide nodes (out-degree > 3): one workgroup per (node, tile), children dealt round-robin
// to its 4 waves (64 encodings per vector load, two children fetched before either is
// counted); the waves' bit-sliced counters are summed through LDS (the sum of the
// per-wave counts is the node's count: src/fitchSankoff.cpp:391-402 is a sum over
// children), then Z0 / Z1 as in k_sankoff_up.
template <int B>
__device__ __forceinline__ void sankoff_wide_node(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int wave,
                                                  int lane, uint32_t (*part)[kWave]) {
    const int32_t n = d.node, e0 = d.e0, e1 = d.e1;
    const int64_t word = (int64_t)tile * kWave + lane;
    uint32_t cnt[16][B];
#pragma unroll
    for (int v = 0; v < 16; ++v)
#pragma unroll
        for (int b = 0; b < B; ++b) cnt[v][b] = 0;
    uint32_t finite = 0;
    for (int32_t base = e0 + wave; base < e1; base += kWavesPerBlock * kWave) {
        const int32_t my = base + kWavesPerBlock * lane;
        const int32_t enc = my < e1 ? a.child_enc[my] : 0;
        const int4 vl = my < e1 && enc >= 0 && (enc & kVirtualBit) ? a.vleaf[enc & kDenseMask]
                                                                   : make_int4(-1, -1, -1, -1);
        const int cntc = min(kWave, (e1 - base + kWavesPerBlock - 1) / kWavesPerBlock);
        for (int k = 0; k < cntc; k += 2) {
            uint32_t z0[16], z1[16];
            const int32_t c0 = __builtin_amdgcn_readlane(enc, k);
            child_z0(a, c0, __builtin_amdgcn_readlane(vl.x, k), __builtin_amdgcn_readlane(vl.y, k), tile, lane, word, z0);
            const bool two = k + 1 < cntc;
            if (two) {
                const int32_t c1 = __builtin_amdgcn_readlane(enc, k + 1);
                child_z0(a, c1, __builtin_amdgcn_readlane(vl.x, k + 1), __builtin_amdgcn_readlane(vl.y, k + 1), tile,
                         lane, word, z1);
            }
            count_child<B>(cnt, finite, z0);
            if (two) count_child<B>(cnt, finite, z1);
        }
    }
    // sum the waves' counters into wave 0, one wave at a time through one LDS buffer
    for (int w = 1; w < kWavesPerBlock; ++w) {
        if (wave == w) {
#pragma unroll
            for (int v = 0; v < 16; ++v)
#pragma unroll
                for (int b = 0; b < B; ++b) part[v * B + b][lane] = cnt[v][b];
            part[16 * B][lane] = finite;
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                uint32_t carry = 0;
#pragma unroll
                for (int b = 0; b < B; ++b) {
                    const uint32_t x = part[v * B + b][lane], y = cnt[v][b];
                    cnt[v][b] = x ^ y ^ carry;
                    carry = (x & y) | (carry & (x ^ y));
                }
            }
            finite |= part[16 * B][lane];
        }
        __syncthreads();
    }
    if (wave != 0) return;
    uint32_t cand[16], mx[B];
#pragma unroll
    for (int v = 0; v < 16; ++v) cand[v] = ~0u;
#pragma unroll
    for (int b = B - 1; b >= 0; --b) {
        uint32_t hit = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) hit |= cand[v] & cnt[v][b];
        mx[b] = hit;
#pragma unroll
        for (int v = 0; v < 16; ++v) cand[v] &= cnt[v][b] | ~hit;
    }
    uint32_t mm1[B], borrow = ~0u;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        mm1[b] = mx[b] ^ borrow;
        borrow &= ~mx[b];
    }
    uint32_t z0[16], z1[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        uint32_t eq = finite;
#pragma unroll
        for (int b = 0; b < B; ++b) eq &= ~(cnt[v][b] ^ mm1[b]);
        z0[v] = cand[v] & finite;
        z1[v] = eq;
    }
    uint64_t rx, rs, rd;
    store_sankoff(a.sets, a.cmask, a.cons, n, a.tiles, tile, lane, word, z0, z1, true, rx, rs, rd);
    if (a.upm != nullptr) push_up_slot(a, a.pslot[gi], tile, lane, rx, rs);   // (subtree form)
    push_children(a, tile, lane, e0, e1, d.c0, d.c1, rx, rs);
}

template <int B>
__global__ __launch_bounds__(kBlock) void k_sankoff_up_wide(UpArgs a) {
    __shared__ uint32_t part[16 * B + 1][kWave];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    block_item(a.tiles, item, tile);
    sankoff_wide_node<B>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, wave, lane, part);
}

// A small level holding nodes of out-degree <= 3 and 4..255 in ONE launch instead of two or
// three dependent ones (deep trees with polytomies): blocks [0, narrow_blocks) are
// k_sankoff_up's waves over a.desc, the rest one workgroup per (wide node, tile) over wdesc
// with BW-bit counters (the 16-child class counted at the wider width: same sums).
static_assert(PM_TILE_FAST, "k_sankoff_up_mixed numbers its blocks on one grid axis");
template <int BW, bool AP, bool SUB = false, bool GROUP = false>
__global__ __launch_bounds__(kBlock) void k_sankoff_up_mixed(UpArgs a, const NodeDesc* wdesc, int32_t narrow_blocks) {
    __shared__ uint32_t part[16 * BW + 1][kWave];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if ((int32_t)blockIdx.x < narrow_blocks) {
        int32_t item;
        int tile;
        wave_item(wave, a.tiles, item, tile);
        if (item < a.count) sankoff_up_node<2, AP, SUB, GROUP>(a, a.desc[item], (int32_t)(a.desc - a.desc_all) + item, tile, lane);
        return;
    }
    const int32_t b = (int32_t)blockIdx.x - narrow_blocks;
    const int32_t item = b / a.tiles;
    sankoff_wide_node<BW>(a, wdesc[item], (int32_t)(wdesc - a.desc_all) + item, b - item * a.tiles, wave, lane, part);
}

// Narrow post-order levels (PM_OPT_NARROW, see k_fitch_up_band): a run of levels whose
// nodes all have out-degree <= 3, at most narrow_max of them per level, walked by one
// launch, one 1024-thread workgroup per tile, a barrier between levels.
template <bool AP, bool SUB = false, bool GROUP = false>
__global__ __launch_bounds__(kBandBlock) void k_sankoff_up_band(UpArgs a, const int32_t* class_off, int32_t h0, int32_t h1) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int tile = blockIdx.x;
    for (int32_t h = h0; h < h1; ++h) {
        const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1];
        for (int32_t i = b + wave; i < m; i += kBandWaves) sankoff_up_node<2, AP, SUB, GROUP>(a, a.desc[i], i, tile, lane);
        __syncthreads();
    }
}

// ---- LDS-staged post-order sweeps (PM_OPT_CLUSTER; schedule pm_cluster.cpp, as
// k_fitch_up_cluster): one wave per (cluster, tile) walks the cluster depth first; a child of the
// same cluster hands its Z0 -- all a parent reads of it (src/fitchSankoff.cpp:376-402) -- through
// an LDS slot, every other child is read as k_sankoff_up reads it.  Taken when the plan sweeps
// every height (the level kernels' grouped order is not built around the clusters) and no swept
// node has more than 255 children (8-bit counters; more: k_sankoff_part).
template <int B>
__device__ __forceinline__ void sankoff_z(const uint32_t (&cnt)[16][B], uint32_t finite, uint32_t* z0, uint32_t* z1) {
    uint32_t cand[16], mx[B];   // maximum count per site, most significant bit first
#pragma unroll
    for (int v = 0; v < 16; ++v) cand[v] = ~0u;
#pragma unroll
    for (int b = B - 1; b >= 0; --b) {
        uint32_t hit = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) hit |= cand[v] & cnt[v][b];
        mx[b] = hit;
#pragma unroll
        for (int v = 0; v < 16; ++v) cand[v] &= cnt[v][b] | ~hit;
    }
    uint32_t mm1[B], borrow = ~0u;   // max - 1
#pragma unroll
    for (int b = 0; b < B; ++b) {
        mm1[b] = mx[b] ^ borrow;
        borrow &= ~mx[b];
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        uint32_t eq = finite;
#pragma unroll
        for (int b = 0; b < B; ++b) eq &= ~(cnt[v][b] ^ mm1[b]);
        z0[v] = cand[v] & finite;
        z1[v] = eq;
    }
}

// Z0 / Z1 to the record (as k_sankoff_up / k_sankoff_up_wide write them), the masks into the
// parent's up slot (a parent in a later band) and to the materialised children, Z0 into the
// node's LDS slot when its parent is in this cluster.
__device__ __forceinline__ void sk_cluster_finish(const UpArgs& a, const NodeDesc& d, int32_t ps, ClSlots& S, int tile,
                                                  int lane, int64_t word, const uint32_t* z0, const uint32_t* z1,
                                                  bool dirty_extra) {
    uint64_t rx, rs, rd;
    store_sankoff(a.sets, a.cmask, a.cons, d.node, a.tiles, tile, lane, word, z0, z1, dirty_extra, rx, rs, rd);
    push_up_slot(a, ps, tile, lane, rx, rs);
    if (d.e1 - d.e0 > 3) push_children(a, tile, lane, d.e0, d.e1, d.c0, d.c1, rx, rs);
    else push_children(a, tile, lane, d.e0, d.e1, d.c0, d.c1, rx, rs, rd, d.node == a.root_dense);
    if (d.parent >= 0) slot_write(S, d.parent, lane, z0);
}

// A node of out-degree <= 3: sankoff_up_node<2, true, true>'s reads, in-cluster children from LDS.
__device__ __forceinline__ void sk_cluster_node(const UpArgs& a, const ClArgs& c, const ClMeta& m, ClSlots& S, int tile,
                                                int lane, int64_t word) {
    const NodeDesc& d = m.d;
    const int32_t e0 = d.e0, e1 = d.e1;
    uint32_t cnt[16][2], finite = 0, z[16], sd = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) cnt[v][0] = cnt[v][1] = 0;
    const int4 vl0 = make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), vl1 = make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]);
    ChildFetch f0, f1;
    if (d.pad0 < 0) fetch_child_ap<kSankoffRec, false, true, true>(a, d.c0, vl0, tile, lane, word, f0, m.s.x0, m.s.s0);
    if (e1 - e0 > 1 && d.pad1 < 0) fetch_child_ap<kSankoffRec, false, true, true>(a, d.c1, vl1, tile, lane, word, f1, m.s.x1, m.s.s1);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t vd = 0;
    if (d.pad0 >= 0) slot_read(S, d.pad0, lane, z);
    else {
        child_set_ap<true>(d.c0, vl0, f0, z, vd);
        if (kid_shape(d.c0)) sd |= vd;
    }
    count_child<2>(cnt, finite, z);
    if (e1 - e0 > 1) {
        vd = 0;
        if (d.pad1 >= 0) slot_read(S, d.pad1, lane, z);
        else {
            child_set_ap<true>(d.c1, vl1, f1, z, vd);
            if (kid_shape(d.c1)) sd |= vd;
        }
        count_child<2>(cnt, finite, z);
    }
    for (int32_t e = e0 + 2; e < e1; ++e) {   // an out-degree-3 node's third child
        const int32_t ch = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        const int32_t s = materialised(ch) ? __builtin_amdgcn_readfirstlane(c.slot_of[ch]) : -1;
        if (s >= 0) {
            slot_read(S, s, lane, z);
        } else {
            const int4 vl = ch >= 0 && (ch & kVirtualBit) ? a.vleaf[ch & kDenseMask] : make_int4(-1, -1, -1, -1);
            child_z0(a, ch, __builtin_amdgcn_readfirstlane(vl.x), __builtin_amdgcn_readfirstlane(vl.y), tile, lane, word, z);
        }
        count_child<2>(cnt, finite, z);
    }
    uint32_t z0[16], z1[16];
    sankoff_z<2>(cnt, finite, z0, z1);
    sk_cluster_finish(a, d, m.ps, S, tile, lane, word, z0, z1, e1 - e0 > 2 || sd != 0u);
}

// A node of out-degree 4..255 (sankoff_wide_node's counts, one wave): B-bit counters.
template <int B>
__device__ __forceinline__ void sk_cluster_wide(const UpArgs& a, const ClArgs& c, const ClMeta& m, ClSlots& S, int tile,
                                                int lane, int64_t word) {
    const NodeDesc& d = m.d;
    uint32_t cnt[16][B], finite = 0, z[16];
#pragma unroll
    for (int v = 0; v < 16; ++v)
#pragma unroll
        for (int b = 0; b < B; ++b) cnt[v][b] = 0;
    for (int32_t e = d.e0; e < d.e1; ++e) {
        const int32_t ch = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        const int32_t s = materialised(ch) ? __builtin_amdgcn_readfirstlane(c.slot_of[ch]) : -1;
        if (s >= 0) {
            slot_read(S, s, lane, z);
        } else {
            const int4 vl = ch >= 0 && (ch & kVirtualBit) ? a.vleaf[ch & kDenseMask] : make_int4(-1, -1, -1, -1);
            child_z0(a, ch, __builtin_amdgcn_readfirstlane(vl.x), __builtin_amdgcn_readfirstlane(vl.y), tile, lane, word, z);
        }
        count_child<B>(cnt, finite, z);
    }
    uint32_t z0[16], z1[16];
    sankoff_z<B>(cnt, finite, z0, z1);
    sk_cluster_finish(a, d, m.ps, S, tile, lane, word, z0, z1, true);
}

#ifndef PM_SK_CL_WAVES   // waves per SIMD (occupancy bound of the Sankoff sweep kernel)
#define PM_SK_CL_WAVES 2
#endif
__global__ __launch_bounds__(kWave, PM_SK_CL_WAVES) void k_sankoff_up_cluster(UpArgs a, ClArgs c) {
    __shared__ ClSlots S;
    const int lane = threadIdx.x;
    const int32_t b = (int32_t)blockIdx.x;
    const int32_t wl = b / a.tiles;
    const int tile = b - wl * a.tiles;
    const int32_t i0 = c.wg_off[c.wg0 + wl], steps = c.wg_off[c.wg0 + wl + 1] - i0;
    const int64_t word = (int64_t)tile * kWave + lane;
    // the next step's descriptor and up slots in flight during this one
    uint32_t mv = cl_meta_load(a, c, i0, tile, lane);
    for (int32_t r = 0; r < steps; ++r) {
        ClMeta m;
        cl_meta_get(mv, m);
        if (r + 1 < steps) mv = cl_meta_load(a, c, i0 + r + 1, tile, lane);
        const int32_t deg = m.d.e1 - m.d.e0;
        if (deg <= 3) sk_cluster_node(a, c, m, S, tile, lane, word);
        else if (deg <= 15) sk_cluster_wide<4>(a, c, m, S, tile, lane, word);
        else sk_cluster_wide<8>(a, c, m, S, tile, lane, word);
    }
}

// Nodes of any out-degree above 255 (src/fitchSankoff.cpp:391-402 sums over every child,
// whatever their number): the children are cut into parts of kPartChildren; one wave per
// (part, tile) counts its part into 8-bit bit-sliced counters (k_sankoff_part) and writes
// them to scratch; one wave per (node, tile) then adds the parts code by code into BW-bit
// counters and keeps the running maximum with the codes at the maximum (Z0) and one below
// it (Z1) as it goes (k_sankoff_merge), so no 16 x BW counter file is ever held.
__global__ __launch_bounds__(kBlock) void k_sankoff_part(UpArgs a, const PartDesc* parts, int32_t nparts,
                                                         uint32_t* scratch) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t pi;
    int tile;
    wave_item(wave, a.tiles, pi, tile);
    if (pi >= nparts) return;
    const PartDesc pd = parts[pi];
    const NodeDesc& d = a.desc[pd.item];
    const int32_t lo = d.e0 + pd.sub * kPartChildren, hi = min(d.e1, lo + kPartChildren);
    const int64_t word = (int64_t)tile * kWave + lane;
    uint32_t cnt[16][8];
#pragma unroll
    for (int v = 0; v < 16; ++v)
#pragma unroll
        for (int b = 0; b < 8; ++b) cnt[v][b] = 0;
    uint32_t finite = 0;
    for (int32_t base = lo; base < hi; base += kWave) {
        const int32_t my = base + lane;
        const int32_t enc = my < hi ? a.child_enc[my] : 0;
        const int4 vl = my < hi && enc >= 0 && (enc & kVirtualBit) ? a.vleaf[enc & kDenseMask]
                                                                   : make_int4(-1, -1, -1, -1);
        const int cntc = min(kWave, hi - base);
        for (int k = 0; k < cntc; k += 2) {
            uint32_t z0[16], z1[16];
            const int32_t c0 = __builtin_amdgcn_readlane(enc, k);
            child_z0(a, c0, __builtin_amdgcn_readlane(vl.x, k), __builtin_amdgcn_readlane(vl.y, k), tile, lane, word, z0);
            const bool two = k + 1 < cntc;
            if (two) {
                const int32_t c1 = __builtin_amdgcn_readlane(enc, k + 1);
                child_z0(a, c1, __builtin_amdgcn_readlane(vl.x, k + 1), __builtin_amdgcn_readlane(vl.y, k + 1), tile,
                         lane, word, z1);
            }
            count_child<8>(cnt, finite, z0);
            if (two) count_child<8>(cnt, finite, z1);
        }
    }
    uint32_t* out = scratch + (size_t)pd.global * kPartPlanes * a.wpad + word;
#pragma unroll
    for (int v = 0; v < 16; ++v)
#pragma unroll
        for (int b = 0; b < 8; ++b) out[(size_t)(v * 8 + b) * a.wpad] = cnt[v][b];
    out[(size_t)128 * a.wpad] = finite;
}

template <int BW>
__global__ __launch_bounds__(kBlock) void k_sankoff_merge(UpArgs a, const uint32_t* scratch) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    wave_item(wave, a.tiles, item, tile);
    if (item >= a.count) return;
    const NodeDesc& d = a.desc[item];
    const int32_t n = d.node, e0 = d.e0, e1 = d.e1;
    const int32_t p0 = d.pad0, np = (e1 - e0 + kPartChildren - 1) / kPartChildren;
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t* base = scratch + (size_t)p0 * kPartPlanes * a.wpad + word;
    uint32_t finite = 0;
    for (int32_t p = 0; p < np; ++p) finite |= base[((size_t)p * kPartPlanes + 128) * a.wpad];
    uint32_t M[BW], z0[16], z1[16];
#pragma unroll
    for (int b = 0; b < BW; ++b) M[b] = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) z0[v] = z1[v] = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        uint32_t acc[BW];
#pragma unroll
        for (int b = 0; b < BW; ++b) acc[b] = 0;
        for (int32_t p = 0; p < np; ++p) {
            const uint32_t* q = base + ((size_t)p * kPartPlanes + v * 8) * a.wpad;
            uint32_t x[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) x[b] = q[(size_t)b * a.wpad];
            uint32_t carry = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t s = acc[b] ^ x[b] ^ carry;
                carry = (acc[b] & x[b]) | (carry & (acc[b] ^ x[b]));
                acc[b] = s;
            }
#pragma unroll
            for (int b = 8; b < BW; ++b) {
                const uint32_t s = acc[b] ^ carry;
                carry &= acc[b];
                acc[b] = s;
            }
        }
        // compare the code's count c with the running maximum M: c > M, c == M, c == M + 1,
        // and c == M - 1 (as c + 1 == M)
        uint32_t gt = 0, eqs = ~0u, cy_m = ~0u, cy_c = ~0u, eqp1 = ~0u, eqm1 = ~0u;
#pragma unroll
        for (int b = BW - 1; b >= 0; --b) {
            gt |= eqs & acc[b] & ~M[b];
            eqs &= ~(acc[b] ^ M[b]);
        }
#pragma unroll
        for (int b = 0; b < BW; ++b) {
            const uint32_t mp1 = M[b] ^ cy_m, cp1 = acc[b] ^ cy_c;
            cy_m &= M[b];
            cy_c &= acc[b];
            eqp1 &= ~(acc[b] ^ mp1);
            eqm1 &= ~(cp1 ^ M[b]);
        }
        // new maximum: Z1 = the old Z0 if it is one below, else empty; Z0 = {v}.
        // equal: v joins Z0; one below: v joins Z1
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t nz1 = bsel(gt, eqp1 & z0[u], z1[u] | (u == v ? eqm1 : 0u));
            z0[u] = bsel(gt, u == v ? ~0u : 0u, z0[u] | (u == v ? eqs : 0u));
            z1[u] = nz1;
        }
#pragma unroll
        for (int b = 0; b < BW; ++b) M[b] = bsel(gt, acc[b], M[b]);
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        z0[v] &= finite;
        z1[v] &= finite;
    }
    uint64_t rx, rs, rd;
    store_sankoff(a.sets, a.cmask, a.cons, n, a.tiles, tile, lane, word, z0, z1, true, rx, rs, rd);
    if (a.upm != nullptr) push_up_slot(a, a.pslot[(int32_t)(a.desc - a.desc_all) + item], tile, lane, rx, rs);
    push_children(a, tile, lane, e0, e1, d.c0, d.c1, rx, rs);
}

}  // namespace

hipError_t launch_sankoff(pm_ctx* c, bool block) {
    const HostTree& ht = c->ht;
    const DevTree& dt = c->dt;
    const int32_t tiles = (c->words + kWave - 1) / kWave;
    const int64_t wpad = (int64_t)tiles * kWave;

    // nucleotide Sankoff evaluates leaf-parents of one or two leaves inline, like Fitch, and
    // with every leaf present the S2 / S3 subtrees too (subtree form: their Z0 in the parent's
    // post-order wave, their finals and records in the tail)
    const bool virt = !block && c->virtual_leaf_parents;
    const bool sub = virt && c->subtree_form && c->leaves_all_present && ht.num_sshape > 0;
    const bool grp = sub && c->up_group;   // grouped post-order launches (PM_OPT_UP_GROUP)
    const int form = sub ? 2 : virt ? 1 : 0;
    const int32_t* child_enc = sub ? dt.child_enc_k : virt ? dt.child_enc_v : dt.child_enc;
    const NodeDesc* up_desc = grp ? dt.up_desc_gs : sub ? dt.up_desc_k : virt ? dt.up_desc_v : dt.up_desc;
    const NodeDesc* down_desc = sub ? dt.down_desc_k : virt ? dt.down_desc_v : dt.down_desc;
    const std::vector<int32_t>& class_off = grp ? ht.up_class_off_gs : sub ? ht.up_class_off_k
                                          : virt ? ht.up_class_off_v : ht.up_class_off;
    const std::vector<int32_t>& part_off = grp ? ht.part_off_gs : sub ? ht.part_off_k : virt ? ht.part_off_v : ht.part_off;
    const PartDesc* parts = grp ? dt.part_desc_gs : sub ? dt.part_desc_k : virt ? dt.part_desc_v : dt.part_desc;
    const std::vector<int32_t>& down_off = sub ? ht.down_level_off_k : virt ? ht.down_level_off_v : ht.down_level_off;
    UpArgs up{};
    up.child_off = dt.child_off;
    up.child_enc = child_enc;
    up.vleaf = reinterpret_cast<const int4*>(dt.vleaf);
    up.leaf_flag = c->leaf_flag;
    up.leaf_planes = c->leaf_planes;
    up.leaf_present = c->leaf_present;
    up.sets = reinterpret_cast<uint4*>(c->sets);
    up.cmask = c->cmask;
    up.cons = c->cons;
    up.forced = nullptr;   // Sankoff forces the root in the backward pass only
    up.absent_code0 = block;
    up.all_present = c->leaves_all_present;
    up.root_dense = dt.root_dense;
    up.tiles = tiles;
    up.wpad = wpad;
    up.desc_all = up_desc;   // grouped launches: pad0 / pad1 index the whole array
    // up slots: the subtree form's kernels (alloc_work sizes them for its up orders)
    if (sub && c->upm == nullptr) return hipErrorInvalidValue;
    up.upm = sub ? c->upm : nullptr;
    up.pslot = grp ? dt.pslot_gs : dt.pslot_k;
    // LDS-staged sweeps over every height (k_sankoff_up_cluster) when the plan covers the whole
    // post-order and no swept node has more than 255 children; the level kernels otherwise
    const ClusterPlan& clp = ht.cl;
    const bool sk_clu = sub && c->cluster && clp.band_wg.size() > 1 && clp.h0 == 0 && clp.max_degree <= 255;
    const int H = sk_clu ? 0 : (int)(grp ? ht.up_level_off_gs : sub ? ht.up_level_off_k : virt ? ht.up_level_off_v : ht.up_level_off).size() - 1;
    if (sk_clu) {
        const ClArgs ca0{dt.cl_items, dt.cl_wg_off, dt.cl_slot_of, dt.cl_pslot, clp.upm_base, 0};
        for (size_t bnd = 0; bnd + 1 < clp.band_wg.size(); ++bnd) {
            ClArgs ca = ca0;
            ca.wg0 = clp.band_wg[bnd];
            const int64_t nwg = clp.band_wg[bnd + 1] - ca.wg0;
            if (nwg == 0) continue;
            timer_begin(c, 0);
            hipLaunchKernelGGL(k_sankoff_up_cluster, dim3((unsigned)(nwg * tiles)), dim3(kWave), 0, c->stream, up, ca);
            timer_end(c, 0);
        }
    }
    // nodes [b, e) of one level with more than 255 children: parts, then the merge
    auto launch_parts = [&](int32_t b, int32_t e, hipStream_t s) {
        const int32_t p0 = part_off[b], np = part_off[e] - p0;
        int32_t widest = 0;
        for (int32_t i = b; i < e; ++i) widest = std::max(widest, ht.up_degree[grp ? 3 : form][i]);
        UpArgs pa = up;
        pa.desc = up_desc;   // parts name their node by its global up-order position
        UpArgs mg = up;
        mg.desc = up_desc + b;
        mg.count = e - b;
        const dim3 grid = wave_grid(mg.count, tiles);
        timer_begin(c, 0);
        hipLaunchKernelGGL(k_sankoff_part, wave_grid(np, tiles), dim3(kBlock), 0, s, pa, parts + p0, np, c->sk_parts);
        if (widest < (1 << 16)) hipLaunchKernelGGL(k_sankoff_merge<16>, grid, dim3(kBlock), 0, s, mg, c->sk_parts);
        else hipLaunchKernelGGL(k_sankoff_merge<32>, grid, dim3(kBlock), 0, s, mg, c->sk_parts);
        timer_end(c, 0);
    };
    // runs of >= 2 narrow levels with only out-degree <= 3 nodes (PM_OPT_NARROW): one band each
    auto narrow_up = [&](int h) {
        const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1],
                      e = class_off[(h + 1) * kDegreeClasses];
        return e == m && m - b <= c->narrow_max;
    };
    for (int h = 0; h < H; ++h) {
        if (c->narrow_max > 0 && narrow_up(h)) {
            int h1 = h + 1;
            while (h1 < H && narrow_up(h1)) ++h1;
            if (h1 - h >= 2) {
                up.desc = up_desc;
                const int32_t* tab = dt.lvl + ht.lvl_up[grp ? 4 : form];
                timer_begin(c, 0);
                if (grp) hipLaunchKernelGGL((k_sankoff_up_band<true, true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else if (sub) hipLaunchKernelGGL((k_sankoff_up_band<true, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else if (c->leaves_all_present) hipLaunchKernelGGL((k_sankoff_up_band<true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                else hipLaunchKernelGGL((k_sankoff_up_band<false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, up, tab, h, h1);
                timer_end(c, 0);
                h = h1 - 1;
                continue;
            }
        }
        {   // a small level with narrow and wide (<= 255 children) nodes: one launch
            const int32_t b = class_off[h * kDegreeClasses], m = class_off[h * kDegreeClasses + 1],
                          w4 = class_off[h * kDegreeClasses + 2], w8 = class_off[h * kDegreeClasses + 3];
            if (m > b && w8 > m && (int64_t)(m - b) * tiles <= kMixedMaxWaves) {
                up.desc = up_desc + b;
                up.count = m - b;
                const int32_t nb = (int32_t)wave_grid(up.count, tiles).x;
                const dim3 grid((unsigned)(nb + (int64_t)(w8 - m) * tiles));
                timer_begin(c, 0);
                if (w8 > w4 && grp) hipLaunchKernelGGL((k_sankoff_up_mixed<8, true, true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (grp) hipLaunchKernelGGL((k_sankoff_up_mixed<4, true, true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (w8 > w4 && sub) hipLaunchKernelGGL((k_sankoff_up_mixed<8, true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (sub) hipLaunchKernelGGL((k_sankoff_up_mixed<4, true, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (w8 > w4 && c->leaves_all_present) hipLaunchKernelGGL((k_sankoff_up_mixed<8, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (w8 > w4) hipLaunchKernelGGL((k_sankoff_up_mixed<8, false>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else if (c->leaves_all_present) hipLaunchKernelGGL((k_sankoff_up_mixed<4, true>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                else hipLaunchKernelGGL((k_sankoff_up_mixed<4, false>), grid, dim3(kBlock), 0, c->stream, up, up_desc + m, nb);
                timer_end(c, 0);
                // the level's nodes above 255 children (if any) still go to the parts below
                for (int k = 3; k < kDegreeClasses; ++k) {
                    const int32_t pb = class_off[h * kDegreeClasses + k], pe = class_off[h * kDegreeClasses + k + 1];
                    if (pe > pb) launch_parts(pb, pe, c->stream);
                }
                continue;
            }
        }
        // the level's degree classes are independent: the wide ones run on the side stream,
        // beside the narrow launch (parallel graph branches), when both kinds are present
        const int32_t lb = class_off[h * kDegreeClasses], lm = class_off[h * kDegreeClasses + 1],
                      le = class_off[(h + 1) * kDegreeClasses];
        const bool fork = lm > lb && le > lm;
        if (fork) {
            const hipError_t fe = side_fork(c);
            if (fe != hipSuccess) return fe;
        }
        for (int k = kDegreeClasses - 1; k >= 0; --k) {   // wide classes first: they go to the side
            const int32_t b = class_off[h * kDegreeClasses + k];
            const int32_t e = class_off[h * kDegreeClasses + k + 1];
            if (e == b) continue;
            hipStream_t s = fork && k > 0 ? c->side : c->stream;
            // the grouped order's plain prefix of the narrow class: the lean kernel first
            int32_t np = k == 0 && grp && c->plain_up ? std::min(ht.up_plain_gs[h], e - b) : 0;
            if ((int64_t)np * tiles < (c->plain_min_waves > 0 ? c->plain_min_waves : kPlainMinWaves)) np = 0;
            if (np > 0) {
                up.desc = up_desc + b;
                up.count = np;
                timer_begin(c, 0);
                hipLaunchKernelGGL((k_sankoff_up<2, true, true, false, true>), wave_grid(np, tiles), dim3(kBlock), 0, s, up);
                timer_end(c, 0);
                if (np == e - b) continue;
            }
            up.desc = up_desc + b + np;
            up.count = e - b - np;
            const dim3 grid = wave_grid(up.count, tiles), wide = block_grid(up.count, tiles);
            timer_begin(c, 0);
            if (k == 0 && grp && ht.up_recomp_gs[h]) hipLaunchKernelGGL((k_sankoff_up<2, true, true, true>), grid, dim3(kBlock), 0, s, up);
            else if (k == 0 && sub) hipLaunchKernelGGL((k_sankoff_up<2, true, true>), grid, dim3(kBlock), 0, s, up);
            else if (k == 0 && c->leaves_all_present) hipLaunchKernelGGL((k_sankoff_up<2, true>), grid, dim3(kBlock), 0, s, up);
            else if (k == 0) hipLaunchKernelGGL((k_sankoff_up<2, false>), grid, dim3(kBlock), 0, s, up);
            else if (k == 1) hipLaunchKernelGGL(k_sankoff_up_wide<4>, wide, dim3(kBlock), 0, s, up);
            else if (k == 2) hipLaunchKernelGGL(k_sankoff_up_wide<8>, wide, dim3(kBlock), 0, s, up);
            else {   // more than 255 children: parts, then the merge
                timer_end(c, 0);
                launch_parts(b, e, s);
                continue;
            }
            timer_end(c, 0);
        }
        if (fork) {
            const hipError_t je = side_join(c);
            if (je != hipSuccess) return je;
        }
    }

    hipError_t err = hipMemsetAsync(c->shard_cnt, 0, sizeof(uint32_t) * kShards, c->stream);
    if (err != hipSuccess) return err;
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
    dn.forced = c->has_forced ? c->forced : nullptr;
    dn.absent_code0 = block;
    dn.all_present = c->leaves_all_present;
    dn.vleaf = reinterpret_cast<const int4*>(dt.vleaf);
    dn.vinner = dt.vinner;
    // pre-order sweeps over the planner's clusters (PM_OPT_CLUSTER, every level swept: the
    // same schedule as the Fitch pre-order's, k_down_cluster<Sankoff>), the bands top-down
    const ClusterPlan& cl = ht.cl;
    const bool cld = sub && c->cluster && cl.band_wg.size() > 1 && cl.down;
    if (cld) {
        for (size_t bnd = cl.band_wg.size() - 1; bnd-- > 0;) {
            const ClDownArgs ca{dt.cl_down_items, dt.cl_wg_off, cl.band_wg[bnd]};
            const int64_t nwg = cl.band_wg[bnd + 1] - ca.wg0;
            if (nwg == 0) continue;
            timer_begin(c, 1);
            hipLaunchKernelGGL(k_down_cluster<Mode::kSankoff>, dim3((unsigned)(nwg * tiles)), dim3(kWave), 0, c->stream, dn, ca);
            timer_end(c, 1);
        }
    }
    const int D = cld ? 0 : (int)down_off.size() - 1;
    // a pre-order level = one range of dense indices: [down_off[d], down_off[d+1]) in the
    // leaf-parent form, from down_dense_base_k[d] in the subtree form
    const bool dense_all = sub ? ht.down_dense_k : virt && ht.down_dense_v;
    auto dense_base_of = [&](int l) { return !dense_all ? -1 : sub ? ht.down_dense_base_k[l] : down_off[l]; };
    for (int d = 0; d < D; ++d) {
        if (c->narrow_max > 0 && down_off[d + 1] - down_off[d] <= c->narrow_max) {   // PM_OPT_NARROW
            int d1 = d + 1;
            while (d1 < D && down_off[d1 + 1] - down_off[d1] <= c->narrow_max) ++d1;
            if (d1 - d >= 2) {
                dn.desc = down_desc;
                const int32_t* tab = dt.lvl + ht.lvl_down[form];
                const int32_t* base = !dense_all ? nullptr : sub ? dt.lvl + ht.lvl_base_k : tab;
                timer_begin(c, 1);
                const bool grp = c->group_waves > 0;   // level groups inside the band
                if (c->leaves_all_present && grp) hipLaunchKernelGGL((k_down_band<Mode::kSankoff, true, false, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (c->leaves_all_present) hipLaunchKernelGGL((k_down_band<Mode::kSankoff, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else if (grp) hipLaunchKernelGGL((k_down_band<Mode::kSankoff, false, false, true>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                else hipLaunchKernelGGL((k_down_band<Mode::kSankoff, false>), dim3(tiles), dim3(kBandBlock), 0, c->stream, dn, tab, base, d, d1);
                timer_end(c, 1);
                d = d1 - 1;
                continue;
            }
        }
        dn.desc = down_desc + down_off[d];
        dn.count = down_off[d + 1] - down_off[d];
        if (dn.count == 0) continue;
        const bool dense = dense_all;
        dn.dense_base = dense_base_of(d);
        // levels d .. d + g - 1 in one launch (PM_OPT_GROUP_*; see launch_fitch)
        auto narrow_down = [&](int l) { return c->narrow_max > 0 && down_off[l + 1] - down_off[l] <= c->narrow_max; };
        auto band_at = [&](int l) { return narrow_down(l) && l + 1 < D && narrow_down(l + 1); };
        int g = 1;
        int64_t items = dn.count;
        while (c->group_waves > 0 && g < std::min(c->group_levels, kGroupLevels) && d + g < D) {
            const int32_t ng = down_off[d + g + 1] - down_off[d + g];
            if (ng == 0 || (items + ng) * tiles > c->group_waves || band_at(d + g)) break;
            items += ng;
            ++g;
        }
        if (g > 1) {
            for (int k = 0; k < 4; ++k) {
                const int l = std::min(d + k, d + g - 1);
                if (k > 0) dn.split[k - 1] = k < g ? down_off[d + k] - down_off[d] : (int32_t)items;
                dn.dense_g[k] = dense_base_of(l);
            }
            dn.count = (int32_t)items;
            const dim3 grid = wave_grid(dn.count, tiles);
            timer_begin(c, 1);
            if (c->leaves_all_present && dense) hipLaunchKernelGGL((k_down<Mode::kSankoff, true, true, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else if (c->leaves_all_present) hipLaunchKernelGGL((k_down<Mode::kSankoff, true, false, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            else hipLaunchKernelGGL((k_down<Mode::kSankoff, false, false, false, true>), grid, dim3(kBlock), 0, c->stream, dn);
            timer_end(c, 1);
            d += g - 1;
            continue;
        }
        const dim3 grid = wave_grid(dn.count, tiles);
        timer_begin(c, 1);
        if (c->leaves_all_present && dense) hipLaunchKernelGGL((k_down<Mode::kSankoff, true, true>), grid, dim3(kBlock), 0, c->stream, dn);
        else if (c->leaves_all_present) hipLaunchKernelGGL((k_down<Mode::kSankoff, true, false>), grid, dim3(kBlock), 0, c->stream, dn);
        else hipLaunchKernelGGL((k_down<Mode::kSankoff, false, false>), grid, dim3(kBlock), 0, c->stream, dn);
        timer_end(c, 1);
    }
    // children beyond a node's second: one flat launch after the levels (k_tail)
    const int32_t tail_total = sub ? ht.num_tail_k : virt ? ht.num_tail_v : ht.num_tail;
    if (tail_total > 0) {
        DownArgs t = dn;
        t.tail = sub ? dt.tail_desc_k : virt ? dt.tail_desc_v : dt.tail_desc;
        t.count = tail_total;
        t.num_s = sub ? ht.num_tail_s : 0;
        t.sbase = ht.sbase;
        t.sub_planes = c->sub_planes;
        const dim3 grid = wave_grid(t.count, tiles);
        timer_begin(c, 5);
        if (sub) hipLaunchKernelGGL((k_tail<Mode::kSankoff, true, true>), grid, dim3(kBlock), 0, c->stream, t);
        else if (c->leaves_all_present) hipLaunchKernelGGL((k_tail<Mode::kSankoff, true>), grid, dim3(kBlock), 0, c->stream, t);
        else hipLaunchKernelGGL((k_tail<Mode::kSankoff, false>), grid, dim3(kBlock), 0, c->stream, t);
        timer_end(c, 5);
    }
    return hipGetLastError();
}

// This file's code object, loaded ahead of its first launch (pm_warmup).
hipError_t warm_sankoff() {
    hipFuncAttributes at;
    return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_sankoff_up_wide<4>));
}

}  // namespace pm
