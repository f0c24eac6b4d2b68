// pm_kernels.h -- device pieces shared by the Fitch and Sankoff passes.
//
// State-set records: one (node, 64-word tile) record holds Q quads x 64 lanes of uint4
// (Q = 4 for Fitch's 16 one-hot planes, Q = 8 for Sankoff's Z0 + Z1 planes), so every
// wave-instruction moves a contiguous 1 KiB.
#pragma once

#include "pm_bits.h"
#include "pm_internal.h"

// Set-record load policy of this translation unit: pm_fitch.hip / pm_sankoff.hip build the
// kernels with ordinary loads, pm_fitch_nt.hip / pm_sankoff_nt.hip with non-temporal ones
// (PM_NT_LOADS), each copy in a namespace of its own; launch_all picks one per run (nt_policy).
#ifndef PM_NT_LOADS
#define PM_NT_LOADS 0
#endif
#if PM_NT_LOADS
#define PM_KNS kern_nt
#else
#define PM_KNS kern
#endif

namespace pm {
inline namespace PM_KNS {

enum class Mode { kFitch, kSankoff, kBlockFitch };

// Level launches number their (item, tile) waves tile-fastest: the tiles of one node run
// side by side, so its leaf rows, records and parent's records -- contiguous per node --
// stream as whole rows (DRAM pages, TLB entries) instead of 1-KiB pieces of thousands of
// rows.  One-wave kernels: wave g = (item g / tiles, tile g % tiles); one-workgroup
// kernels: workgroup b likewise.  (PM_TILE_FAST=0: the former 2-D grid, tile = blockIdx.y.)
#ifndef PM_TILE_FAST
#define PM_TILE_FAST 1
#endif
__device__ __forceinline__ void wave_item(int wave, int32_t tiles, int32_t& item, int& tile) {
#if PM_TILE_FAST
    const int32_t g = (int32_t)blockIdx.x * kWavesPerBlock + wave;
    item = g / tiles;
    tile = g - item * tiles;
#else
    item = (int32_t)blockIdx.x * kWavesPerBlock + wave;
    tile = blockIdx.y;
#endif
}

__device__ __forceinline__ void block_item(int32_t tiles, int32_t& item, int& tile) {
#if PM_TILE_FAST
    item = (int32_t)blockIdx.x / tiles;
    tile = (int32_t)blockIdx.x - item * tiles;
#else
    item = blockIdx.x;
    tile = blockIdx.y;
#endif
}

// Grids of the level launches (count items x tiles; memory bounds count * tiles far below 2^31).
inline dim3 wave_grid(int32_t count, int32_t tiles) {
#if PM_TILE_FAST
    return dim3((unsigned)(((int64_t)count * tiles + kWavesPerBlock - 1) / kWavesPerBlock));
#else
    return dim3((count + kWavesPerBlock - 1) / kWavesPerBlock, tiles);
#endif
}
inline dim3 block_grid(int32_t count, int32_t tiles) {
#if PM_TILE_FAST
    return dim3((unsigned)((int64_t)count * tiles));
#else
    return dim3(count, tiles);
#endif
}

// Levels holding nodes of both out-degree classes go to one mixed launch when the narrow
// part is at most this many waves (the mixed kernel runs at the wide kernel's occupancy).
#ifndef PM_MIXED_MAX_WAVES
#define PM_MIXED_MAX_WAVES 4096
#endif
constexpr int64_t kMixedMaxWaves = PM_MIXED_MAX_WAVES;
// Narrow-level band launches (PM_OPT_NARROW): one workgroup of 16 waves per tile.
#ifndef PM_BAND_WAVES
#define PM_BAND_WAVES 16
#endif
constexpr int kBandWaves = PM_BAND_WAVES;
// Plain post-order prefixes (PM_OPT_PLAIN_UP) get a launch of their own only from this many
// (node, tile) waves: the lean kernel's higher occupancy pays on levels that fill the chip
// many times over, a second dependent launch costs more on smaller ones (C3 with a split at
// every level: +0.2 ms).
#ifndef PM_PLAIN_MIN_WAVES
#define PM_PLAIN_MIN_WAVES 65536
#endif
constexpr int64_t kPlainMinWaves = PM_PLAIN_MIN_WAVES;
constexpr int kBandBlock = kBandWaves * kWave;

struct UpArgs {
    const int32_t* order;  // Sankoff: level items
    const NodeDesc* desc;  // level items
    const NodeDesc* desc_all;  // grouped post-order launches: the whole descriptor array (pad0 / pad1 index it)
    const int4* vleaf;     // virtual node -> its (one or two) leaves, -1 padded
    int32_t count;
    const int32_t* child_off;
    const int32_t* child_enc;
    const uint8_t* leaf_flag;
    const uint4* leaf_planes;
    const uint32_t* leaf_present;
    uint4* sets;
    uint64_t* cmask;       // record class masks, 2 per (node, tile) (see rec_store_head)
    const uint4* cons;     // consensus codes (the "consensus" record class)
    const uint4* forced;   // nullable
    int32_t root_dense;
    int32_t tiles;
    int64_t wpad;
    bool absent_code0;     // block Sankoff: a leaf missing from the column is state 0
    bool all_present;      // every leaf present at every site (dirty-lane rules)
    // Up slots (Fitch subtree form; null otherwise): per (descriptor item, tile) the (x, s)
    // masks of the item's first two children, {c0.x, c0.s, c1.x, c1.s}, written by each child's
    // own post-order wave (pslot[item] = parent item * 2 + slot, or -1).  A node's wave loads
    // them beside its descriptor -- both addressed by its item index alone -- so its children's
    // record loads wait for one round trip instead of two (descriptor, then the children's
    // mask records).
    uint64_t* upm;
    const int32_t* pslot;
};

struct UpSlots {
    uint64_t x0, s0, x1, s1;
};

// Item gi's up slots, loaded from nothing but gi (no dependence on its descriptor).
__device__ __forceinline__ UpSlots load_up_slots(const UpArgs& a, int32_t gi, int tile) {
    const uint64_t* q = a.upm + ((size_t)gi * a.tiles + tile) * 4;
    return UpSlots{q[0], q[1], q[2], q[3]};
}

// A node's (x, s) masks into its parent's slot (lane 0; ps = pslot[gi], loaded early).
__device__ __forceinline__ void push_up_slot(const UpArgs& a, int32_t ps, int tile, int lane, uint64_t mx, uint64_t ms) {
    if (ps >= 0 && lane == 0) {
        uint64_t* q = a.upm + ((size_t)(ps >> 1) * a.tiles + tile) * 4 + (ps & 1) * 2;
        q[0] = mx;
        q[1] = ms;
    }
}

// The leaf words of S2 / S3 node `item` (dense index sbase + item) at one word: vl[0..3]'s
// words in four consecutive uint4 (pm_ctx::sub_planes).
__device__ __forceinline__ const uint4* sub_word(const uint4* sub_planes, int32_t item, int64_t wpad, int64_t word) {
    return sub_planes + ((size_t)item * wpad + word) * 4;
}

// Load 16 planes (quads q0..q0+3) of a record of Q quads.
template <int Q = 4>
__device__ __forceinline__ void load_set16(const uint4* sets, int64_t node, int32_t tiles, int tile,
                                           int lane, uint32_t* s, int q0 = 0) {
    const uint4* p = sets + ((size_t)node * tiles + tile) * (Q * 64) + q0 * 64 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = p[q * 64];
        s[4 * q + 0] = v.x;
        s[4 * q + 1] = v.y;
        s[4 * q + 2] = v.z;
        s[4 * q + 3] = v.w;
    }
}

template <int Q = 4>
__device__ __forceinline__ void store_set16(uint4* sets, int64_t node, int32_t tiles, int tile,
                                            int lane, const uint32_t* s, int q0 = 0) {
    uint4* p = sets + ((size_t)node * tiles + tile) * (Q * 64) + q0 * 64 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q * 64] = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}

// Set records, compressed.  Per (node, 64-word tile) a word is one of three classes:
//   consensus -- every site a single code equal to the block consensus: nothing stored;
//   simple    -- every site a single code: 4 code planes (16 B), packed by rank among the
//                simple lanes at the front of the record;
//   complex   -- an empty or multi-code set somewhere: the full planes (Fitch: 16 one-hot
//                planes; Sankoff: Z0 and Z1), packed by rank among the complex lanes,
//                quad-major so each quad of the complex lanes is one contiguous run.
// Two u64 ballots per (node, tile) mark the complex and simple lanes (mbcnt gives a lane
// its rank).  Traffic per record: 16 B per simple and 64 / 128 B per complex word
// instead of 64 / 128 B for every word.  (At N*, 93 % of Fitch words are single-code.)
// Fitch, compact complex lanes (kCxCompact): a complex word is its code planes A (area 1; a
// multi-code site's bits there are unused) and B = {M, s0|s1<<16, s2|s3<<16, s4|s5<<16}
// (area 2): M marks its multi-code (or empty) sites, s_i is the 16-bit set of M's i-th site.
// A word with more than kCxSets such sites is "full": B.x = kCxFull, its 16 planes in areas
// 1, 3, 4, 5.  32 B per complex word instead of 64; the reader loads A in place of the code
// word it loads anyway, plus B, and patches the one-hot expansion of A at M's sites.
constexpr int kFitchRec = kFitchRecQuads * kWave;   // uint4 per (node, tile)
constexpr int kCxSets = 6;
constexpr uint32_t kCxFull = ~0u;
constexpr int kSankoffRec = 9 * kWave;   // uint4 per (node, tile)

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint4 load_stream(const uint4* p) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Set records are read once, by the next wave that needs them.  With levels of many waves
// the lines are gone from L2 / MALL before anything reads them again, and non-temporal loads
// keep them from displacing what is reused (N* Fitch 14.7 -> 14.06 ms, Sankoff 20.2 -> 19.7
// ms); with small levels (a deep tree's) the next level finds the records it reads in cache,
// and non-temporal loads cost C3 Fitch 0.12 ms, Sankoff 0.4 ms.  A branch per load on the
// launch's size made every kernel slower (N* 16.7 ms), so the policy is per translation unit.
__device__ __forceinline__ uint4 load_rec(const uint4* p) {
#if PM_NT_LOADS
    return load_stream(p);
#else
    return *p;
#endif
}

struct RecMask {
    uint64_t x, s, d;   // complex lanes, simple (non-consensus) lanes, dirty lanes (below)
    uint64_t px, ps;    // the parent's x and s, pushed by the parent's post-order wave
};

__device__ __forceinline__ RecMask rec_mask(const uint64_t* cm, size_t rec) {
    const uint64_t* q = cm + kMaskWords * rec;
    return RecMask{q[0], q[1], q[2], q[3], q[4]};
}

// A node's post-order wave copies its x / s masks into each materialised child's mask
// record (words 3, 4), so the child's pre-order wave finds its parent's final (compact
// finals, see node_final) from its own masks -- loaded with its descriptor -- instead of
// loading the parent's masks after the descriptor.
__device__ __forceinline__ void push_masks(uint64_t* cm, int32_t tiles, int tile, int32_t child, uint64_t mx, uint64_t ms) {
    uint64_t* q = cm + kMaskWords * ((size_t)child * tiles + tile);
    q[3] = mx;
    q[4] = ms;
}

// push_masks for every materialised child of the node with children [e0, e1) (child
// encodings as in UpArgs::child_enc; the first two also in c0, c1); lanes share the list.
// An S2 / S3 child (subtree form) gets the node's dirty lanes too (word 5; every lane at the
// root): its tail wave reads the three from its own, never otherwise used, mask record --
// addressed by its item index alone -- instead of the parent's behind its descriptor.
__device__ __forceinline__ bool materialised(int32_t c) { return c >= 0 && !(c & kVirtualBit); }

__device__ __forceinline__ void push_sub(uint64_t* cm, int32_t tiles, int tile, int32_t c, uint64_t mx, uint64_t ms,
                                         uint64_t md) {
    uint64_t* q = cm + kMaskWords * ((size_t)(c & kDenseMask) * tiles + tile);
    q[3] = mx;
    q[4] = ms;
    q[5] = md;
}

__device__ __forceinline__ bool sub_shaped(int32_t c) { return c >= 0 && (c & kVirtualBit) && ((c >> kShapeShift) & 3); }

// md0 / md1: the lanes an S2 / S3 first / second child's tail wave must read (Fitch: the
// node's complex lanes plus that child's own disagreeing-leaf lanes, see fitch_up_node;
// otherwise the node's dirty lanes).
__device__ __forceinline__ void push_children2(const UpArgs& a, int tile, int lane, int32_t e0, int32_t e1, int32_t c0,
                                               int32_t c1, uint64_t mx, uint64_t ms, uint64_t md0, uint64_t md1, bool root) {
    if (lane == 0) {
        if (materialised(c0)) push_masks(a.cmask, a.tiles, tile, c0, mx, ms);
        if (e1 - e0 > 1 && materialised(c1)) push_masks(a.cmask, a.tiles, tile, c1, mx, ms);
        if (sub_shaped(c0)) push_sub(a.cmask, a.tiles, tile, c0, mx, ms, root ? ~0ull : md0);
        if (e1 - e0 > 1 && sub_shaped(c1)) push_sub(a.cmask, a.tiles, tile, c1, mx, ms, root ? ~0ull : md1);
    }
    for (int32_t e = e0 + 2 + lane; e < e1; e += kWave) {
        const int32_t c = a.child_enc[e];
        if (materialised(c)) push_masks(a.cmask, a.tiles, tile, c, mx, ms);
    }
}

__device__ __forceinline__ void push_children(const UpArgs& a, int tile, int lane, int32_t e0, int32_t e1, int32_t c0,
                                              int32_t c1, uint64_t mx, uint64_t ms, uint64_t md = 0, bool root = false) {
    push_children2(a, tile, lane, e0, e1, c0, c1, mx, ms, md, md, root);
}

// Fitch records: the lanes the pre-order pass must read the first / second child's leaves
// at (words 6, 7; fitch_up_node), a subset of d.
__device__ __forceinline__ void store_kid_masks(uint64_t* cm, size_t rec, int lane, uint64_t k0, uint64_t k1) {
    if (lane == 0) {
        cm[kMaskWords * rec + 6] = k0;
        cm[kMaskWords * rec + 7] = k1;
    }
}

// Code planes of a non-complex lane: stored (simple) or the consensus word.
__device__ __forceinline__ uint4 rec_code(const uint4* p, const RecMask& m, int lane, const uint4* cons, int64_t word) {
    if ((m.s >> lane) & 1ull) return load_rec(p + lanes_below(m.s));
    return cons[word];
}

// Classify a word from its single-code test and code planes, write code / masks.
// Dirty lanes (d): the lanes whose leaf / leaf-parent children the pre-order pass must
// read -- complex lanes plus every lane the caller flags (`dirty_extra`).  Elsewhere each
// site's set is one code c reached by the AND of every child's set, so each leaf child
// holds c, the node's final is c (src/fitchSankoff.cpp:115-123) and no child record exists.
__device__ __forceinline__ void rec_store_head(uint4* p, uint64_t* cm, size_t rec, int lane, bool complex_word,
                                               bool dirty_extra, const uint32_t* code, const uint4& cw, uint64_t& mx,
                                               uint64_t& ms, uint64_t& md) {
    const bool same = !complex_word && code[0] == cw.x && code[1] == cw.y && code[2] == cw.z && code[3] == cw.w;
    mx = __ballot(complex_word);
    ms = __ballot(!complex_word && !same);
    md = __ballot(complex_word || dirty_extra);
    if (!complex_word && !same) store_stream(p + lanes_below(ms), make_uint4(code[0], code[1], code[2], code[3]));
    if (lane == 0) {
        cm[kMaskWords * rec] = mx;
        cm[kMaskWords * rec + 1] = ms;
        cm[kMaskWords * rec + 2] = md;
    }
}

// Code planes of any lane of a record (complex lanes: unused), one load from a per-lane
// address: the stored word of a simple lane or the consensus word (see kid_fetch on why
// loads are not selected between branches).  CX (compact Fitch records): a complex lane's A.
template <bool CX = false>
__device__ __forceinline__ uint4 rec_code_all(const uint4* p, const RecMask& m, int lane, const uint4* cons,
                                              int64_t word) {
    const uint4* src = ((m.s >> lane) & 1ull) ? p + lanes_below(m.s) : cons + word;
    if (CX && ((m.x >> lane) & 1ull)) src = p + kWave + lanes_below(m.x);
    return load_rec(src);
}

// A compact record's B word (area 2) for every lane: complex lanes their own, the others the
// first complex lane's (unused) -- or, no complex lane at all, a consensus word (see cx_base).
__device__ __forceinline__ uint4 cx_b_load(const uint4* p, const RecMask& m, int lane, const uint4* cons) {
    const bool cx = (m.x >> lane) & 1ull;
    return load_rec((m.x ? p + 2 * kWave : cons + kWave) + (cx ? lanes_below(m.x) : 0u));
}

// Compact complex lanes: x = the one-hot expansion of the lane's A (every lane: its code's);
// at a complex lane (cx) clear M's sites and set each one's 16-bit set from B.  A full lane
// (B.x == kCxFull) takes A as planes 0-3 and loads planes 4-15 from areas 3-5 of record p
// (mx: its complex lanes) -- a second round trip, taken only by a wave holding such a lane.
// Wave-uniform trip count: the most multi-code sites any lane of the wave has.
__device__ __forceinline__ void cx_decode(uint32_t* x, const uint4& A, const uint4& B, bool cx, const uint4* p, uint64_t mx) {
    const uint32_t M = cx ? B.x : 0u;
    if (__ballot(M != 0u) == 0) return;
    const bool full = M == kCxFull;
    uint32_t rem = full ? 0u : M;
#pragma unroll
    for (int v = 0; v < 16; ++v) x[v] &= ~rem;
    const uint32_t w[3] = {B.y, B.z, B.w};
#pragma unroll
    for (int i = 0; i < kCxSets; ++i) {
        if (__ballot(rem != 0u) == 0) break;
        const uint32_t bit = rem & (0u - rem);   // M's i-th site (0 once the lane has none left)
        const uint32_t set = w[i >> 1] >> (16 * (i & 1));
#pragma unroll
        for (int v = 0; v < 16; ++v) x[v] |= bit & (uint32_t)((int32_t)(set << (31 - v)) >> 31);
        rem &= rem - 1u;
    }
    if (__ballot(full) != 0) {
        if (full) {
            const uint4* q = p + kWave + lanes_below(mx);
            x[0] = A.x; x[1] = A.y; x[2] = A.z; x[3] = A.w;
#pragma unroll
            for (int j = 1; j < 4; ++j) {
                const uint4 t = load_rec(q + (j + 1) * kWave);
                x[4 * j] = t.x; x[4 * j + 1] = t.y; x[4 * j + 2] = t.z; x[4 * j + 3] = t.w;
            }
        }
    }
}

// Compact complex lanes, the writer (every lane calls; cx: the lane's word is complex, k its
// rank among the complex lanes, s its 16 planes, multi its multi-code / empty sites, code its
// code planes).  The sets are gathered site by site, as many rounds as the wave's most.
__device__ __forceinline__ void cx_store(uint4* p, uint32_t k, const uint32_t* s, uint32_t multi, bool cx,
                                         const uint32_t* code) {
    const bool full = cx && __builtin_popcount(multi) > kCxSets;
    uint32_t rem = cx && !full ? multi : 0u;
    uint32_t w[3] = {0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < kCxSets; ++i) {
        if (__ballot(rem != 0u) == 0) break;
        const uint32_t b = rem ? (uint32_t)__builtin_ctz(rem) : 0u;
        uint32_t set = 0u;
#pragma unroll
        for (int v = 0; v < 16; ++v) set |= ((s[v] >> b) & 1u) << v;
        w[i >> 1] |= (rem ? set : 0u) << (16 * (i & 1));
        rem &= rem - 1u;
    }
    if (!cx) return;
    store_stream(p + kWave + k, full ? make_uint4(s[0], s[1], s[2], s[3]) : make_uint4(code[0], code[1], code[2], code[3]));
    store_stream(p + 2 * kWave + k, full ? make_uint4(kCxFull, 0u, 0u, 0u) : make_uint4(multi, w[0], w[1], w[2]));
    if (full) {
#pragma unroll
        for (int j = 1; j < 4; ++j)
            store_stream(p + (j + 2) * kWave + k, make_uint4(s[4 * j], s[4 * j + 1], s[4 * j + 2], s[4 * j + 3]));
    }
}

// Where a wave's complex-slot loads point: the record's complex area, or -- when the record
// has no complex lane (uniform) -- the consensus words, which every wave reads anyway (L2
// resident), instead of four DRAM lines of unused record memory.
__device__ __forceinline__ const uint4* cx_base(const uint4* p, const RecMask& m, const uint4* cons) {
    return m.x ? p + kWave : cons;
}

// A record lane in flight: its code planes and, for a complex lane, its 16 planes.
// (compact records: c = A, v[0] = B; p / mx for a full lane's second load)
struct SetFetch {
    uint4 c, v[4];
    bool cx;
    const uint4* p;
    uint64_t mx;
};

__device__ __forceinline__ void fetch_fitch_set(const uint4* p, const RecMask& m, const uint4* cons, int lane,
                                                int64_t word, SetFetch& f) {
    f.cx = (m.x >> lane) & 1ull;
    if constexpr (kCxCompact) {
        f.c = rec_code_all<true>(p, m, lane, cons, word);
        f.v[0] = cx_b_load(p, m, lane, cons);
        f.p = p;
        f.mx = m.x;
        return;
    }
    f.c = rec_code_all(p, m, lane, cons, word);
    // every lane loads (a branch here makes the compiler copy the results out of the load
    // registers and wait for them): lanes that are not complex read the first complex slot
    // (value unused), or -- no complex lane at all -- the cache-resident consensus
    const uint4* base = cx_base(p, m, cons);
    const uint32_t k = f.cx ? lanes_below(m.x) : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) f.v[q] = load_rec(base + q * kWave + k);
}

__device__ __forceinline__ void expand_fitch_set(const SetFetch& f, uint32_t* s) {
    onehot_from_code(f.c.x, f.c.y, f.c.z, f.c.w, ~0u, s);
    if constexpr (kCxCompact) {
        cx_decode(s, f.c, f.v[0], f.cx, f.p, f.mx);
        return;
    }
    if (f.cx) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            s[4 * q + 0] = f.v[q].x;
            s[4 * q + 1] = f.v[q].y;
            s[4 * q + 2] = f.v[q].z;
            s[4 * q + 3] = f.v[q].w;
        }
    }
}

__device__ __forceinline__ void load_fitch_set(const uint4* p, const RecMask& m, const uint4* cons, int lane,
                                               int64_t word, uint32_t* s) {
    if constexpr (kCxCompact) {
        SetFetch f;
        fetch_fitch_set(p, m, cons, lane, word, f);
        expand_fitch_set(f, s);
        return;
    }
    const bool cx = (m.x >> lane) & 1ull;
    const uint4 c = rec_code_all(p, m, lane, cons, word);
    uint4 v[4] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (cx) {
        const uint32_t k = lanes_below(m.x);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = load_rec(p + kWave + q * kWave + k);
    }
    onehot_from_code(c.x, c.y, c.z, c.w, ~0u, s);
    if (cx) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            s[4 * q + 0] = v[q].x;
            s[4 * q + 1] = v[q].y;
            s[4 * q + 2] = v[q].z;
            s[4 * q + 3] = v[q].w;
        }
    }
}

__device__ __forceinline__ void load_fitch_set(const uint4* sets, const uint64_t* cmask, const uint4* cons, int64_t node,
                                               int32_t tiles, int tile, int lane, int64_t word, uint32_t* s) {
    const size_t rec = (size_t)node * tiles + tile;
    load_fitch_set(sets + rec * kFitchRec, rec_mask(cmask, rec), cons, lane, word, s);
}

// Returns the record's (x, s, d) masks through mx / ms / md (for push_children).
__device__ __forceinline__ void store_fitch_set(uint4* sets, uint64_t* cmask, const uint4& cw, int64_t node,
                                                int32_t tiles, int tile, int lane, const uint32_t* s,
                                                bool dirty_extra, uint64_t& mx, uint64_t& ms, uint64_t& md) {
    uint32_t one = 0, two = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        two |= one & s[v];
        one |= s[v];
    }
    const bool complex_word = (one != ~0u) || two != 0u;   // an empty or multi-code set
    const size_t rec = (size_t)node * tiles + tile;
    uint4* p = sets + rec * kFitchRec;
    uint32_t code[4];
    code_from_onehot(s, code[0], code[1], code[2], code[3]);
    rec_store_head(p, cmask, rec, lane, complex_word, dirty_extra, code, cw, mx, ms, md);
    if constexpr (kCxCompact) {
        cx_store(p, lanes_below(mx), s, ~one | two, complex_word, code);
        return;
    }
    if (complex_word) {
        const uint32_t k = lanes_below(mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) store_stream(p + kWave + q * kWave + k, make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]));
    }
}

// Sankoff: a word is single-code when every site has one optimal code (Z0) and no code
// one above optimal (Z1 empty) -- for a binary node, "both children agree".
__device__ __forceinline__ void load_sankoff(const uint4* p, const RecMask& m, const uint4* cons, int lane, int64_t word,
                                             uint32_t* z0, uint32_t* z1, bool want_z1) {
    if ((m.x >> lane) & 1ull) {
        const uint32_t k = lanes_below(m.x);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = load_rec(p + kWave + q * kWave + k);
            z0[4 * q + 0] = v.x; z0[4 * q + 1] = v.y; z0[4 * q + 2] = v.z; z0[4 * q + 3] = v.w;
        }
        if (want_z1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = load_rec(p + 5 * kWave + q * kWave + k);
                z1[4 * q + 0] = v.x; z1[4 * q + 1] = v.y; z1[4 * q + 2] = v.z; z1[4 * q + 3] = v.w;
            }
        }
    } else {
        const uint4 c = rec_code(p, m, lane, cons, word);
        onehot_from_code(c.x, c.y, c.z, c.w, ~0u, z0);
        if (want_z1) {
#pragma unroll
            for (int v = 0; v < 16; ++v) z1[v] = 0u;
        }
    }
}

__device__ __forceinline__ void load_sankoff(const uint4* sets, const uint64_t* cmask, const uint4* cons, int64_t node,
                                             int32_t tiles, int tile, int lane, int64_t word, uint32_t* z0, uint32_t* z1,
                                             bool want_z1) {
    const size_t rec = (size_t)node * tiles + tile;
    load_sankoff(sets + rec * kSankoffRec, rec_mask(cmask, rec), cons, lane, word, z0, z1, want_z1);
}

__device__ __forceinline__ void store_sankoff(uint4* sets, uint64_t* cmask, const uint4* cons, int64_t node,
                                              int32_t tiles, int tile, int lane, int64_t word, const uint32_t* z0,
                                              const uint32_t* z1, bool dirty_extra, uint64_t& mx, uint64_t& ms,
                                              uint64_t& md) {
    uint32_t one = 0, two = 0, any1 = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        two |= one & z0[v];
        one |= z0[v];
        any1 |= z1[v];
    }
    const bool complex_word = (one != ~0u) || two != 0u || any1 != 0u;
    const size_t rec = (size_t)node * tiles + tile;
    uint4* p = sets + rec * kSankoffRec;
    uint32_t code[4];
    code_from_onehot(z0, code[0], code[1], code[2], code[3]);
    rec_store_head(p, cmask, rec, lane, complex_word, dirty_extra, code, cons[word], mx, ms, md);
    if (complex_word) {
        const uint32_t k = lanes_below(mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) store_stream(p + kWave + q * kWave + k, make_uint4(z0[4 * q], z0[4 * q + 1], z0[4 * q + 2], z0[4 * q + 3]));
#pragma unroll
        for (int q = 0; q < 4; ++q)
            store_stream(p + 5 * kWave + q * kWave + k, make_uint4(z1[4 * q], z1[4 * q + 1], z1[4 * q + 2], z1[4 * q + 3]));
    }
}

// ---- Fitch post-order folding: (both, either) accumulate the AND and the OR of the
// children's one-hot sets plane by plane, each child expanded from 4 code planes with the
// lo/hi decomposition of onehot_from_code (8 temporaries instead of a 16-plane set).
struct LoHi {
    uint32_t lo[4], hi[4];
};

__device__ __forceinline__ LoHi lohi_of(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t m) {
    const uint32_t n0 = ~b0, n1 = ~b1, n2 = ~b2, n3 = ~b3;
    return LoHi{{n0 & n1, b0 & n1, n0 & b1, b0 & b1}, {n2 & n3 & m, b2 & n3 & m, n2 & b3 & m, b2 & b3 & m}};
}

__device__ __forceinline__ void fold_set(uint32_t* both, uint32_t* either, const uint32_t* x, int v0, int nv) {
    for (int v = v0; v < v0 + nv; ++v) {
        both[v] &= x[v - v0];
        either[v] |= x[v - v0];
    }
}

// A leaf's word: code planes and present mask (absent: mask 0 = empty set).
template <bool AP, class Args>
__device__ __forceinline__ void leaf_word(const Args& a, int32_t leaf, int64_t word, uint4& L, uint32_t& m) {
    if (!AP) {
        const uint8_t flag = a.leaf_flag[leaf];
        if (flag == kLeafAbsent) {
            L = make_uint4(0, 0, 0, 0);
            m = 0;
            return;
        }
        L = a.leaf_planes[(size_t)leaf * a.wpad + word];
        m = flag == kLeafPartial ? a.leaf_present[(size_t)leaf * a.wpad + word] : ~0u;
        return;
    }
    L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    m = ~0u;
}

// Fold child `c` (child_enc_v encoding; `vl` its leaves if virtual) into (both, either);
// `vd` collects the sites where a leaf-parent's two leaves disagree (dirty lanes).
template <bool AP, int REC = kFitchRec>
__device__ __forceinline__ void fold_child(const UpArgs& a, int32_t c, int4 vl, int tile, int lane, int64_t word,
                                           uint32_t* both, uint32_t* either, uint32_t& vd) {
    if (c < 0) {   // leaf (src/fitchSankoff.cpp:32-38, absent -> 0)
        uint4 L;
        uint32_t m;
        leaf_word<AP>(a, -c - 1, word, L, m);
        const LoHi t = lohi_of(L.x, L.y, L.z, L.w, m);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const uint32_t x = t.lo[v & 3] & t.hi[v >> 2];
            both[v] &= x;
            either[v] |= x;
        }
    } else if (c & kVirtualBit) {   // leaf-parent (one or two leaves): the union of their codes
        const int32_t l0 = __builtin_amdgcn_readfirstlane(vl.x), l1 = __builtin_amdgcn_readfirstlane(vl.y);
        uint4 L0, L1 = make_uint4(0, 0, 0, 0);
        uint32_t m0, m1 = 0;
        leaf_word<AP>(a, l0, word, L0, m0);
        if (l1 >= 0) {
            leaf_word<AP>(a, l1, word, L1, m1);
            vd |= (L0.x ^ L1.x) | (L0.y ^ L1.y) | (L0.z ^ L1.z) | (L0.w ^ L1.w);
        }
        const LoHi t0 = lohi_of(L0.x, L0.y, L0.z, L0.w, m0), t1 = lohi_of(L1.x, L1.y, L1.z, L1.w, m1);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const uint32_t x = (t0.lo[v & 3] & t0.hi[v >> 2]) | (t1.lo[v & 3] & t1.hi[v >> 2]);
            both[v] &= x;
            either[v] |= x;
        }
    } else {       // materialised internal child: compressed record
        const size_t rec = (size_t)c * a.tiles + tile;
        const RecMask mk = rec_mask(a.cmask, rec);
        const uint4* p = a.sets + rec * REC;
        if constexpr (kCxCompact && REC == kFitchRec) {
            SetFetch f;
            fetch_fitch_set(p, mk, a.cons, lane, word, f);
            uint32_t x[16];
            expand_fitch_set(f, x);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                both[v] &= x[v];
                either[v] |= x[v];
            }
        } else if ((mk.x >> lane) & 1ull) {
            const uint32_t k = lanes_below(mk.x);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 w = load_rec(p + kWave + q * kWave + k);
                const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    both[4 * q + j] &= x[j];
                    either[4 * q + j] |= x[j];
                }
            }
        } else {
            const uint4 w = rec_code(p, mk, lane, a.cons, word);
            const LoHi t = lohi_of(w.x, w.y, w.z, w.w, ~0u);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const uint32_t x = t.lo[v & 3] & t.hi[v >> 2];
                both[v] &= x;
                either[v] |= x;
            }
        }
    }
}

// All-present post-order children in two phases, so that both children's loads are in
// flight together: a fetch into `code` (leaf codes, or the record's code planes) and `v`
// (a leaf-parent's second leaf in v[0], or a complex lane's 16 planes), written only by
// loads -- zero-filling them on a sibling branch makes the compiler drain all outstanding
// loads -- then the fold into (both, either).
struct ChildFetch {
    uint4 code, v[4];
    bool cx;
    const uint4* p;   // compact Fitch records: code = A, v[0] = B; p / mx for cx_decode
    uint64_t mx;
};

// LEAFY: the caller knows c is a leaf or a virtual leaf-parent (no record, fewer registers).
// SUB: subtree form -- a virtual child may be an S2 / S3 subtree (three or four leaves, in
// code, v[0], v[1], v[2]).
// SLOT: a record child's (x, s) masks are (sx, ss), from its parent's up slot (UpArgs::upm).
template <int REC = kFitchRec, bool LEAFY = false, bool SUB = false, bool SLOT = false>
__device__ __forceinline__ void fetch_child_ap(const UpArgs& a, int32_t c, int4 vl, int tile, int lane, int64_t word,
                                               ChildFetch& f, uint64_t sx = 0, uint64_t ss = 0) {
    f.cx = false;
    if (c < 0) {
        f.code = a.leaf_planes[(size_t)(-c - 1) * a.wpad + word];
    } else if (c & kVirtualBit) {
        // (an S2 / S3 child's leaves from their rows, every lane: coalesced.  The side-by-side
        // layout, sub_planes, is for the tail's scattered dirty lanes; read here it made the
        // post-order 6 % slower -- four times the cache lines per load instruction.)
        const int32_t l0 = __builtin_amdgcn_readfirstlane(vl.x), l1 = __builtin_amdgcn_readfirstlane(vl.y);
        f.code = a.leaf_planes[(size_t)l0 * a.wpad + word];
        if (l1 >= 0) f.v[0] = a.leaf_planes[(size_t)l1 * a.wpad + word];
        if constexpr (SUB) {
            const int32_t l2 = __builtin_amdgcn_readfirstlane(vl.z), l3 = __builtin_amdgcn_readfirstlane(vl.w);
            if (l2 >= 0) f.v[1] = a.leaf_planes[(size_t)l2 * a.wpad + word];
            if (l3 >= 0) f.v[2] = a.leaf_planes[(size_t)l3 * a.wpad + word];
        }
    } else if (!LEAFY) {
        const size_t rec = (size_t)c * a.tiles + tile;
        const RecMask m = SLOT ? RecMask{sx, ss, 0, 0, 0} : rec_mask(a.cmask, rec);
        const uint4* p = a.sets + rec * REC;   // Sankoff: the Z0 planes
        f.cx = (m.x >> lane) & 1ull;
        if constexpr (kCxCompact && REC == kFitchRec) {
            f.code = rec_code_all<true>(p, m, lane, a.cons, word);
            f.v[0] = cx_b_load(p, m, lane, a.cons);
            f.p = p;
            f.mx = m.x;
            return;
        }
        f.code = rec_code_all(p, m, lane, a.cons, word);
        const uint4* base = cx_base(p, m, a.cons);   // see fetch_fitch_set
        const uint32_t k = f.cx ? lanes_below(m.x) : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) f.v[q] = load_rec(base + q * kWave + k);
    }
}

// fetch_child_ap for a child whose record masks (x, s) the caller already holds (wide nodes:
// every child's masks are loaded up front, one per lane, so a child's record loads wait for
// no mask load of their own)
template <int REC = kFitchRec>
__device__ __forceinline__ void fetch_child_ap_m(const UpArgs& a, int32_t c, int4 vl, uint64_t mx, uint64_t ms, int tile,
                                                 int lane, int64_t word, ChildFetch& f) {
    if (c < 0 || (c & kVirtualBit)) {
        fetch_child_ap<REC, false, false>(a, c, vl, tile, lane, word, f);
        return;
    }
    const size_t rec = (size_t)c * a.tiles + tile;
    const RecMask m{mx, ms, 0, 0, 0};
    const uint4* p = a.sets + rec * REC;
    f.cx = (m.x >> lane) & 1ull;
    if constexpr (kCxCompact && REC == kFitchRec) {
        f.code = rec_code_all<true>(p, m, lane, a.cons, word);
        f.v[0] = cx_b_load(p, m, lane, a.cons);
        f.p = p;
        f.mx = m.x;
        return;
    }
    f.code = rec_code_all(p, m, lane, a.cons, word);
    const uint4* base = cx_base(p, m, a.cons);   // see fetch_fitch_set
    const uint32_t k = f.cx ? lanes_below(m.x) : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) f.v[q] = load_rec(base + q * kWave + k);
}

// (the builtin returns int: each half goes through uint32_t, or the low half's bit 31 would
// sign-extend over the high half)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t code_ne(const uint4& p, const uint4& q) {
    return (p.x ^ q.x) | (p.y ^ q.y) | (p.z ^ q.z) | (p.w ^ q.w);
}

// An S2 (cherry (a, b), leaf c) or S3 (cherries (a, b), (c, d)) child's Fitch set, from the
// union of its cherry's leaves (src/fitchSankoff.cpp:39-55 applied twice):
//   S2: {c} where c is a or b, else {a, b, c};   S3: X & Y where the cherries share a code,
//   else X | Y.  vd: sites where the subtree's leaves are not all one code (dirty lanes).
__device__ __forceinline__ void subtree_set_ap(int shape, const ChildFetch& f, uint32_t* x, uint32_t& vd) {
    const uint4 A = f.code, B = f.v[0], Cc = f.v[1];
    const LoHi u = lohi_of(B.x, B.y, B.z, B.w, ~0u), w = lohi_of(Cc.x, Cc.y, Cc.z, Cc.w, ~0u);
#pragma unroll
    for (int v = 0; v < 16; ++v) x[v] |= u.lo[v & 3] & u.hi[v >> 2];   // X = {a, b}
    if (shape == 1) {
        vd |= code_ne(A, B) | code_ne(A, Cc);
        const uint32_t in_x = ~code_ne(Cc, A) | ~code_ne(Cc, B);
#pragma unroll
        for (int v = 0; v < 16; ++v) x[v] = (x[v] & ~in_x) | (w.lo[v & 3] & w.hi[v >> 2]);
    } else {
        const uint4 D = f.v[2];
        vd |= code_ne(A, B) | code_ne(A, Cc) | code_ne(A, D);
        const LoHi z = lohi_of(D.x, D.y, D.z, D.w, ~0u);
        const uint32_t nz = ~code_ne(A, Cc) | ~code_ne(A, D) | ~code_ne(B, Cc) | ~code_ne(B, D);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const uint32_t y = (w.lo[v & 3] & w.hi[v >> 2]) | (z.lo[v & 3] & z.hi[v >> 2]);
            x[v] = (x[v] & y) | ((x[v] | y) & ~nz);
        }
    }
}

// A fetched child's 16-plane set (Fitch) / optimal set Z0 (Sankoff); vd as fold_child's.
// CXC: a record child is a compact Fitch record (fetch_child_ap<kFitchRec>).
template <bool SUB = false, bool CXC = false>
__device__ __forceinline__ void child_set_ap(int32_t c, int4 vl, const ChildFetch& f, uint32_t* x, uint32_t& vd) {
    const LoHi t = lohi_of(f.code.x, f.code.y, f.code.z, f.code.w, ~0u);
#pragma unroll
    for (int v = 0; v < 16; ++v) x[v] = t.lo[v & 3] & t.hi[v >> 2];
    if (SUB && c >= 0 && (c & kVirtualBit) && ((c >> kShapeShift) & 3)) {
        subtree_set_ap((c >> kShapeShift) & 3, f, x, vd);
    } else if (c >= 0 && (c & kVirtualBit)) {
        if (__builtin_amdgcn_readfirstlane(vl.y) >= 0) {
            const uint4 L1 = f.v[0];
            vd |= (f.code.x ^ L1.x) | (f.code.y ^ L1.y) | (f.code.z ^ L1.z) | (f.code.w ^ L1.w);
            const LoHi u = lohi_of(L1.x, L1.y, L1.z, L1.w, ~0u);
#pragma unroll
            for (int v = 0; v < 16; ++v) x[v] |= u.lo[v & 3] & u.hi[v >> 2];
        }
    } else if (CXC && c >= 0) {
        cx_decode(x, f.code, f.v[0], f.cx, f.p, f.mx);
    } else if (c >= 0 && f.cx) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            x[4 * q] = f.v[q].x; x[4 * q + 1] = f.v[q].y; x[4 * q + 2] = f.v[q].z; x[4 * q + 3] = f.v[q].w;
        }
    }
}

// A child of a plain node (leaf, leaf-parent of one or two leaves, or record), branch-free over
// its kind (wave-uniform) and the lane's complex flag: one select per plane.
template <bool CXC = false>
__device__ __forceinline__ void child_set_plain(int32_t c, int4 vl, const ChildFetch& f, uint32_t* x, uint32_t& vd) {
    const bool virt2 = c >= 0 && (c & kVirtualBit) && __builtin_amdgcn_readfirstlane(vl.y) >= 0;
    const bool rec_cx = !CXC && c >= 0 && !(c & kVirtualBit) && f.cx;
    const uint32_t m2 = virt2 ? ~0u : 0u;
    const uint4 L1 = f.v[0];
    vd |= m2 & code_ne(f.code, L1);
    const LoHi t = lohi_of(f.code.x, f.code.y, f.code.z, f.code.w, ~0u), u = lohi_of(L1.x, L1.y, L1.z, L1.w, m2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t w[4] = {f.v[q].x, f.v[q].y, f.v[q].z, f.v[q].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int v = 4 * q + k;
            const uint32_t y = (t.lo[v & 3] & t.hi[v >> 2]) | (u.lo[v & 3] & u.hi[v >> 2]);
            x[v] = rec_cx ? w[k] : y;
        }
    }
    if (CXC && c >= 0 && !(c & kVirtualBit)) cx_decode(x, f.code, f.v[0], f.cx, f.p, f.mx);
}

template <bool SUB = false, bool CXC = false>
__device__ __forceinline__ void fold_child_ap(int32_t c, int4 vl, const ChildFetch& f, uint32_t* both, uint32_t* either,
                                              uint32_t& vd) {
    uint32_t x[16];
    child_set_ap<SUB, CXC>(c, vl, f, x, vd);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        both[v] &= x[v];
        either[v] |= x[v];
    }
}

// Leaf child as a one-hot set: src/fitchSankoff.cpp:32-38 (absent leaf -> 0).
template <class Args>
__device__ __forceinline__ void leaf_set16(const Args& a, int32_t leaf, int64_t word, uint32_t* s) {
    const uint8_t flag = a.leaf_flag[leaf];
    if (flag == kLeafAbsent) {
#pragma unroll
        for (int v = 0; v < 16; ++v) s[v] = 0;
        if (a.absent_code0) s[0] = ~0u;
        return;
    }
    const uint4 L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    const uint32_t m = flag == kLeafPartial ? a.leaf_present[(size_t)leaf * a.wpad + word] : ~0u;
    onehot_from_code(L.x, L.y, L.z, L.w, m, s);
    if (a.absent_code0) s[0] |= ~m;
}

// Set of a "virtual" internal node whose children are all leaves (never materialised).
// Leaf sets are single codes or empty, so the Fitch AND is non-empty only when every leaf
// is present with the same code -- and then equals the OR: the set is always the union of
// the present leaves' codes (src/fitchSankoff.cpp:39-55).
template <class Args>
__device__ __forceinline__ void virtual_set16(const Args& a, int32_t v, int64_t word, uint32_t* s) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = 0u;
    const int32_t e0 = __builtin_amdgcn_readfirstlane(a.child_off[v]);
    const int32_t e1 = __builtin_amdgcn_readfirstlane(a.child_off[v + 1]);
    for (int32_t e = e0; e < e1; ++e) {
        leaf_set16(a, -__builtin_amdgcn_readfirstlane(a.child_enc[e]) - 1, word, x);
#pragma unroll
        for (int k = 0; k < 16; ++k) s[k] |= x[k];
    }
}

// GROUP (grouped post-order launches, all leaves present).  fold_first_two<SUB, D, REC>: the node
// d's first two children folded into (both, either, vd); a child of this same launch
// (pad0 / pad1 = its descriptor index) is recomputed -- its own first two children folded the
// same way, D - 1 levels further down, then its further children and the AND-else-OR, as its
// own wave computes its set (fitch_up_node), in registers, without the store -- and the
// recomputed children go first, while the accumulators are still one set.  REC: the record
// stride (Fitch sets, or Sankoff's whose first 16 planes are Z0; a recomputed Sankoff child is
// binary, so its Z0 is this same AND-else-OR of its children's Z0).
template <bool SUB, int D, int REC>
__device__ __forceinline__ void fold_first_two(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int lane,
                                               int64_t word, uint32_t* both, uint32_t* either, uint32_t& vd);

template <bool SUB, int D, int REC>
__device__ __forceinline__ void child_recompute(const UpArgs& a, const NodeDesc& cd, int32_t gi, int tile, int lane,
                                                int64_t word, uint32_t* x) {
    uint32_t both[16], either[16], vd = 0;
    fold_first_two<SUB, D, REC>(a, cd, gi, tile, lane, word, both, either, vd);
    for (int32_t e = cd.e0 + 2; e < cd.e1; ++e) {
        const int32_t c = __builtin_amdgcn_readfirstlane(a.child_enc[e]);
        const int4 vl = c >= 0 && (c & kVirtualBit) ? a.vleaf[c & kDenseMask] : make_int4(-1, -1, -1, -1);
        fold_child<true, REC>(a, c, vl, tile, lane, word, both, either, vd);
    }
    const uint32_t nz = any_plane(both);
#pragma unroll
    for (int v = 0; v < 16; ++v) x[v] = both[v] | (either[v] & ~nz);
}

template <bool SUB, int D, int REC>
__device__ __forceinline__ void fold_first_two(const UpArgs& a, const NodeDesc& d, int32_t gi, int tile, int lane,
                                               int64_t word, uint32_t* both, uint32_t* either, uint32_t& vd) {
    constexpr bool SLOT = SUB;   // (subtree form: up slots)
    UpSlots sl{0, 0, 0, 0};
    if constexpr (SLOT) sl = load_up_slots(a, gi, tile);
    const int4 vl0 = make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), vl1 = make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]);
    const bool two = d.e1 - d.e0 > 1;
    if (D > 0 && (d.pad0 >= 0 || d.pad1 >= 0)) {
        uint32_t x0[16];
        const int32_t r0 = d.pad0 >= 0 ? d.pad0 : d.pad1;
        child_recompute<SUB, (D > 0 ? D - 1 : 0), REC>(a, a.desc_all[r0], r0, tile, lane, word, x0);
        if (d.pad0 >= 0 && d.pad1 >= 0) {
            uint32_t x1[16];
            child_recompute<SUB, (D > 0 ? D - 1 : 0), REC>(a, a.desc_all[d.pad1], d.pad1, tile, lane, word, x1);
#pragma unroll
            for (int v = 0; v < 16; ++v) { both[v] = x0[v] & x1[v]; either[v] = x0[v] | x1[v]; }
            return;
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) { both[v] = x0[v]; either[v] = x0[v]; }
        if (d.pad0 < 0 || two) {
            const bool first = d.pad0 < 0;   // the loaded one: slot 0 or slot 1
            const int32_t c = first ? d.c0 : d.c1;
            const int4 vl = first ? vl0 : vl1;
            ChildFetch f;
            fetch_child_ap<REC, false, SUB, SLOT>(a, c, vl, tile, lane, word, f, first ? sl.x0 : sl.x1, first ? sl.s0 : sl.s1);
            fold_child_ap<SUB, kCxCompact && REC == kFitchRec>(c, vl, f, both, either, vd);
        }
        return;
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) { both[v] = ~0u; either[v] = 0u; }
    ChildFetch f0, f1;
    fetch_child_ap<REC, false, SUB, SLOT>(a, d.c0, vl0, tile, lane, word, f0, sl.x0, sl.s0);
    if (two) fetch_child_ap<REC, false, SUB, SLOT>(a, d.c1, vl1, tile, lane, word, f1, sl.x1, sl.s1);
    __builtin_amdgcn_sched_barrier(0);
    fold_child_ap<SUB, kCxCompact && REC == kFitchRec>(d.c0, vl0, f0, both, either, vd);
    if (two) fold_child_ap<SUB, kCxCompact && REC == kFitchRec>(d.c1, vl1, f1, both, either, vd);
}

// bit-sliced a < b for 4-bit codes
__device__ __forceinline__ uint32_t code_less(const uint32_t* A, const uint32_t* B) {
    uint32_t lt = ~A[0] & B[0];
#pragma unroll
    for (int j = 1; j < 4; ++j) lt = (~A[j] & B[j]) | (~(A[j] ^ B[j]) & lt);
    return lt;
}

struct DownArgs {
    const NodeDesc* desc;  // per level item
    const TailDesc* tail;  // k_tail items
    int32_t count;
    const int4* vleaf;     // virtual node -> its (one or two) leaves, -1 padded
    const int32_t* vinner; // subtree form: an S2 / S3 node's cherries (dense), [I][2]
    const int32_t* child_off;
    const int32_t* child_enc;
    const int32_t* parent_dense;
    const int32_t* internal_id;
    const int32_t* leaf_id;
    const uint8_t* leaf_flag;
    const uint4* leaf_planes;
    const uint32_t* leaf_present;
    uint4* sets;           // records; after a node's step its complex lanes' finals sit in final_slot
    const uint64_t* cmask;
    uint4* root_final;     // [W] the root's final codes (a forced root's differ from its set)
    int32_t dense_base;    // k_down<.., DENSE>: the level's first dense index (item k = dense base + k)
    int32_t split[3];      // k_down<.., GROUP>: the first items of the group's levels 1, 2, 3
    int32_t dense_g[4];    // k_down<.., DENSE, .., GROUP>: each level's first dense index
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
    const uint4* forced;   // Sankoff / block defaultState per site (nullable)
    bool absent_code0;     // block Sankoff: a leaf missing from the column is state 0
    bool all_present;      // every leaf present at every site
    int32_t num_s;         // k_tail (subtree form): items [0, num_s) are the S2 / S3 nodes ...
    int32_t sbase;         // ... of dense index sbase + item
    const uint4* sub_planes;   // ... whose leaves sit side by side there (sub_word)
};

template <class Args>
__device__ __forceinline__ uint32_t valid_mask(const Args& a, int64_t word) {
    if (word >= a.words) return 0u;
    const int64_t left = a.sites - word * 32;
    return left >= 32 ? ~0u : ((1u << left) - 1u);
}

// Leaf mutation mask against the parent's final codes F (leaf final = own code).
template <class Args>
__device__ __forceinline__ uint32_t leaf_diff(const Args& a, int32_t leaf, int64_t word, uint32_t valid,
                                              const uint32_t* F, uint4& L) {
    const uint8_t flag = a.leaf_flag[leaf];
    if (flag == kLeafAbsent) {
        if (!a.absent_code0) return 0u;
        L = make_uint4(0, 0, 0, 0);
        return valid & (F[0] | F[1] | F[2] | F[3]);
    }
    L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    uint32_t m = valid;
    if (flag == kLeafPartial) {
        const uint32_t p = a.leaf_present[(size_t)leaf * a.wpad + word];
        if (a.absent_code0) {   // missing sites are state 0
            L.x &= p; L.y &= p; L.z &= p; L.w &= p;
        } else {
            m &= p;
        }
    }
    return m & ((L.x ^ F[0]) | (L.y ^ F[1]) | (L.z ^ F[2]) | (L.w ^ F[3]));
}

// Mutation records (src/fitchSankoff.cpp:140-166, :676-703): one per changed site --
// parent gap -> NI, child gap -> ND (char '-', code 0), else NS; NI / NS carry the child's
// code.  The record's low byte, (type << 4) | code, is the child's code with ND = parent not
// gap & child gap, NI = parent gap (PM_MUT_ND = 1, PM_MUT_NI = 2).
//
// Emission by entries.  A record stream is one node's 32-site word: the mask D of sites where
// its final differs from its parent's, its 4 code planes and its parent's gap plane.  Each
// stream is staged in the wave's LDS area as a 32-B entry -- lanes with D != 0 packed by rank
// (ballot + mbcnt), no per-lane loop while staging -- and a flush reserves the wave's records
// in a shard with one global atomic, then expands the entries one per lane, every lane busy
// whichever lanes the records came from, straight into the reserved range.
static_assert(PM_MUT_NS == 0 && PM_MUT_ND == 1 && PM_MUT_NI == 2, "record type bits");
__device__ __forceinline__ uint32_t bit_at(uint32_t plane, int b) { return __builtin_amdgcn_ubfe(plane, b, 1); }

constexpr uint32_t kEntryCap = 128;          // staged entries per wave (4 KiB of LDS)
constexpr int kEntryQuads = 2 * kEntryCap;   // entry k = quads 2k {D, node, site0, parent gap}, 2k+1 {code planes}

struct Emit {
    uint4* lds;       // the wave's kEntryQuads
    uint32_t shard;   // record shard this wave appends to
    uint32_t n;       // staged entries (wave-uniform)
    uint32_t cnt;     // records of this lane's staged entries
};

// low byte of the record at bit b of an entry
__device__ __forceinline__ uint32_t rec_low(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t pz, int b) {
    const uint32_t code = bit_at(c0, b) | (bit_at(c1, b) << 1) | (bit_at(c2, b) << 2) | (bit_at(c3, b) << 3);
    const uint32_t z = bit_at(pz, b);
    return code | ((uint32_t)(code == 0 && z == 0) << 4) | (z << 5);
}

// An entry whose word holds more than kHeavyBits records (an N run at a leaf, a gap) is
// expanded by 32 lanes at once; the others write theirs one per loop iteration, so a round's
// trip count is at most kHeavyBits plus one per heavy entry instead of the largest count (32).
constexpr int kHeavyBits = 4;

// One round of a flush: entries e0 / e1 (one per lane, D = 0 past the staged ones), the
// lane's first record at p0.
__device__ __forceinline__ void emit_round(pm_mut* out, int64_t cap, const uint4& e0, const uint4& e1, uint32_t p0,
                                           int lane) {
    const uint32_t D = e0.x, node = e0.y, site0 = e0.z, pz = e0.w;
    const uint32_t c = (uint32_t)__builtin_popcount(D);
    {
        const bool heavy = c > (uint32_t)kHeavyBits;
        uint32_t d = heavy ? 0u : D, p = p0;
        while (d) {
            const int b = __builtin_ctz(d);
            d &= d - 1;
            if ((int64_t)p < cap) out[p] = pm_mut{node, ((site0 + (uint32_t)b) << 8) | rec_low(e1.x, e1.y, e1.z, e1.w, pz, b)};
            ++p;
        }
        uint64_t hv = __ballot(heavy);
        const int bit = lane & 31;
        while (hv) {
            const int l = __builtin_ctzll(hv);
            hv &= hv - 1;
            const uint32_t w = __builtin_amdgcn_readlane(D, l);
            const uint32_t h0 = __builtin_amdgcn_readlane(e1.x, l), h1 = __builtin_amdgcn_readlane(e1.y, l),
                           h2 = __builtin_amdgcn_readlane(e1.z, l), h3 = __builtin_amdgcn_readlane(e1.w, l),
                           hz = __builtin_amdgcn_readlane(pz, l), hs = __builtin_amdgcn_readlane(site0, l),
                           hn = __builtin_amdgcn_readlane(node, l), hp = __builtin_amdgcn_readlane(p0, l);
            if (lane < 32 && ((w >> bit) & 1u)) {
                const uint32_t q = hp + __builtin_amdgcn_mbcnt_lo(w, 0u);
                if ((int64_t)q < cap) out[q] = pm_mut{hn, ((hs + (uint32_t)bit) << 8) | rec_low(h0, h1, h2, h3, hz, bit)};
            }
        }
    }
}

// entry j (< kEntryCap: inside the wave's area, so read without a branch); D = 0 past the
// staged entries
__device__ __forceinline__ void emit_load(const Emit& em, uint32_t j, uint4& e0, uint4& e1) {
    e0 = em.lds[2 * j];
    e1 = em.lds[2 * j + 1];
    if (j >= em.n) e0.x = 0;
}

// The reservation (one returned atomic) is issued first; the first round's entries and their
// positions relative to it are read while it is in flight.  (The library is built with
// -amdgpu-atomic-optimizer-strategy=None: the optimizer wraps this already wave-aggregated
// atomic in a scan of its own whose readfirstlane waits for the atomic right away.)
// PEEL: the first round is a copy of its own, its stores also issued before the loop's code
// -- faster for the Fitch kernels (k_down + k_tail 7.08 -> 6.92 ms at N*), slower for the
// larger Sankoff ones (10.18 -> 10.39 ms), which take the loop (10.10 ms).
template <bool PEEL = false, class Args>
__device__ __forceinline__ void emit_flush(const Args& a, Emit& em, int lane) {
    if (em.n == 0) return;
    uint32_t total;
    (void)wave_exclusive_scan(em.cnt, total);
    uint32_t got = 0;
    if (lane == 0) got = atomicAdd(&a.shard_cnt[em.shard], total);
    pm_mut* out = a.recs + (size_t)em.shard * a.shard_cap;
    const int64_t cap = a.shard_cap;
    // each round's entries and relative positions are read before the round; the first
    // round's while the reservation is in flight
    uint4 e0, e1;
    emit_load(em, (uint32_t)lane, e0, e1);
    uint32_t tot;
    uint32_t rel = wave_exclusive_scan((uint32_t)__builtin_popcount(e0.x), tot);
    uint32_t base = __builtin_amdgcn_readfirstlane(got);
    if constexpr (PEEL) {
        emit_round(out, cap, e0, e1, base + rel, lane);
        base += tot;
        for (uint32_t r0 = kWave; r0 < em.n; r0 += kWave) {
            emit_load(em, r0 + (uint32_t)lane, e0, e1);
            const uint32_t p0 = base + wave_exclusive_scan((uint32_t)__builtin_popcount(e0.x), tot);
            emit_round(out, cap, e0, e1, p0, lane);
            base += tot;
        }
        em.n = 0;
        em.cnt = 0;
        return;
    }
    for (uint32_t r0 = kWave;; r0 += kWave) {
        emit_round(out, cap, e0, e1, base + rel, lane);
        base += tot;
        if (r0 >= em.n) break;
        emit_load(em, r0 + (uint32_t)lane, e0, e1);
        rel = wave_exclusive_scan((uint32_t)__builtin_popcount(e0.x), tot);
    }
    em.n = 0;
    em.cnt = 0;
}

// Stage one stream: node id (wave-uniform), diff mask D, the child's code planes c, the
// parent's code planes pc.  Every lane of the wave calls it.
template <class Args>
__device__ __forceinline__ void emit_stream(const Args& a, Emit& em, int lane, uint32_t node, uint32_t D, uint32_t site0,
                                            uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, const uint32_t* pc) {
    const uint64_t m = __ballot(D != 0);
    if (m == 0) return;
    const uint32_t k = (uint32_t)__builtin_popcountll(m);
    if (em.n + k > kEntryCap) emit_flush(a, em, lane);
    if (D) {
        const uint32_t at = em.n + lanes_below(m);
        em.lds[2 * at] = make_uint4(D, node, site0, ~(pc[0] | pc[1] | pc[2] | pc[3]));
        em.lds[2 * at + 1] = make_uint4(c0, c1, c2, c3);
        em.cnt += (uint32_t)__builtin_popcount(D);
    }
    em.n += k;
}

__device__ __forceinline__ uint32_t shard_of(uint32_t salt, int tile) { return (salt * 31u + (uint32_t)tile * 7919u) % kShards; }

// A leaf word for emission: its code planes L and the mask of sites where it can carry a
// mutation (leaf_diff's rules: absent leaves none -- or, block Sankoff, state 0 everywhere;
// partially present rows their present sites).  For Fitch the mask is the presence mask.
template <bool AP, class Args>
__device__ __forceinline__ void leaf_fetch(const Args& a, int32_t leaf, int64_t word, uint4& L, uint32_t& mv) {
    if (AP) {
        L = a.leaf_planes[(size_t)leaf * a.wpad + word];
        mv = ~0u;
        return;
    }
    const uint8_t flag = a.leaf_flag[leaf];
    if (flag == kLeafAbsent) {
        L = make_uint4(0, 0, 0, 0);
        mv = a.absent_code0 ? ~0u : 0u;
        return;
    }
    L = a.leaf_planes[(size_t)leaf * a.wpad + word];
    mv = ~0u;
    if (flag == kLeafPartial) {
        const uint32_t p = a.leaf_present[(size_t)leaf * a.wpad + word];
        if (a.absent_code0) {
            L.x &= p; L.y &= p; L.z &= p; L.w &= p;
        } else {
            mv = p;
        }
    }
}

__device__ __forceinline__ uint32_t diff4(const uint4& L, const uint32_t* F) {
    return (L.x ^ F[0]) | (L.y ^ F[1]) | (L.z ^ F[2]) | (L.w ^ F[3]);
}

// One of the first two children of a node, fetched before the node's own state is known
// (leaf: its word; virtual leaf-parent: its first two leaves' words), with the caller node
// ids its records carry (id0: the child; id1, id2: a virtual child's leaves).
struct Kid {
    int32_t enc = 0;
    int4 vl = make_int4(-1, -1, -1, -1);
    uint4 L0 = make_uint4(0, 0, 0, 0), L1 = make_uint4(0, 0, 0, 0);
    uint32_t m0 = 0, m1 = 0;
    // subtree form (S2 / S3 child): third and fourth leaf, node ids of its cherries
    uint4 L2 = make_uint4(0, 0, 0, 0), L3 = make_uint4(0, 0, 0, 0);
    int32_t ix = -1, iy = -1;
    uint32_t id0 = 0, id1 = 0, id2 = 0;
};

__device__ __forceinline__ int kid_shape(int32_t enc) { return enc >= 0 && (enc & kVirtualBit) ? (enc >> kShapeShift) & 3 : 0; }

// Fitch with every leaf present: at a lane where a node's set is one code c at every site
// (not complex) each leaf child holds c and the node's final is c (rec_store_head), so a
// leaf child's records lie in the node's complex lanes (RecMask::x).  Not for Sankoff (a
// one-code Z0 can take its parent's code from Z1) nor with absent leaves.
template <Mode M, bool AP>
__device__ __forceinline__ bool leaf_rule(int32_t enc) { return M == Mode::kFitch && AP && enc < 0; }

// A clean lane of the parent (not `dirty`, RecMask::d) fetches nothing: its children hold
// the parent's code there, so their masks stay 0 and they emit no records.
// Loads are written as "initialise, then exec-masked load" with the leaf choice made on
// uniform values first: zero-filling a load's registers on a sibling branch instead makes
// the compiler drain every outstanding load (s_waitcnt vmcnt(0)) between the fetches.
// IDS: load the records' node ids (uniform scalar loads, in flight with the words).
template <Mode M, bool AP, bool SUB = false, bool IDS = true>
__device__ __forceinline__ void kid_fetch(const DownArgs& a, int32_t enc, int4 vl, int64_t word, bool dirty, Kid& k) {
    k.enc = enc;
    int32_t l0 = -1, l1 = -1;
    if (enc < 0) {
        l0 = -enc - 1;
        if (IDS) k.id0 = (uint32_t)a.leaf_id[l0];
    } else if (M != Mode::kBlockFitch && (enc & kVirtualBit)) {
        k.vl = make_int4(__builtin_amdgcn_readfirstlane(vl.x), __builtin_amdgcn_readfirstlane(vl.y),
                         __builtin_amdgcn_readfirstlane(vl.z), __builtin_amdgcn_readfirstlane(vl.w));
        l0 = k.vl.x;
        l1 = k.vl.y;
        if (IDS) {
            k.id0 = (uint32_t)a.internal_id[enc & kDenseMask];
            k.id1 = (uint32_t)a.leaf_id[l0];
            if (l1 >= 0) k.id2 = (uint32_t)a.leaf_id[l1];
        }
    }
    k.L0 = k.L1 = make_uint4(0, 0, 0, 0);
    k.m0 = k.m1 = 0;
    if (AP) {
        if (l0 >= 0 && dirty) {
            k.L0 = a.leaf_planes[(size_t)l0 * a.wpad + word];
            k.m0 = ~0u;
        }
        if (l1 >= 0 && dirty) {
            k.L1 = a.leaf_planes[(size_t)l1 * a.wpad + word];
            k.m1 = ~0u;
        }
        if constexpr (SUB) {
            const int sh = kid_shape(enc);
            if (sh) {   // S2 / S3: the other leaves (the cherries' ids come with the tail descriptor)
                k.L2 = k.L3 = make_uint4(0, 0, 0, 0);
                if (dirty) k.L2 = a.leaf_planes[(size_t)k.vl.z * a.wpad + word];
                if (sh == 2 && dirty) k.L3 = a.leaf_planes[(size_t)k.vl.w * a.wpad + word];
            }
        }
    } else {
        if (l0 >= 0 && dirty) leaf_fetch<AP>(a, l0, word, k.L0, k.m0);
        if (l1 >= 0 && dirty) leaf_fetch<AP>(a, l1, word, k.L1, k.m1);
    }
}

// An S2 / S3 child fetched for its parent's pre-order wave (PM_OPT_SUB_DOWN): its leaves'
// words side by side (sub_planes, one 64-B sector per dirty lane), as the tail reads them.
__device__ __forceinline__ void kid_fetch_s(const DownArgs& a, int32_t enc, int64_t word, bool dirty, Kid& k) {
    k.enc = enc;
    k.L0 = k.L1 = k.L2 = k.L3 = make_uint4(0, 0, 0, 0);
    k.m0 = k.m1 = 0;
    const uint4* q = sub_word(a.sub_planes, (enc & kDenseMask) - a.sbase, a.wpad, word);
    if (dirty) {
        k.L0 = q[0];
        k.L1 = q[1];
        k.L2 = q[2];
        k.m0 = k.m1 = ~0u;
    }
    if (dirty && kid_shape(enc) == 2) k.L3 = q[3];
}

// Fold one leaf into a virtual node's union / lowest code / "parent code present" masks.
__device__ __forceinline__ void virt_fold(const uint4& L, uint32_t m, const uint32_t* Fn, uint32_t* low, uint32_t& have,
                                          uint32_t& hit) {
    const uint32_t C[4] = {L.x, L.y, L.z, L.w};
    hit |= m & ~((C[0] ^ Fn[0]) | (C[1] ^ Fn[1]) | (C[2] ^ Fn[2]) | (C[3] ^ Fn[3]));
    const uint32_t take = m & (~have | code_less(C, low));
#pragma unroll
    for (int j = 0; j < 4; ++j) low[j] = (C[j] & take) | (low[j] & ~take);
    have |= m;
}

__device__ __forceinline__ uint4 sel4(uint32_t t, const uint4& p, const uint4& q) {
    return make_uint4(bsel(t, p.x, q.x), bsel(t, p.y, q.y), bsel(t, p.z, q.z), bsel(t, p.w, q.w));
}
__device__ __forceinline__ uint4 min4(const uint4& p, const uint4& q) {   // lower code per site
    const uint32_t P[4] = {p.x, p.y, p.z, p.w}, Q[4] = {q.x, q.y, q.z, q.w};
    return sel4(code_less(Q, P), q, p);
}

// Fitch finals inside an S2 / S3 child v given its parent's final P (src/fitchSankoff.cpp:
// 115-123 at v, then at its cherries; leaves keep their codes):
//   S2 (x = (a, b), c): S_v = {c} if c in {a, b}, else {a, b, c};
//   S3 (x = (a, b), y = (c, d)): S_v = X & Y if the cherries share a code, else X | Y.
//   F_v = P if P in S_v else lowest(S_v);  F_x = F_v if F_v in {a, b} else min(a, b); F_y alike.
struct SubFinals {
    uint4 F, G, H;
};

__device__ __forceinline__ SubFinals subtree_finals(const Kid& k, int sh, const uint4& P) {
    const uint4 A = k.L0, B = k.L1, Cc = k.L2;
    const uint4 mab = min4(A, B);
    const uint32_t ePa = ~code_ne(P, A), ePb = ~code_ne(P, B), ePc = ~code_ne(P, Cc);
    SubFinals r;
    if (sh == 1) {
        const uint32_t in_x = ~code_ne(Cc, A) | ~code_ne(Cc, B);
        const uint32_t hit = ePc | (~in_x & (ePa | ePb));
        r.F = sel4(hit, P, sel4(in_x, Cc, min4(mab, Cc)));
        r.H = r.F;
    } else {
        const uint4 D = k.L3;
        const uint32_t ia = ~code_ne(A, Cc) | ~code_ne(A, D), ib = ~code_ne(B, Cc) | ~code_ne(B, D), nz = ia | ib;
        const uint32_t hit = (nz & ((ePa & ia) | (ePb & ib))) | (~nz & (ePa | ePb | ePc | ~code_ne(P, D)));
        const uint4 mcd = min4(Cc, D);
        r.F = sel4(hit, P, sel4(nz, sel4(ia & ib, mab, sel4(ia, A, B)), min4(mab, mcd)));
        r.H = sel4(~code_ne(r.F, Cc) | ~code_ne(r.F, D), r.F, mcd);
    }
    r.G = sel4(~code_ne(r.F, A) | ~code_ne(r.F, B), r.F, mab);
    return r;
}

// Sankoff finals inside an S2 / S3 child v given its parent's final P (src/fitchSankoff.cpp:
// 487-531 at v, then at its cherries, unit costs; leaves keep their codes).  Z0 = codes of
// the maximum child count, Z1 = one below it (see pm_sankoff.hip):
//   cherry x = (a, b): a == b: Z0 = {a}, Z1 = {};  else Z0 = {a, b}, Z1 = every other code.
//   v = (x, y): X & Y != {} ? Z0 = X & Y, Z1 = X ^ Y : Z0 = X | Y, Z1 = every other code
//   (S2: y = {c}).  A node's final: P if P in Z0, else the lowest of Z0 -- or P when P is in
//   Z1 and below that lowest code (ties go to the lowest index).
__device__ __forceinline__ uint4 cherry_final_sankoff(const uint4& A, const uint4& B, const uint4& F) {
    const uint4 mab = min4(A, B);
    const uint4 open = sel4(~code_ne(F, A) | ~code_ne(F, B), F, min4(mab, F));   // a != b: Z1 = the rest
    return sel4(~code_ne(A, B), A, open);
}

__device__ __forceinline__ SubFinals subtree_finals_sankoff(const Kid& k, int sh, const uint4& P) {
    const uint4 A = k.L0, B = k.L1, Cc = k.L2;
    const uint4 mab = min4(A, B);
    const uint32_t pX = ~code_ne(P, A) | ~code_ne(P, B);
    SubFinals r;
    if (sh == 1) {
        const uint32_t inx = ~code_ne(Cc, A) | ~code_ne(Cc, B);
        // c in X: Z0 = {c}, Z1 = X \ {c};  else Z0 = {a, b, c}, Z1 = the rest
        const uint4 f_in = sel4(pX & code_less(&P.x, &Cc.x), P, Cc);
        const uint4 f_out = sel4(pX | ~code_ne(P, Cc), P, min4(min4(mab, Cc), P));
        r.F = sel4(inx, f_in, f_out);
        r.H = r.F;
    } else {
        const uint4 D = k.L3;
        const uint4 mcd = min4(Cc, D);
        const uint32_t ia = ~code_ne(A, Cc) | ~code_ne(A, D), ib = ~code_ne(B, Cc) | ~code_ne(B, D), nz = ia | ib;
        const uint32_t pY = ~code_ne(P, Cc) | ~code_ne(P, D);
        const uint32_t p_z0 = (~code_ne(P, A) & ia) | (~code_ne(P, B) & ib);
        const uint4 low = sel4(ia & ib, mab, sel4(ia, A, B));
        const uint4 f_nz = sel4(p_z0 | ((pX ^ pY) & code_less(&P.x, &low.x)), P, low);
        const uint4 f_z = sel4(pX | pY, P, min4(min4(mab, mcd), P));
        r.F = sel4(nz, f_nz, f_z);
        r.H = cherry_final_sankoff(Cc, D, r.F);
    }
    r.G = cherry_final_sankoff(A, B, r.F);
    return r;
}

template <class Args>
__device__ __forceinline__ void emit_code(const Args& a, Emit& em, int lane, uint32_t node, uint32_t D, uint32_t site0,
                                          const uint4& c, const uint4& pc) {
    const uint32_t p4[4] = {pc.x, pc.y, pc.z, pc.w};
    emit_stream(a, em, lane, node, D, site0, c.x, c.y, c.z, c.w, p4);
}

// Records of an S2 / S3 subtree: v, x, a, b, c (S2: c under v) [, y, d]; ids = the
// child's node id, then its leaves' (id[1..4]), cherries ix / iy.
template <Mode M, class Args>
__device__ __forceinline__ void subtree_emit(const Args& a, Emit& em, int lane, const int32_t* id, int32_t ix, int32_t iy,
                                             const Kid& k, int sh, uint32_t valid, const uint32_t* Fn, uint32_t site0) {
    const uint4 P = make_uint4(Fn[0], Fn[1], Fn[2], Fn[3]);
    const SubFinals f = M == Mode::kSankoff ? subtree_finals_sankoff(k, sh, P) : subtree_finals(k, sh, P);
    const uint32_t msk = valid & k.m0;
    emit_code(a, em, lane, (uint32_t)id[0], msk & code_ne(f.F, P), site0, f.F, P);
    emit_code(a, em, lane, (uint32_t)ix, msk & code_ne(f.G, f.F), site0, f.G, f.F);
    emit_code(a, em, lane, (uint32_t)id[1], msk & code_ne(k.L0, f.G), site0, k.L0, f.G);
    emit_code(a, em, lane, (uint32_t)id[2], msk & code_ne(k.L1, f.G), site0, k.L1, f.G);
    const uint4 pc = sh == 1 ? f.F : f.H;
    emit_code(a, em, lane, (uint32_t)id[3], msk & code_ne(k.L2, pc), site0, k.L2, pc);
    if (sh == 2) {
        emit_code(a, em, lane, (uint32_t)iy, msk & code_ne(f.H, f.F), site0, f.H, f.F);
        emit_code(a, em, lane, (uint32_t)id[4], msk & code_ne(k.L3, f.H), site0, k.L3, f.H);
    }
}

// What a child of a node with final codes Fn records: a leaf its changed sites; a virtual
// child (one or two leaves, prefetched) its final F, its own changed sites (against Fn) and
// its leaves' (against F).  A virtual child's final:
//   Fitch   (src/fitchSankoff.cpp:115-123 on the union set): Fn if among the leaves'
//           codes, else the lowest of them.
//   Sankoff (:513-530): the optimal codes are the present leaves' codes; every other code
//           is one above optimal unless both leaves are present with one code (then two
//           above).  So Fn wins if among the leaves' codes, otherwise the lowest of them
//           and -- when Fn is one above optimal -- Fn (ties go to the lowest index).
// ids: the child's id, then its leaves'.
template <Mode M, class Args>
__device__ __forceinline__ void kid_emit(const Args& a, Emit& em, int lane, const Kid& k, uint32_t id0, uint32_t id1,
                                         uint32_t id2, uint32_t valid, const uint32_t* Fn, uint32_t site0) {
    if (k.enc < 0) {
        emit_stream(a, em, lane, id0, valid & k.m0 & diff4(k.L0, Fn), site0, k.L0.x, k.L0.y, k.L0.z, k.L0.w, Fn);
        return;
    }
    if (M == Mode::kBlockFitch || !(k.enc & kVirtualBit)) return;
    uint32_t low[4] = {0, 0, 0, 0}, have = 0, hit = 0;
    virt_fold(k.L0, k.m0, Fn, low, have, hit);
    virt_fold(k.L1, k.m1, Fn, low, have, hit);
    if (M == Mode::kSankoff) {
        // Fn is one above optimal (in Z1) unless both leaves are present with equal codes
        const uint32_t z1_has_fn =
            (k.m0 ^ k.m1) |
            (k.m0 & k.m1 & ((k.L0.x ^ k.L1.x) | (k.L0.y ^ k.L1.y) | (k.L0.z ^ k.L1.z) | (k.L0.w ^ k.L1.w)));
        const uint32_t take = z1_has_fn & code_less(Fn, low);
#pragma unroll
        for (int j = 0; j < 4; ++j) low[j] = bsel(take, Fn[j], low[j]);
    }
    uint32_t F[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) F[j] = bsel(hit, Fn[j], low[j]);
    const uint32_t self = have & valid & ((F[0] ^ Fn[0]) | (F[1] ^ Fn[1]) | (F[2] ^ Fn[2]) | (F[3] ^ Fn[3]));
    emit_stream(a, em, lane, id0, self, site0, F[0], F[1], F[2], F[3], Fn);
    emit_stream(a, em, lane, id1, valid & k.m0 & diff4(k.L0, F), site0, k.L0.x, k.L0.y, k.L0.z, k.L0.w, F);
    if (k.vl.y >= 0)
        emit_stream(a, em, lane, id2, valid & k.m1 & diff4(k.L1, F), site0, k.L1.x, k.L1.y, k.L1.z, k.L1.w, F);
}

// Where a complex lane's final goes: the record's simple area past the simple lanes' codes
// (slots popc(s) .. popc(s) + popc(x) - 1 are never used by the set, x and s being
// disjoint), so the set's complex planes stay intact after the node's pre-order step and a
// descendant's wave in the same launch may still recompute the node's final from them
// (k_down level groups).
__device__ __forceinline__ uint32_t final_slot(const RecMask& m) {
    return (uint32_t)__builtin_popcountll(m.s) + lanes_below(m.x);
}

// Compact finals.  After an internal node's pre-order step its final codes are: the
// root's in root_final; a complex lane's in its final_slot of the record's simple area;
// every other lane's its record code -- a single-code set resolves to
// its code whatever the parent holds (src/fitchSankoff.cpp:115-123 and :513-530 with
// Z0 = {c}, Z1 = {}).  Only complex lanes are written; a child reads 16 B per lane only
// for its parent's non-consensus lanes, locating them with the parent's x / s masks
// (pushed into its own mask record by the post-order pass, RecMask::px / ps).
__device__ __forceinline__ uint4 rec_final(const uint4* p, const RecMask& m, int lane, const uint4* cons, int64_t word) {
    const uint4* src = ((m.x >> lane) & 1ull) ? p + final_slot(m)
                                              : ((m.s >> lane) & 1ull) ? p + lanes_below(m.s) : cons + word;
    return *src;
}

// The parent's final for a node whose own masks (with the pushed parent masks) are `m`.
template <int REC>
__device__ __forceinline__ uint4 parent_final(const DownArgs& a, int32_t parent, const RecMask& m, int tile, int lane,
                                              int64_t word) {
    if (parent == a.root_dense) return a.root_final[word];
    const RecMask pm{m.px, m.ps, 0, 0, 0};
    return rec_final(a.sets + ((size_t)parent * a.tiles + tile) * REC, pm, lane, a.cons, word);
}

// Any internal node's final, its own masks loaded here (tail kernel).
template <int REC>
__device__ __forceinline__ uint4 node_final(const DownArgs& a, int32_t node, int tile, int lane, int64_t word) {
    if (node == a.root_dense) return a.root_final[word];
    const size_t rec = (size_t)node * a.tiles + tile;
    return rec_final(a.sets + rec * REC, rec_mask(a.cmask, rec), lane, a.cons, word);
}

__device__ __forceinline__ void store_final(const DownArgs& a, bool is_root, uint4* p, const RecMask& m, int lane,
                                            int64_t word, const uint32_t* F) {
    if (is_root) a.root_final[word] = make_uint4(F[0], F[1], F[2], F[3]);
    else if ((m.x >> lane) & 1ull) store_stream(p + final_slot(m), make_uint4(F[0], F[1], F[2], F[3]));
}

// The node's final codes F (code planes) and the sites where it is resolved (pres), from
// its own set (Fitch: one-hot planes; Sankoff: Z0 / Z1) and its parent's final pc.
template <Mode M>
__device__ __forceinline__ void resolve_final(const DownArgs& a, bool is_root, int64_t word, const uint32_t* own,
                                              const uint32_t* z1, const uint32_t* pc, uint32_t* F, uint32_t& pres) {
    if constexpr (M == Mode::kFitch || M == Mode::kBlockFitch) {
        // "parent code in own set" (hit) by a multiplexer on the parent's code bits, the
        // lowest code of the set by a binary search; state 0: subtree absent, skipped
        // (:101-103, :136-138)
        uint32_t c[4];
        pres = lowest_code_planes(own, c);
        // root: lowest code of its set; otherwise (and always for blocks, :249-264)
        // parent & own ? parent : lowest(own)   (src/fitchSankoff.cpp:98-123)
        const bool generic = !is_root || M == Mode::kBlockFitch;
        const uint32_t hit = generic ? plane_at(own, pc) : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) F[j] = bsel(hit, pc[j], c[j]);
        if (M == Mode::kBlockFitch && is_root && a.forced) {   // defaultValue (:249-250)
            const uint4 f = a.forced[word];
            F[0] = f.x; F[1] = f.y; F[2] = f.z; F[3] = f.w;
            pres = ~0u;
        }
    } else {
        if (is_root && a.forced) {   // defaultState (src/fitchSankoff.cpp:492-493)
            const uint4 f = a.forced[word];
            F[0] = f.x; F[1] = f.y; F[2] = f.z; F[3] = f.w;
            pres = ~0u;
        } else {
            // Root: argmin = lowest optimal code (:495-507).  Otherwise the parent's code if
            // optimal (Z0), else the lowest of Z0 and -- if it is one above optimal (Z1) --
            // the parent's code (:513-530, ties to the lowest index); an all-INF subtree
            // (Z0 = Z1 = 0) stays unresolved.
            uint32_t c[4];
            const uint32_t any0 = lowest_code_planes(own, c);
            uint32_t hit = 0, z1hit = 0;
            if (!is_root) {
                hit = plane_at(own, pc);
                z1hit = plane_at(z1, pc);
                const uint32_t take = z1hit & (~any0 | code_less(pc, c));
#pragma unroll
                for (int j = 0; j < 4; ++j) c[j] = bsel(take, pc[j], c[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) F[j] = bsel(hit, pc[j], c[j]);
            pres = any0 | z1hit;
        }
    }
}

// Pre-order + assignment for one node and its leaf children.  Final state:
//   Fitch   (src/fitchSankoff.cpp:96-129): root -> lowest code of its set; otherwise
//           parent if parent & own, else lowest(own); own == 0 stays unresolved.
//   Sankoff (src/fitchSankoff.cpp:487-531): root -> forced code or lowest optimal code
//           (Z0); otherwise parent if optimal, else the lowest of Z0 and (parent if it is
//           one above optimal, Z1); an all-INF subtree (Z0 == 0) stays unresolved (-1).
// Leaf children keep their own code in both modes.  Mutations (:131-171, :676-703):
// parent code 0 -> NI, child code 0 -> ND, else NS.
// Every load that does not depend on the parent's final (own set, parent final, the first
// two children's words) is issued before any of them is consumed.
// DENSE: the level's nodes are the dense indices dense_base + item (DevTree down order),
// so the record masks are fetched alongside the descriptor, not after it.

// SUB: subtree form (Fitch, every leaf present) -- the first two children may be S2 / S3
// subtrees, whose inner finals and records this wave produces (subtree_prepare).
#ifndef PM_SUB_DOWN_WAVES
#define PM_SUB_DOWN_WAVES 5
#endif
// One pre-order wave: node `n` (its descriptor d) x tile; `salt` spreads the waves over the
// record shards; `stage` is the wave's LDS entry area (kEntryQuads, see emit_stream).
// GROUP: the launch holds up to kGroupLevels consecutive levels; a wave of
// the group's level g > 0 does not wait for its ancestors' finals to be stored -- it
// recomputes them top down, each from the ancestor's set (intact: final_slot) and the final
// above it, starting from the last final stored before the launch (descriptor: pad0 =
// grandparent, pad1 = great-grandparent; the fourth level's top ancestor's parent is one
// scalar load beside the mask loads), so g + 1 levels cost one launch.
#ifndef PM_GROUP_LEVELS
#define PM_GROUP_LEVELS 4
#endif
constexpr int kGroupLevels = PM_GROUP_LEVELS;
static_assert(kGroupLevels >= 2 && kGroupLevels <= 4, "level groups: 2 to 4 levels");
template <Mode M, bool AP, bool SUB, bool GROUP = false>
__device__ __forceinline__ void down_node(const DownArgs& a, const NodeDesc& d, int32_t n, uint32_t salt, int tile,
                                          int lane, uint4* stage, int gen = 0) {
    const int32_t parent = d.parent, e0 = d.e0, e1 = d.e1;
    const uint32_t node_id = (uint32_t)a.internal_id[n];   // (scalar load, in flight with the rest)
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t valid = valid_mask(a, word);
    const bool is_root = parent < 0;

    constexpr int REC = M == Mode::kSankoff ? kSankoffRec : kFitchRec;
    const size_t rec = (size_t)n * a.tiles + tile;
    const RecMask m = rec_mask(a.cmask, rec);
    uint4* const p = a.sets + rec * REC;
    uint32_t own[16], pc[4], F[4];
    if (GROUP && gen > 0) {
        // ancestors inside the group, top first: chain[3 - gen .. 2], chain[2] = parent
        const int32_t chain[3] = {d.pad1, d.pad0, parent};
        // the top one's parent, whose final is stored (-1: the top one is the root)
        const int32_t above = gen == 1 ? d.pad0 : gen == 2 ? d.pad1 : d.pad1 >= 0 ? a.parent_dense[d.pad1] : -1;
        // every ancestor's masks first (uniform loads, all in flight together), then each
        // set: the chain waits on one round trip per ancestor, not two
        RecMask mv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < gen) mv[k] = rec_mask(a.cmask, (size_t)chain[k + 3 - gen] * a.tiles + tile);
        uint4 q;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= gen) break;
            const size_t vrec = (size_t)chain[k + 3 - gen] * a.tiles + tile;
            const bool vroot = k == 0 && above < 0;
            // (the top one: the final above it, from its pushed (px, ps))
            if (k == 0) q = vroot ? a.cons[word] : parent_final<REC>(a, above, mv[0], tile, lane, word);
            uint32_t vown[16], vz1[16], gc[4] = {q.x, q.y, q.z, q.w}, VF[4], vpres;
            if constexpr (M == Mode::kSankoff) {
                load_sankoff(a.sets + vrec * REC, mv[k], a.cons, lane, word, vown, vz1, !vroot);
            } else {
                SetFetch f;
                fetch_fitch_set(a.sets + vrec * REC, mv[k], a.cons, lane, word, f);
                expand_fitch_set(f, vown);
            }
            resolve_final<M>(a, vroot, word, vown, vz1, gc, VF, vpres);
            q = make_uint4(VF[0], VF[1], VF[2], VF[3]);
        }
        pc[0] = q.x; pc[1] = q.y; pc[2] = q.z; pc[3] = q.w;
    } else {
        const uint4 q = is_root ? a.cons[word] : parent_final<REC>(a, parent, m, tile, lane, word);
        pc[0] = q.x; pc[1] = q.y; pc[2] = q.z; pc[3] = q.w;
    }
    // Fitch, every leaf present: a leaf child differs from this node's final only at its
    // complex lanes, a virtual child only there and where its own leaves disagree (mask
    // words 6, 7: store_kid_masks) -- not at the lanes another child made dirty
    uint64_t k0 = m.d, k1 = m.d;
    // SUB (PM_OPT_SUB_DOWN): the descriptor keeps S2 / S3 children, done here instead of in
    // the tail: an S child's lanes are the ones its parent's post-order wave pushed into its
    // own mask record (word 5); words 6 / 7 follow the descriptor without S children
    // (fitch_up_node's store_kid_masks), so a second child's are word 6 after an S first one
    const bool s0 = SUB && kid_shape(d.c0) != 0, s1 = SUB && e1 - e0 > 1 && kid_shape(d.c1) != 0;
    if constexpr (M == Mode::kFitch && AP) {
        const uint64_t* q = a.cmask + kMaskWords * rec;
        auto sub_lanes = [&](int32_t c) { return a.cmask[kMaskWords * ((size_t)(c & kDenseMask) * a.tiles + tile) + 5]; };
        k0 = d.c0 < 0 ? m.x : s0 ? sub_lanes(d.c0) : q[6];
        k1 = d.c1 < 0 ? m.x : s1 ? sub_lanes(d.c1) : s0 ? q[6] : q[7];
    }
    const bool dirty0 = is_root || ((k0 >> lane) & 1ull);
    const bool dirty1 = is_root || ((k1 >> lane) & 1ull);
    Kid kids[2];
    if (s0) kid_fetch_s(a, d.c0, word, dirty0, kids[0]);
    else kid_fetch<M, AP, false>(a, d.c0, make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), word, dirty0, kids[0]);
    if (s1) kid_fetch_s(a, d.c1, word, dirty1, kids[1]);
    else if (e1 - e0 > 1) kid_fetch<M, AP, false>(a, d.c1, make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]), word, dirty1, kids[1]);
    uint32_t z1[16];
    if constexpr (M == Mode::kSankoff) {
        load_sankoff(p, m, a.cons, lane, word, own, z1, !is_root);
    } else {
        SetFetch f;
        fetch_fitch_set(p, m, a.cons, lane, word, f);
        __builtin_amdgcn_sched_barrier(0);   // every load above is issued before any is consumed
        expand_fitch_set(f, own);
    }
    uint32_t pres;
    resolve_final<M>(a, is_root, word, own, z1, pc, F, pres);
    store_final(a, is_root, p, m, lane, word, F);

    if (is_root) {
        for (int b = 0; b < 32; ++b) {
            const int64_t site = word * 32 + b;
            if (site < a.sites)
                a.root_code[site] = ((pres >> b) & 1u) ? (uint8_t)code_at(F[0], F[1], F[2], F[3], b) : (uint8_t)255;
        }
    }

    const uint32_t self_diff = pres & valid & ((F[0] ^ pc[0]) | (F[1] ^ pc[1]) | (F[2] ^ pc[2]) | (F[3] ^ pc[3]));
    // records: the node's and its first two children's streams, staged and expanded
    Emit em{stage, shard_of(salt, tile), 0u, 0u};
    const uint32_t site0 = (uint32_t)(word * 32);
    emit_stream(a, em, lane, node_id, self_diff, site0, F[0], F[1], F[2], F[3], pc);
    // (an S child's node ids come with its tail descriptor: item = dense index - sbase)
    if (s0) {
        const TailDesc& t = a.tail[(d.c0 & kDenseMask) - a.sbase];
        subtree_emit<M>(a, em, lane, t.id, t.ix, t.iy, kids[0], kid_shape(d.c0), valid, F, site0);
    } else {
        kid_emit<M>(a, em, lane, kids[0], kids[0].id0, kids[0].id1, kids[0].id2, valid, F, site0);
    }
    if (s1) {
        const TailDesc& t = a.tail[(d.c1 & kDenseMask) - a.sbase];
        subtree_emit<M>(a, em, lane, t.id, t.ix, t.iy, kids[1], kid_shape(d.c1), valid, F, site0);
    } else if (e1 - e0 > 1) {
        kid_emit<M>(a, em, lane, kids[1], kids[1].id0, kids[1].id1, kids[1].id2, valid, F, site0);
    }
    emit_flush<M != Mode::kSankoff>(a, em, lane);
}

// GROUP: items [split[g-1], split[g]) are the group's level g (split[-1] = 0, unused
// splits = count), dense from dense_g[g].
template <Mode M, bool AP, bool DENSE, bool SUB = false, bool GROUP = false>
#ifndef PM_SK_GROUP_WAVES
#define PM_SK_GROUP_WAVES 7
#endif
#ifndef PM_DOWN_WAVES
#define PM_DOWN_WAVES 8
#endif
#ifndef PM_SK_DOWN_WAVES
#define PM_SK_DOWN_WAVES 6
#endif
__global__ __launch_bounds__(kBlock, GROUP ? (M == Mode::kSankoff ? PM_SK_GROUP_WAVES : SUB ? PM_SUB_DOWN_WAVES : 8) : SUB ? PM_SUB_DOWN_WAVES : (M == Mode::kFitch && AP) ? PM_DOWN_WAVES : (M == Mode::kSankoff && AP) ? PM_SK_DOWN_WAVES : 1) void k_down(DownArgs a) {
    __shared__ uint4 stage[kWavesPerBlock][kEntryQuads];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    wave_item(wave, a.tiles, item, tile);
    if (item >= a.count) return;   // whole wave leaves together
    const NodeDesc& d = a.desc[item];
    const int gen = !GROUP ? 0 : (item >= a.split[0]) + (item >= a.split[1]) + (item >= a.split[2]);
    const int32_t first = gen == 0 ? 0 : a.split[gen > 0 ? gen - 1 : 0];
    const int32_t n = !DENSE ? d.node : (GROUP ? a.dense_g[gen] : a.dense_base) + (item - first);
    down_node<M, AP, SUB, GROUP>(a, d, n, (uint32_t)item, tile, lane, stage[wave], gen);
}

// Narrow pre-order levels (PM_OPT_NARROW; see k_fitch_up_band): levels [d0, d1) of the
// level table `level_off` (descriptor ranges) walked by one launch, one 1024-thread workgroup
// per tile, a workgroup barrier between levels.  `dense_base` (nullable): each level's first
// dense index when the level is one dense range.
// GROUP: kGroupLevels levels between barriers, the lower ones recomputing their ancestors'
// finals (down_node's level groups).
template <Mode M, bool AP, bool SUB = false, bool GROUP = false>
__global__ __launch_bounds__(kBandBlock) void k_down_band(DownArgs a, const int32_t* level_off, const int32_t* dense_base,
                                                          int32_t d0, int32_t d1) {
    __shared__ uint4 stage[kBandWaves][kEntryQuads];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int tile = blockIdx.x;
    constexpr int G = GROUP ? kGroupLevels : 1;
    for (int32_t l0 = d0; l0 < d1; l0 += G) {
        const int32_t l1 = min(l0 + G, d1);
        for (int32_t i = level_off[l0] + wave; i < level_off[l1]; i += kBandWaves) {
            int32_t l = l0;
            while (l + 1 < l1 && i >= level_off[l + 1]) ++l;
            const NodeDesc& d = a.desc[i];
            const int32_t base = dense_base ? dense_base[l] : -1;
            down_node<M, AP, SUB, GROUP>(a, d, base >= 0 ? base + (i - level_off[l]) : d.node, (uint32_t)i, tile, lane,
                                         stage[wave], l - l0);
        }
        __syncthreads();
    }
}

// Records of the leaf / virtual children beyond a node's second (polytomies), after the
// pre-order levels: wave = (tail item, tile), parent final read back (node_final).
// SUB: subtree form -- the S2 / S3 children are tail items too (their inner finals and
// records from the parent's final and their leaves, subtree_put), so the level kernels stay
// lean.
#ifndef PM_TAIL_WAVES
#define PM_TAIL_WAVES 6
#endif
template <Mode M, bool AP, bool SUB = false>
__global__ __launch_bounds__(kBlock, SUB ? PM_TAIL_WAVES : 1) void k_tail(DownArgs a) {
    __shared__ uint4 stage[kWavesPerBlock][kEntryQuads];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int32_t item;
    int tile;
    wave_item(wave, a.tiles, item, tile);
    if (item >= a.count) return;
    const TailDesc& t = a.tail[item];
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t valid = valid_mask(a, word);
    constexpr int REC = M == Mode::kSankoff ? kSankoffRec : kFitchRec;
    // the parent's (x, s, d) masks: an S2 / S3 item finds them in its own mask record, pushed
    // there by the parent's post-order wave (every lane dirty at the root), loaded beside the
    // descriptor; other items read the parent's record after the descriptor
    RecMask pm;
    bool proot;
    if (SUB && item < a.num_s) {
        const uint64_t* q = a.cmask + kMaskWords * ((size_t)(a.sbase + item) * a.tiles + tile);
        pm = RecMask{q[3], q[4], q[5], 0, 0};
        if (pm.d == 0) return;   // no dirty lane: the child holds the parent's code everywhere
        proot = t.parent == a.root_dense;
    } else {
        proot = t.parent == a.root_dense;
        pm = rec_mask(a.cmask, (size_t)t.parent * a.tiles + tile);
        if (leaf_rule<M, AP>(t.enc)) pm.d = pm.x;   // a leaf: the parent's complex lanes only
        if (!proot && pm.d == 0) return;
    }
    const size_t prec = (size_t)t.parent * a.tiles + tile;
    const bool dirty = proot || ((pm.d >> lane) & 1ull);
    Kid k;
    if (SUB && item < a.num_s) {   // an S2 / S3 node: its leaves' words in one 64-B row
        k.enc = t.enc;
        k.L0 = k.L1 = k.L2 = k.L3 = make_uint4(0, 0, 0, 0);
        k.m0 = k.m1 = 0;
        const uint4* q = sub_word(a.sub_planes, item, a.wpad, word);
        if (dirty) {
            k.L0 = q[0];
            k.L1 = q[1];
            k.L2 = q[2];
            k.m0 = k.m1 = ~0u;
        }
        if (dirty && kid_shape(t.enc) == 2) k.L3 = q[3];
    } else {
        kid_fetch<M, AP, SUB, false>(a, t.enc, make_int4(t.vl[0], t.vl[1], t.vl[2], t.vl[3]), word, dirty, k);
    }
    // the parent's final, dirty lanes only (elsewhere the child emits nothing)
    const uint4* fsrc = proot ? a.root_final + word
                              : ((pm.x >> lane) & 1ull) ? a.sets + prec * REC + final_slot(pm)
                              : ((pm.s >> lane) & 1ull) ? a.sets + prec * REC + lanes_below(pm.s) : a.cons + word;
    uint4 q = make_uint4(0, 0, 0, 0);
    if (dirty) q = *fsrc;
    const uint32_t F[4] = {q.x, q.y, q.z, q.w};
    // records: node ids from the descriptor
    Emit em{stage[wave], shard_of((uint32_t)item, tile), 0u, 0u};
    const uint32_t site0 = (uint32_t)(word * 32);
    if (SUB && kid_shape(t.enc)) subtree_emit<M>(a, em, lane, t.id, t.ix, t.iy, k, kid_shape(t.enc), valid, F, site0);
    else kid_emit<M>(a, em, lane, k, (uint32_t)t.id[0], (uint32_t)t.id[1], (uint32_t)t.id[2], valid, F, site0);
    emit_flush<M != Mode::kSankoff>(a, em, lane);
}

// ---- LDS-staged post-order sweeps: what the Fitch and Sankoff sweep kernels share (schedule:
// pm_cluster.cpp).  One wave = one (cluster, tile): the cluster's nodes in depth-first
// post-order, one per step; a child of the same cluster comes from its LDS slot (16 planes:
// the Fitch set / the Sankoff Z0, 4 KiB per (node, tile)).
struct ClArgs {
    const NodeDesc* items;
    const int32_t* wg_off;
    const int32_t* slot_of;
    const int32_t* pslot;   // per item: the parent's up slot (parent in a later band), -1
    int32_t upm_base;       // up slots of item i: UpArgs::upm item upm_base + i (after the level items')
    int32_t wg0;
};
typedef uint4 ClSlots[kClSlots][4][kWave];

__device__ __forceinline__ void slot_read(const ClSlots& S, int s, int lane, uint32_t* x) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = S[s][q][lane];
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ void slot_write(ClSlots& S, int s, int lane, const uint32_t* x) {
#pragma unroll
    for (int q = 0; q < 4; ++q) S[s][q][lane] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
}

// An item's descriptor, up slots and up-slot target, fetched as one VECTOR load (lane k < 16:
// descriptor dword k; 16..23: the up slots' dwords; 24..: the target) and moved to scalar
// registers one round later: a scalar load in flight would hold every LDS barrier of the round
// (s_waitcnt lgkmcnt(0) covers both).
struct ClMeta {
    NodeDesc d;
    UpSlots s;
    int32_t ps;
};

__device__ __forceinline__ uint32_t cl_meta_load(const UpArgs& a, const ClArgs& c, int32_t it, int tile, int lane) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(c.pslot + it);
    if (lane < 16) src = reinterpret_cast<const uint32_t*>(c.items + it) + lane;
    else if (lane < 24) src = reinterpret_cast<const uint32_t*>(a.upm + ((size_t)(c.upm_base + it) * a.tiles + tile) * 4) + (lane - 16);
    return *src;
}

__device__ __forceinline__ void cl_meta_get(uint32_t m, ClMeta& x) {
    int32_t* p = reinterpret_cast<int32_t*>(&x.d);
#pragma unroll
    for (int k = 0; k < 16; ++k) p[k] = __builtin_amdgcn_readlane((int)m, k);
    auto u64 = [&](int k) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)m, k + 1) << 32) | (uint32_t)__builtin_amdgcn_readlane((int)m, k);
    };
    x.s = UpSlots{u64(16), u64(18), u64(20), u64(22)};
    x.ps = __builtin_amdgcn_readlane((int)m, 24);
}

// ---- LDS-staged pre-order sweeps over the post-order's clusters (plan_cluster_down) -------
// One wave = one (cluster, tile), the bands top-down: the cluster's nodes in depth-first
// pre-order, one per step -- down_node's work for the node and its first two (non-S2 / S3)
// children (Fitch: src/fitchSankoff.cpp:96-171; Sankoff: :487-531, :676-703), with the parent's final from the LDS slot its own
// step wrote (the cluster root's from memory, stored by an earlier band), its own final into a
// slot for its children and, compact, to memory for the tail launch.  Records are staged in
// the wave's LDS entries across steps and flushed when full (one returned atomic per 128
// entries, not per node).  The step's descriptor, masks and record node ids come from vector
// loads two / one steps ahead; its own record code, the cluster root's parent final and its
// children's dirty leaf words one step ahead.
struct ClDownArgs {
    const NodeDesc* items;
    const int32_t* wg_off;
    int32_t wg0;
};
typedef uint4 ClFinals[kClFSlots][kWave];

// (vector) the item's descriptor: lane k < 16 = dword k
__device__ __forceinline__ uint32_t cld_desc_load(const ClDownArgs& c, int32_t it, int lane) {
    return reinterpret_cast<const uint32_t*>(c.items + it)[lane & 15];
}

// (vector) the node's masks (lanes 0..15: 8 u64 words), its node id (16), its first two
// children's record node ids (17..19, 20..22: the child, a leaf-parent's leaves)
__device__ __forceinline__ uint32_t cld_mask_load(const DownArgs& a, const NodeDesc& d, int tile, int lane) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.cmask + kMaskWords * ((size_t)d.node * a.tiles + tile)) + (lane & 15);
    const int k = lane >= 20 ? 1 : 0, j = lane - (k ? 20 : 17);
    const int32_t enc = k ? d.c1 : d.c0;
    const int32_t v0 = k ? d.vl1[0] : d.vl0[0], v1 = k ? d.vl1[1] : d.vl0[1];
    const bool has = !k || d.e1 - d.e0 > 1;
    if (lane == 16) src = reinterpret_cast<const uint32_t*>(a.internal_id + d.node);
    else if (lane >= 17 && lane < 23 && has) {
        if (enc < 0) src = reinterpret_cast<const uint32_t*>(a.leaf_id + (j == 0 ? -enc - 1 : 0));
        else if (enc & kVirtualBit)
            src = j == 0 ? reinterpret_cast<const uint32_t*>(a.internal_id + (enc & kDenseMask))
                         : reinterpret_cast<const uint32_t*>(a.leaf_id + (j == 1 ? v0 : v1 >= 0 ? v1 : v0));
    }
    return *src;
}

struct ClDownMeta {
    NodeDesc d;
    RecMask m;
    uint64_t w6, w7;
    uint32_t id, kid[2][3];
};

__device__ __forceinline__ void cld_desc_get(uint32_t v, NodeDesc& d) {
    int32_t* p = reinterpret_cast<int32_t*>(&d);
#pragma unroll
    for (int k = 0; k < 16; ++k) p[k] = __builtin_amdgcn_readlane((int)v, k);
}

__device__ __forceinline__ void cld_mask_get(uint32_t v, ClDownMeta& x) {
    auto u64 = [&](int k) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)v, 2 * k + 1) << 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 2 * k);
    };
    x.m = RecMask{u64(0), u64(1), u64(2), u64(3), u64(4)};
    x.w6 = u64(6);
    x.w7 = u64(7);
    x.id = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j) x.kid[k][j] = (uint32_t)__builtin_amdgcn_readlane((int)v, 17 + 3 * k + j);
}

// A step's loads issued one step ahead: its record's code word, the cluster root's parent final,
// its first two children's leaf words at their dirty lanes.
struct ClDownFetch {
    uint4 code, pf, cxb;   // (cxb: compact records' B word)
    Kid k0, k1;
};

template <Mode M>
__device__ __forceinline__ void cld_issue(const DownArgs& a, const ClDownMeta& x, int tile, int lane, int64_t word,
                                          ClDownFetch& f) {
    constexpr int REC = M == Mode::kSankoff ? kSankoffRec : kFitchRec;
    constexpr bool CX = M == Mode::kFitch && kCxCompact;
    const NodeDesc& d = x.d;
    const bool is_root = d.parent < 0;
    const uint4* p = a.sets + ((size_t)d.node * a.tiles + tile) * REC;
    f.code = rec_code_all<CX>(p, x.m, lane, a.cons, word);
    if constexpr (CX) f.cxb = cx_b_load(p, x.m, lane, a.cons);
    if (d.pad0 < 0) f.pf = is_root ? a.cons[word] : parent_final<REC>(a, d.parent, x.m, tile, lane, word);
    // Fitch, every leaf present: a leaf child differs from the final only at the complex lanes,
    // a virtual one there and where its own leaves disagree (mask words 6, 7); Sankoff: the
    // node's dirty lanes (see down_node)
    const uint64_t k0 = M == Mode::kFitch ? (d.c0 < 0 ? x.m.x : x.w6) : x.m.d;
    const uint64_t k1 = M == Mode::kFitch ? (d.c1 < 0 ? x.m.x : x.w7) : x.m.d;
    kid_fetch<M, true, false, false>(a, d.c0, make_int4(d.vl0[0], d.vl0[1], d.vl0[2], d.vl0[3]), word,
                                     is_root || ((k0 >> lane) & 1ull), f.k0);
    if (d.e1 - d.e0 > 1)
        kid_fetch<M, true, false, false>(a, d.c1, make_int4(d.vl1[0], d.vl1[1], d.vl1[2], d.vl1[3]), word,
                                         is_root || ((k1 >> lane) & 1ull), f.k1);
}

template <Mode M>
__device__ __forceinline__ void cld_step(const DownArgs& a, const ClDownMeta& x, const ClDownFetch& f, ClFinals& FS, Emit& em,
                                         int tile, int lane, int64_t word, uint32_t valid) {
    constexpr int REC = M == Mode::kSankoff ? kSankoffRec : kFitchRec;
    const NodeDesc& d = x.d;
    const bool is_root = d.parent < 0;
    uint4* const p = a.sets + ((size_t)d.node * a.tiles + tile) * REC;
    uint32_t own[16], z1[16];
    onehot_from_code(f.code.x, f.code.y, f.code.z, f.code.w, ~0u, own);
    if constexpr (M == Mode::kSankoff) {   // (load_sankoff: a complex lane's Z0 and Z1 planes)
#pragma unroll
        for (int v = 0; v < 16; ++v) z1[v] = 0u;
        if ((x.m.x >> lane) & 1ull) {
            const uint32_t k = lanes_below(x.m.x);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 w = load_rec(p + kWave + q * kWave + k);
                own[4 * q] = w.x; own[4 * q + 1] = w.y; own[4 * q + 2] = w.z; own[4 * q + 3] = w.w;
            }
            if (!is_root) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 w = load_rec(p + 5 * kWave + q * kWave + k);
                    z1[4 * q] = w.x; z1[4 * q + 1] = w.y; z1[4 * q + 2] = w.z; z1[4 * q + 3] = w.w;
                }
            }
        }
    } else if constexpr (kCxCompact) {
        cx_decode(own, f.code, f.cxb, (x.m.x >> lane) & 1ull, p, x.m.x);
    } else if (x.m.x != 0 && ((x.m.x >> lane) & 1ull)) {   // a complex lane: its 16 planes
        const uint4* q = p + kWave + lanes_below(x.m.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 w = load_rec(q + j * kWave);
            own[4 * j] = w.x; own[4 * j + 1] = w.y; own[4 * j + 2] = w.z; own[4 * j + 3] = w.w;
        }
    }
    const uint4 q = d.pad0 >= 0 ? FS[d.pad0][lane] : f.pf;
    const uint32_t pc[4] = {q.x, q.y, q.z, q.w};
    uint32_t F[4], pres;
    resolve_final<M>(a, is_root, word, own, M == Mode::kSankoff ? z1 : nullptr, pc, F, pres);
    store_final(a, is_root, p, x.m, lane, word, F);
    if (d.pad1 >= 0) FS[d.pad1][lane] = make_uint4(F[0], F[1], F[2], F[3]);
    if (is_root) {
        for (int b = 0; b < 32; ++b) {
            const int64_t site = word * 32 + b;
            if (site < a.sites)
                a.root_code[site] = ((pres >> b) & 1u) ? (uint8_t)code_at(F[0], F[1], F[2], F[3], b) : (uint8_t)255;
        }
    }
    const uint32_t self_diff = pres & valid & ((F[0] ^ pc[0]) | (F[1] ^ pc[1]) | (F[2] ^ pc[2]) | (F[3] ^ pc[3]));
    const uint32_t site0 = (uint32_t)(word * 32);
    emit_stream(a, em, lane, x.id, self_diff, site0, F[0], F[1], F[2], F[3], pc);
    kid_emit<M>(a, em, lane, f.k0, x.kid[0][0], x.kid[0][1], x.kid[0][2], valid, F, site0);
    if (d.e1 - d.e0 > 1) kid_emit<M>(a, em, lane, f.k1, x.kid[1][0], x.kid[1][1], x.kid[1][2], valid, F, site0);
}

#ifndef PM_CLD_WAVES
#define PM_CLD_WAVES 3
#endif
template <Mode M>
__global__ __launch_bounds__(kWave, PM_CLD_WAVES) void k_down_cluster(DownArgs a, ClDownArgs c) {
    __shared__ ClFinals FS;
    __shared__ uint4 stage[kEntryQuads];
    const int lane = threadIdx.x;
    const int32_t b = (int32_t)blockIdx.x;
    const int32_t wl = b / a.tiles;
    const int tile = b - wl * a.tiles;
    const int32_t i0 = c.wg_off[c.wg0 + wl], steps = c.wg_off[c.wg0 + wl + 1] - i0;
    const int64_t word = (int64_t)tile * kWave + lane;
    const uint32_t valid = valid_mask(a, word);
    Emit em{stage, shard_of((uint32_t)(c.wg0 + wl), tile), 0u, 0u};
    // pipeline: descriptors three steps ahead (vector loads), masks / ids two, data one
    ClDownMeta X0, X1;
    ClDownFetch fA, fB;
    NodeDesc dn;
    cld_desc_get(cld_desc_load(c, i0, lane), X0.d);
    cld_mask_get(cld_mask_load(a, X0.d, tile, lane), X0);
    cld_issue<M>(a, X0, tile, lane, word, fA);
    uint32_t vm1 = 0u, vd2 = 0u;
    if (steps > 1) {
        cld_desc_get(cld_desc_load(c, i0 + 1, lane), X1.d);
        vm1 = cld_mask_load(a, X1.d, tile, lane);
    }
    if (steps > 2) vd2 = cld_desc_load(c, i0 + 2, lane);
    for (int32_t r = 0; r < steps; r += 2) {
        // step r (X0, fA); step r + 1's data into fB; step r + 2's masks; step r + 3's descriptor
        const uint32_t vd3 = r + 3 < steps ? cld_desc_load(c, i0 + r + 3, lane) : 0u;
        uint32_t vm2 = 0u;
        if (r + 2 < steps) {
            cld_desc_get(vd2, dn);
            vm2 = cld_mask_load(a, dn, tile, lane);
        }
        if (r + 1 < steps) {
            cld_mask_get(vm1, X1);
            cld_issue<M>(a, X1, tile, lane, word, fB);
        }
        cld_step<M>(a, X0, fA, FS, em, tile, lane, word, valid);
        if (r + 1 >= steps) break;
        // step r + 1 (X1, fB); step r + 2's data into fA; step r + 3's masks; step r + 4's descriptor
        const uint32_t vd4 = r + 4 < steps ? cld_desc_load(c, i0 + r + 4, lane) : 0u;
        NodeDesc d3 = dn;
        uint32_t vm3 = 0u;
        if (r + 3 < steps) {
            cld_desc_get(vd3, d3);
            vm3 = cld_mask_load(a, d3, tile, lane);
        }
        if (r + 2 < steps) {
            X0.d = dn;
            cld_mask_get(vm2, X0);
            cld_issue<M>(a, X0, tile, lane, word, fA);
        }
        cld_step<M>(a, X1, fB, FS, em, tile, lane, word, valid);
        X1.d = d3;
        vm1 = vm3;
        vd2 = vd4;
    }
    emit_flush<M != Mode::kSankoff>(a, em, lane);
}

}  // namespace PM_KNS
}  // namespace pm
