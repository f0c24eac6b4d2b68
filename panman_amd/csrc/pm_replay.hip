// pm_replay.hip -- root-to-leaf mutation replay for FASTA extraction (gfx950).
//
// Restates the per-leaf sequence reconstruction of Tree::printFASTAUltraFast
// (src/fasta.cpp:1993-2089) and printFASTAUltraFastHelper's mutation pass (:1795-1935):
// every leaf starts from the expanded block consensus (gap slots as '-') and applies the
// nucleotide mutations of each node on its root->leaf path in order, only for blocks that
// are present at the leaf (blockSequence, :1766-1787, :1842).
//
//   k_replay  one workgroup per (leaf, 8 column tiles of 16 KiB), tile after tile: the
//             consensus tile -> LDS (LDS-DMA), the path nodes' edits inside the tile written
//             by all four waves, absent blocks restored, one coalesced write of the tile:
//             1 B per leaf-column to HBM, the replay roofline of SURVEY.md §8d.  Any depth.
//
// Edit order.  printFASTAUltraFastHelper applies each path node's mutations root first, so
// of several edits of one column along a path the deepest wins.  The host marks an edit that
// rewrites a column some ancestor edits (kEditOverrides; the flag holds for every leaf below
// the node) and stores each node's edits as [plain | overriding], both column-sorted, with a
// per-(node, tile) table of where each part starts (ReplayDev::tile2).  Along one path the
// plain edits touch distinct columns (the shallowest edit of each column), so a tile's plain
// edits are written by all waves in any order; the overriding ones (rare: collisions of two
// edits on one path) are then gathered into an LDS list in path order and each is written
// unless a later list entry -- a deeper node -- has the same column.  Tiles with more than
// kOvrCap overriding edits apply them in path order instead, wave by wave.
#include "pm_bits.h"
#include "pm_internal.h"

namespace pm {
namespace {

// A chunk is up to 64 path nodes (lane = path node): their slice lengths in this tile and a
// wave prefix sum over them; a round gathers kEditsPerLane x 64 of the chunk's edits at once
// (one memory round trip).  2 per lane: 1.72 -> 1.67 ms at C5, 4.27 -> 3.45 ms on the
// SARS-like tree against 4 (r05, interleaved); 1: 1.74 / 3.41.
#ifndef PM_REPLAY_EPL
#define PM_REPLAY_EPL 2
#endif
constexpr int kEditsPerLane = PM_REPLAY_EPL;
constexpr int32_t kRound = kEditsPerLane * kWave;   // edits per wave-round

struct EditChunk {
    int cnt;
    int32_t lo;       // this lane's node: first edit of its slice
    int32_t len;      // this lane's node: slice length
    int32_t excl;     // exclusive prefix of the lengths
    int32_t total;    // edits in the chunk
};

__device__ __forceinline__ EditChunk edit_chunk_from(int cnt, int32_t lo, int32_t hi, int lane) {
    EditChunk c;
    c.cnt = cnt;
    c.lo = lo;
    c.len = lane < cnt ? hi - lo : 0;
    const int32_t incl = (int32_t)wave_inclusive_scan((uint32_t)c.len);
    c.total = __builtin_amdgcn_readlane(incl, kWave - 1);
    c.excl = incl - c.len;
    return c;
}

// A round in flight: col / chr straight from their loads (not combined with anything until
// they are written, so a prefetched round does not wait for its loads); g = the edit's index
// in the chunk, kNoEdit: none.
struct EditRound {
    uint32_t col[kEditsPerLane];
    uint32_t chr[kEditsPerLane];
    int32_t g[kEditsPerLane];
};
constexpr int32_t kNoEdit = -1;

__device__ __forceinline__ void edit_round(const ReplayDev& d, const EditChunk& c, int32_t base, int64_t c0, int lane,
                                           EditRound& r) {
    int32_t e[kEditsPerLane];
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        // edit g of the chunk belongs to the last path node whose slice starts at or before
        // g: a binary search over the lanes' prefix sums (64 nodes: 6 steps)
        const int32_t g = base + lane + j * kWave;
        int k_lo = 0, k_hi = c.cnt - 1;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const int mid = (k_lo + k_hi + 1) >> 1;
            if (__shfl(c.excl, mid) <= g) k_lo = mid;
            else k_hi = mid - 1;
        }
        r.g[j] = g < c.total ? g : kNoEdit;
        e[j] = __shfl(c.lo, k_lo) + (g - __shfl(c.excl, k_lo));
    }
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        r.col[j] = (uint32_t)c0;
        r.chr[j] = 0;
        if (r.g[j] != kNoEdit) {
            r.col[j] = d.edit_col[e[j]];
            r.chr[j] = d.edit_chr[e[j]];
        }
    }
}

__device__ __forceinline__ void edit_write_all(const EditRound& r, char* buf, int64_t c0) {
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j)
        if (r.g[j] != kNoEdit) buf[r.col[j] - c0] = (char)(r.chr[j] & 0x7fu);
}

// Fallback for a tile with more than kOvrCap overriding edits: a round's edits node by node
// in path order (the first pending edit -- edits are in path order -- names the next node;
// g orders the nodes as it orders the edits).  node_of: the path position of each edit.
__device__ __forceinline__ void edit_write_ordered(const EditRound& r, const int32_t* node_of, char* buf, int64_t c0) {
    const int lane = (int)threadIdx.x & (kWave - 1);
    uint64_t pend[kEditsPerLane];
    bool any = false;
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        pend[j] = __ballot(r.g[j] != kNoEdit);
        any |= pend[j] != 0;
    }
    while (any) {
        int32_t k = 0;
        bool found = false;
#pragma unroll
        for (int j = 0; j < kEditsPerLane; ++j)
            if (!found && pend[j]) {
                k = __builtin_amdgcn_readlane(node_of[j], (int)__builtin_ctzll(pend[j]));
                found = true;
            }
        any = false;
#pragma unroll
        for (int j = 0; j < kEditsPerLane; ++j) {
            const bool mine = ((pend[j] >> lane) & 1ull) && node_of[j] == k;
            if (mine) buf[r.col[j] - c0] = (char)(r.chr[j] & 0x7fu);
            pend[j] &= ~__ballot(mine);
            any |= pend[j] != 0;
        }
    }
}

// Blocks absent at the leaf that overlap tile t, as tile-relative column ranges in LDS
// (rng[0] = count, -1 = more than kRestoreRanges: the restore walks the blocks itself).
constexpr int kRestoreRanges = 6;

template <int64_t TB = kReplayTile>
__device__ __forceinline__ void absent_ranges(const ReplayDev& d, int32_t leaf, int32_t t, int32_t* rng) {
    const int64_t c0 = (int64_t)t * TB, c1 = min(c0 + TB, d.row_stride);
    const uint32_t* pres = d.presence + (size_t)leaf * d.presence_words;
    int nr = 0;
    for (int32_t id = d.tile_blk[t]; id < d.blocks; ++id) {
        const int64_t b_lo = d.blk_lo[id];
        if (b_lo >= c1) break;
        if ((pres[id >> 5] >> (id & 31)) & 1u) continue;
        if (nr == kRestoreRanges) {
            nr = -1;
            break;
        }
        rng[1 + 2 * nr] = (int32_t)(max(b_lo, c0) - c0);
        rng[2 + 2 * nr] = (int32_t)(min(d.blk_hi[id], c1) - c0);
        ++nr;
    }
    rng[0] = nr;
}

// blocks absent at the leaf keep the consensus (their edits are not applied: :1842)
__device__ __forceinline__ void restore_absent(const ReplayDev& d, int32_t leaf, int32_t t, const int32_t* rng,
                                               char* buf, int first, int stride) {
    const int64_t c0 = (int64_t)t * kReplayTile, c1 = min(c0 + kReplayTile, d.row_stride);
    const int nr = rng[0];
    if (nr >= 0) {
        const uint4* cons16 = reinterpret_cast<const uint4*>(d.cons_row + c0);
        uint4* buf16 = reinterpret_cast<uint4*>(buf);
        for (int i = 0; i < nr; ++i) {
            const int32_t a = rng[1 + 2 * i], b = rng[2 + 2 * i];
            const int32_t a16 = min((a + 15) & ~15, b), b16 = max(b & ~15, a16);
            // ragged ends byte by byte, the aligned middle 16 B per thread
            if (first < a16 - a) buf[a + first] = d.cons_row[c0 + a + first];
            if (first < b - b16) buf[b16 + first] = d.cons_row[c0 + b16 + first];
            for (int32_t k = a16 / 16 + first; k < b16 / 16; k += stride) buf16[k] = cons16[k];
        }
        return;
    }
    const uint32_t* pres = d.presence + (size_t)leaf * d.presence_words;
    for (int32_t id = d.tile_blk[t]; id < d.blocks; ++id) {
        const int64_t b_lo = d.blk_lo[id];
        if (b_lo >= c1) break;
        if ((pres[id >> 5] >> (id & 31)) & 1u) continue;
        const int64_t a = max(b_lo, c0), b = min(d.blk_hi[id], c1);
        for (int64_t k = a + first; k < b; k += stride) buf[k - c0] = d.cons_row[k];
    }
}

// Column tiles per workgroup (a workgroup = (leaf, kReplayGroup tiles), tile after tile).
#ifndef PM_REPLAY_GROUP
#define PM_REPLAY_GROUP 8
#endif
constexpr int kReplayGroup = PM_REPLAY_GROUP;


// LDS-DMA copy-in of the consensus tile t (1 KiB per wave-instruction, all in flight).
__device__ __forceinline__ void tile_copy_in(const ReplayDev& d, int32_t t, uint4* dst, int wave, int lane) {
    const int64_t c0 = (int64_t)t * kReplayTile;
    const int64_t n = min(kReplayTile, d.row_stride - c0);   // multiple of 16
    const uint4* src = reinterpret_cast<const uint4*>(d.cons_row + c0);
    for (int64_t b = (int64_t)wave * kWave; b < n / 16; b += 4 * kWave) {
        const int64_t k = b + lane;
        if (k < n / 16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + k),
                                             (__attribute__((address_space(3))) void*)(dst + b), 16, 0, 0);
    }
}

// Overriding edits of a tile resolved in parallel (list in LDS, 4 B each); more: in path order.
constexpr int kOvrCap = 1024;

#ifndef PM_REPLAY_WAVES
#define PM_REPLAY_WAVES 6
#endif

// The path's tile bounds in LDS.  A chunk's slice bounds for tile t are {plain, overriding}
// starts at t and t + 1 for each of its path nodes; the first ReplayDev::ring path nodes keep
// three tiles of them in a ring (dynamic LDS, `ring` = [3][d.ring]), written two tiles ahead by
// the thread that owns the node (nodes tid, tid + 256), so a tile's chunks wait on no bounds
// load; deeper path nodes (beyond the ring) load theirs from HBM.
struct PathCtx {
    int64_t p0;
    int depth;
    const int2* ring;
    int32_t ring_n;
};

__device__ __forceinline__ void chunk_bounds(const ReplayDev& d, const PathCtx& pc, int q, int s0, int s1, int32_t t,
                                             int lane, int& cnt, int2& lo, int2& hi) {
    cnt = min(kWave, pc.depth - q);
    lo = hi = make_int2(0, 0);
    if (lane < cnt) {
        const int k = q + lane;
        if (k < pc.ring_n) {
            lo = pc.ring[s0 * pc.ring_n + k];
            hi = pc.ring[s1 * pc.ring_n + k];
        } else {
            const int2* te = d.tile2 + (size_t)d.path[pc.p0 + k] * (d.tiles + 1) + t;
            lo = te[0];
            hi = te[1];
        }
    }
}

// One workgroup = (leaf, group of kReplayGroup column tiles).  Per tile: copy-in; the plain
// edits, chunk after chunk, rounds dealt to the four waves (the first round of the first
// chunk prefetched during the previous tile's write-out); the overriding edits staged in path
// order and resolved; absent blocks restored; write-out.
__global__ __launch_bounds__(256, PM_REPLAY_WAVES) void k_replay(ReplayDev d) {
    __shared__ uint4 tile_buf[kReplayTile / 16];
    __shared__ uint32_t olist[kOvrCap];   // (column in tile) | chr << 16, path order
    __shared__ int32_t rng[2][2 + 2 * kRestoreRanges];
    extern __shared__ int2 ring[];        // [3][d.ring]
    char* buf = reinterpret_cast<char*>(tile_buf);
    const int32_t leaf = blockIdx.x;
    const int32_t t_begin = (int32_t)blockIdx.y * kReplayGroup;
    const int32_t t_end = min(d.tiles, t_begin + kReplayGroup);
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & (kWave - 1);
    PathCtx pc;
    pc.p0 = d.path_off[leaf];
    pc.depth = (int)(d.path_off[leaf + 1] - pc.p0);
    pc.ring = ring;
    pc.ring_n = d.ring;
    const int ring_use = min(pc.depth, d.ring);
    // the ring: tiles t_begin, t_begin + 1 now, t_begin + 2 in flight (pre)
    int2 pre[2] = {make_int2(0, 0), make_int2(0, 0)};
    int32_t pnode[2] = {-1, -1};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = tid + 256 * h;
        if (k < ring_use) {
            pnode[h] = d.path[pc.p0 + k];
            const int2* te = d.tile2 + (size_t)pnode[h] * (d.tiles + 1);
            ring[k] = te[t_begin];
            ring[d.ring + k] = te[t_begin + 1];
            if (t_begin + 2 <= t_end) pre[h] = te[t_begin + 2];
        }
    }
    if (tid == kWave) absent_ranges(d, leaf, t_begin, rng[0]);
    EditChunk ch{}, co{};
    EditRound r{}, ro{};
    bool have_pf = false;   // (ch, r), (co, ro): tile t's first chunk and its first rounds
    for (int32_t t = t_begin; t < t_end; ++t) {
        const int64_t c0 = (int64_t)t * kReplayTile;
        const int64_t n = min(kReplayTile, d.row_stride - c0);   // multiple of 16
        const int s0 = (t - t_begin) % 3, s1 = (t - t_begin + 1) % 3;
        tile_copy_in(d, t, tile_buf, wave, lane);
        __syncthreads();   // the copy-in landed; the ring's slots for t, t + 1 written
        // Chunk by chunk: the plain edits written (any order), the overriding ones staged in
        // path order (chunk base + index in the chunk); both parts' first rounds are issued
        // together (for the first chunk during the previous tile's write-out)
        int32_t no = 0;   // (uniform) overriding edits staged so far
        for (int q = 0; q < pc.depth; q += kWave) {
            if (q > 0 || !have_pf) {
                int cnt;
                int2 lo, hi;
                chunk_bounds(d, pc, q, s0, s1, t, lane, cnt, lo, hi);
                ch = edit_chunk_from(cnt, lo.x, hi.x, lane);
                co = edit_chunk_from(cnt, lo.y, hi.y, lane);
                if (wave * kRound < ch.total) edit_round(d, ch, wave * kRound, c0, lane, r);
                if (wave * kRound < co.total) edit_round(d, co, wave * kRound, c0, lane, ro);
            }
            for (int32_t sr = 0; sr < ch.total; sr += 4 * kRound) {   // (uniform)
                const int32_t base = sr + wave * kRound;
                if (base >= ch.total) break;
                if (sr > 0) edit_round(d, ch, base, c0, lane, r);
                edit_write_all(r, buf, c0);
            }
            for (int32_t sr = 0; sr < co.total; sr += 4 * kRound) {
                const int32_t base = sr + wave * kRound;
                if (base >= co.total) break;
                if (sr > 0) edit_round(d, co, base, c0, lane, ro);
#pragma unroll
                for (int j = 0; j < kEditsPerLane; ++j)
                    if (ro.g[j] != kNoEdit && no + ro.g[j] < kOvrCap)
                        olist[no + ro.g[j]] = (uint32_t)(ro.col[j] - c0) | (ro.chr[j] & 0x7fu) << 16;
            }
            no += co.total;
        }
        have_pf = false;
        if (no > 0) {   // (uniform)
            lds_barrier();   // the plain edits and the list are in LDS
            if (no <= kOvrCap) {
                // an entry is written unless a later one (a deeper path node) has its column
                for (int32_t i = tid; i < no; i += 256) {
                    const uint32_t e = olist[i], col = e & 0xffffu;
                    bool later = false;
                    for (int32_t k = i + 1; k < no && !later; ++k) later = (olist[k] & 0xffffu) == col;
                    if (!later) buf[col] = (char)(e >> 16);
                }
            } else {
                // in path order: the overriding rounds again, wave by wave, each round's edits
                // node by node
                for (int q = 0; q < pc.depth; q += kWave) {
                    int cnt;
                    int2 lo, hi;
                    chunk_bounds(d, pc, q, s0, s1, t, lane, cnt, lo, hi);
                    const EditChunk cf = edit_chunk_from(cnt, lo.y, hi.y, lane);
                    for (int32_t sr = 0; sr < cf.total; sr += 4 * kRound) {
                        const int32_t base = sr + wave * kRound;
                        EditRound rf{};
                        int32_t node_of[kEditsPerLane];
#pragma unroll
                        for (int j = 0; j < kEditsPerLane; ++j) node_of[j] = 0;
                        if (base < cf.total) {
                            edit_round(d, cf, base, c0, lane, rf);
#pragma unroll
                            for (int j = 0; j < kEditsPerLane; ++j) {   // path position of each edit
                                int k_lo = 0, k_hi = cf.cnt - 1;
#pragma unroll
                                for (int st = 0; st < 6; ++st) {
                                    const int mid = (k_lo + k_hi + 1) >> 1;
                                    if (__shfl(cf.excl, mid) <= base + lane + j * kWave) k_lo = mid;
                                    else k_hi = mid - 1;
                                }
                                node_of[j] = q + k_lo;
                            }
                        }
                        for (int w = 0; w < 4; ++w) {
                            if (wave == w && base < cf.total) edit_write_ordered(rf, node_of, buf, c0);
                            lds_barrier();
                        }
                    }
                }
            }
        }
        lds_barrier();   // every edit in LDS before the restore overwrites absent blocks
        restore_absent(d, leaf, t, rng[(t - t_begin) & 1], buf, tid, blockDim.x);
        // the ring slot of tile t - 1 (read by nobody any more) takes tile t + 2
        if (t + 2 <= t_end) {
            const int s2 = (t - t_begin + 2) % 3;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = tid + 256 * h;
                if (k < ring_use) {
                    ring[s2 * d.ring + k] = pre[h];
                    if (t + 3 <= t_end) pre[h] = d.tile2[(size_t)pnode[h] * (d.tiles + 1) + t + 3];
                }
            }
        }
        if (tid == kWave && t + 1 < t_end) absent_ranges(d, leaf, t + 1, rng[(t + 1 - t_begin) & 1]);
        lds_barrier();
        if (t + 1 < t_end) {
            // the next tile's first plain round, in flight through the write-out and copy-in
            int cnt;
            int2 lo, hi;
            chunk_bounds(d, pc, 0, s1, (t - t_begin + 2) % 3, t + 1, lane, cnt, lo, hi);
            ch = edit_chunk_from(cnt, lo.x, hi.x, lane);
            co = edit_chunk_from(cnt, lo.y, hi.y, lane);
            if (wave * kRound < ch.total) edit_round(d, ch, wave * kRound, c0 + kReplayTile, lane, r);
            if (wave * kRound < co.total) edit_round(d, co, wave * kRound, c0 + kReplayTile, lane, ro);
            have_pf = true;
        }
        uint4* dst = reinterpret_cast<uint4*>(d.rows + (size_t)leaf * d.row_stride + c0);
        // a fixed count of stores (the compiler then waits for an earlier load with
        // vmcnt(#stores) instead of draining them)
        static_assert(kReplayTile / 16 % 256 == 0, "write-out: whole rounds of 256 threads");
#pragma unroll
        for (int j = 0; j < kReplayTile / 16 / 256; ++j) {
            const int k = tid + 256 * j;
            if (k < n / 16) store_stream(dst + k, tile_buf[k]);
        }
        lds_barrier();   // the tile buffer is refilled next
    }
}

// ---- k_replay_dfs: one wave = (leaf group, column tile), the leaves of the group in
// depth-first order against ONE copy of the tile in the wave's own LDS.
//
// Consecutive leaves in depth-first order share their path down to their lowest common
// ancestor, so leaf i's row is leaf i - 1's with the edits of the nodes below the LCA on
// i - 1's path undone and those on i's path applied: every edge of the group's subtree is
// applied and undone once per tile, instead of every path node once per leaf (C5: 3.6x
// fewer edit writes; a SARS-like tree ~7x), and the consensus tile is copied in once per
// group instead of once per leaf.  Undo: every applied edit pushes the byte it overwrote
// (plain edits onto one stack, overriding ones onto another, frames per path position); the
// exit pops the overriding frames deepest first, node by node, then every plain entry at
// once (plain edits of one path touch distinct columns).  A wave's LDS operations take effect
// in issue order, so the phases need no barrier.  Blocks absent at a leaf are substituted
// with the consensus at write-out.  A leaf whose edits would overflow a stack rebuilds its
// row (consensus copy-in, whole path, nothing pushed), as do the group's later leaves.
static_assert(kDfsLeaves <= kWave && kDfsUnionCap <= 256, "k_replay_dfs: a lane per leaf, u8 group node indices");
static_assert(kDfsTile <= 32768, "k_replay_dfs: in-tile columns in 16 bits (undo stacks) and int16 block bounds");
#ifndef PM_DFS_PCAP
#define PM_DFS_PCAP 384
#endif
constexpr int kDfsPCap = PM_DFS_PCAP;   // plain edits on the current path in one tile
constexpr int kDfsOCap = 64;    // overriding edits on the current path in one tile

struct DfsLds {
    uint4 tile[kDfsTile / 16];
    int4 bnd[kDfsUnionCap];          // per group node: {plain lo, plain hi, overriding lo, hi} of this tile
    uint32_t pst[kDfsPCap];          // plain undo stack: (column in tile) | old byte << 16
    uint32_t ost[kDfsOCap];          // overriding undo stack
    uint16_t psp_at[kDfsUnionCap];   // stack pointers before each path position's pushes
    uint16_t osp_at[kDfsUnionCap];
    uint8_t cur_u[kDfsUnionCap];     // group node index at each position of the current path
    // the tile's blocks (tile-relative [ba, bb), nb of them; -1: more than the table holds) and,
    // per leaf of the group, its row, path length, shared prefix and absent-block mask
    int16_t ba[kWave], bb[kWave];
    int32_t nb;
    uint64_t absent[kDfsLeaves];
    int32_t lrow[kDfsLeaves];
    uint16_t llen[kDfsLeaves], llp[kDfsLeaves];
};

// edit_round plus each edit's node (position in the chunk) for the ordered apply
__device__ __forceinline__ void edit_nodes(const EditChunk& c, int32_t base, int lane, int32_t* node_of) {
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        const int32_t g = base + lane + j * kWave;
        int k_lo = 0, k_hi = c.cnt - 1;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const int mid = (k_lo + k_hi + 1) >> 1;
            if (__shfl(c.excl, mid) <= g) k_lo = mid;
            else k_hi = mid - 1;
        }
        node_of[j] = k_lo;
    }
}


// Item start: the tile's blocks, and for each leaf of the group its metadata and which of
// those blocks are absent at it (one pass of loads, in flight with the consensus copy-in).
__device__ __forceinline__ void dfs_leaf_tables(const ReplayDev& d, DfsLds& S, int32_t i0, int32_t cnt, int32_t t,
                                                int64_t c0, int64_t n, int lane) {
    const int32_t id = d.tile_blk[t] + lane;
    bool ok = false;
    if (id < d.blocks) {
        const int64_t lo = d.blk_lo[id];
        ok = lo < c0 + n;
        if (ok) {
            S.ba[lane] = (int16_t)(max(lo, c0) - c0);
            S.bb[lane] = (int16_t)(min(d.blk_hi[id], c0 + n) - c0);
        }
    }
    const int nb = __popcll(__ballot(ok));   // (blocks are in column order: a prefix of the lanes)
    if (lane < cnt) {
        S.lrow[lane] = d.dfs_row[i0 + lane];
        S.llen[lane] = d.dfs_len[i0 + lane];
        S.llp[lane] = d.dfs_lpfx[i0 + lane];
        S.absent[lane] = 0;
    }
    S.nb = nb == kWave ? -1 : nb;
    if (nb == kWave) return;   // (the write-out walks the blocks itself)
    const int32_t id0 = d.tile_blk[t];
    for (int32_t e = lane; e < cnt * nb; e += kWave) {
        const int32_t k = e / nb, j = e - k * nb, bid = id0 + j;
        const uint32_t w = d.presence[(size_t)S.lrow[k] * d.presence_words + (bid >> 5)];
        if (!((w >> (bid & 31)) & 1u)) atomicOr(reinterpret_cast<unsigned long long*>(&S.absent[k]), 1ull << j);
    }
}

// The leaf's row for this tile from the LDS tile, blocks absent at the leaf from the consensus.
__device__ __forceinline__ uint32_t byte_span_mask(int32_t w0, int32_t a, int32_t b) {   // bytes of dword [w0, w0 + 4) in [a, b)
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) m |= (w0 + k >= a && w0 + k < b) ? 0xffu << (8 * k) : 0u;
    return m;
}

__device__ __forceinline__ void dfs_write_out(const ReplayDev& d, DfsLds& S, int32_t li, int32_t t, int64_t c0, int64_t n,
                                              int lane) {
    const int32_t row = S.lrow[li];
    const int nb = S.nb;
    const uint64_t am = nb >= 0 ? S.absent[li] : ~0ull;
    uint4* dst = reinterpret_cast<uint4*>(d.rows + (size_t)row * d.row_stride + c0);
    const uint4* cons16 = reinterpret_cast<const uint4*>(d.cons_row + c0);
    static_assert(kDfsTile / 16 % kWave == 0, "write-out: whole rounds of 64 lanes");
    // (uniform) the common case -- a whole tile, no absent block: every round's LDS reads
    // first, then the stores (C5 1.27 -> 1.20 ms, SARS-like 2.37 -> 2.31 ms against the loop)
    if (am == 0 && n == kDfsTile) {
        constexpr int R = kDfsTile / 16 / kWave;
        uint4 v[R];
#pragma unroll
        for (int j = 0; j < R; ++j) v[j] = S.tile[lane + kWave * j];
#pragma unroll
        for (int j = 0; j < R; ++j) store_stream(dst + lane + kWave * j, v[j]);
        return;
    }
    for (int j = 0; j < kDfsTile / 16 / kWave; ++j) {
        const int k = lane + kWave * j;
        if (k >= n / 16) break;
        uint4 v = S.tile[k];
        if (am != 0) {   // (uniform)
            uint32_t m[4] = {0, 0, 0, 0};
            if (nb >= 0) {
                for (uint64_t x = am; x; x &= x - 1) {
                    const int bj = __builtin_ctzll(x);
                    const int32_t a = S.ba[bj], b = S.bb[bj];
                    if (a < 16 * k + 16 && b > 16 * k)
#pragma unroll
                        for (int w = 0; w < 4; ++w) m[w] |= byte_span_mask(16 * k + 4 * w, a, b);
                }
            } else {   // more blocks than the table holds: walk them
                const uint32_t* pres = d.presence + (size_t)row * d.presence_words;
                for (int32_t id = d.tile_blk[t]; id < d.blocks; ++id) {
                    const int64_t b_lo = d.blk_lo[id];
                    if (b_lo >= c0 + 16 * k + 16) break;
                    if ((pres[id >> 5] >> (id & 31)) & 1u) continue;
                    const int32_t a = (int32_t)(max(b_lo, c0) - c0), b = (int32_t)(min(d.blk_hi[id], c0 + n) - c0);
#pragma unroll
                    for (int w = 0; w < 4; ++w) m[w] |= byte_span_mask(16 * k + 4 * w, a, b);
                }
            }
            if (m[0] | m[1] | m[2] | m[3]) {
                const uint4 cv = cons16[k];
                v.x = (v.x & ~m[0]) | (cv.x & m[0]);
                v.y = (v.y & ~m[1]) | (cv.y & m[1]);
                v.z = (v.z & ~m[2]) | (cv.z & m[2]);
                v.w = (v.w & ~m[3]) | (cv.w & m[3]);
            }
        }
        store_stream(dst + k, v);
    }
}

// A leaf's first chunk of entering positions (lane = position, group nodes u_lo + lane) and
// the first round of its plain and of its overriding edits, issued ahead (during the previous
// leaf's write-out).
struct DfsPrefetch {
    EditChunk ch, co;
    EditRound r, ro;
};

__device__ __forceinline__ void dfs_prefetch(const ReplayDev& d, const DfsLds& S, int32_t u_lo, int32_t cnt, int64_t c0,
                                             int lane, DfsPrefetch& f) {
    int4 b = make_int4(0, 0, 0, 0);
    if (lane < cnt) b = S.bnd[u_lo + lane];
    f.ch = edit_chunk_from(cnt, b.x, b.y, lane);
    f.co = edit_chunk_from(cnt, b.z, b.w, lane);
    if (f.ch.total > 0) edit_round(d, f.ch, 0, c0, lane, f.r);
    if (f.co.total > 0) edit_round(d, f.co, 0, c0, lane, f.ro);
}

// Apply the edits of path positions [p_lo, p_hi) of the current path (group nodes cur_u[p]):
// plain ones first (all positions at once, any order), then the overriding ones position by
// position in path order.  PUSH: save every overwritten byte and record the frames.  `pf`:
// the first chunk and its first rounds are in `f` (dfs_prefetch).
template <bool PUSH>
__device__ __forceinline__ void dfs_apply(const ReplayDev& d, DfsLds& S, int32_t p_lo, int32_t p_hi, int64_t c0, int lane,
                                          int32_t& psp, int32_t& osp, bool pf, DfsPrefetch& f) {
    char* buf = reinterpret_cast<char*>(S.tile);
    for (int32_t q = p_lo; q < p_hi; q += kWave) {   // plain
        const int cnt = min(kWave, p_hi - q);
        const bool first = pf && q == p_lo;
        if (!first) {
            int4 b = make_int4(0, 0, 0, 0);
            if (lane < cnt) b = S.bnd[S.cur_u[q + lane]];
            f.ch = edit_chunk_from(cnt, b.x, b.y, lane);
        }
        const EditChunk& ch = f.ch;
        if (PUSH && lane < cnt) S.psp_at[q + lane] = (uint16_t)(psp + ch.excl);
        for (int32_t base = 0; base < ch.total; base += kRound) {
            if (!first || base > 0) edit_round(d, ch, base, c0, lane, f.r);
            const EditRound& r = f.r;
#pragma unroll
            for (int j = 0; j < kEditsPerLane; ++j)
                if (r.g[j] != kNoEdit) {
                    const uint32_t col = r.col[j] - (uint32_t)c0;
                    if (PUSH) S.pst[psp + r.g[j]] = col | (uint32_t)(uint8_t)buf[col] << 16;
                    buf[col] = (char)(r.chr[j] & 0x7fu);
                }
        }
        if (PUSH) psp += ch.total;
    }
    for (int32_t q = p_lo; q < p_hi; q += kWave) {   // overriding, in path order
        const int cnt = min(kWave, p_hi - q);
        const bool first = pf && q == p_lo;
        if (!first) {
            int4 b = make_int4(0, 0, 0, 0);
            if (lane < cnt) b = S.bnd[S.cur_u[q + lane]];
            f.co = edit_chunk_from(cnt, b.z, b.w, lane);
        }
        const EditChunk& co = f.co;
        if (PUSH && lane < cnt) S.osp_at[q + lane] = (uint16_t)(osp + co.excl);
        for (int32_t base = 0; base < co.total; base += kRound) {
            if (!first || base > 0) edit_round(d, co, base, c0, lane, f.ro);
            const EditRound& r = f.ro;
            int32_t node_of[kEditsPerLane];
            edit_nodes(co, base, lane, node_of);
            uint64_t pend[kEditsPerLane];
            bool any = false;
#pragma unroll
            for (int j = 0; j < kEditsPerLane; ++j) {
                pend[j] = __ballot(r.g[j] != kNoEdit);
                any |= pend[j] != 0;
            }
            while (any) {   // node by node: the first pending edit names the next node
                int32_t k = 0;
                bool found = false;
#pragma unroll
                for (int j = 0; j < kEditsPerLane; ++j)
                    if (!found && pend[j]) {
                        k = __builtin_amdgcn_readlane(node_of[j], (int)__builtin_ctzll(pend[j]));
                        found = true;
                    }
                any = false;
#pragma unroll
                for (int j = 0; j < kEditsPerLane; ++j) {
                    const bool mine = ((pend[j] >> lane) & 1ull) && node_of[j] == k;
                    if (mine) {
                        const uint32_t col = r.col[j] - (uint32_t)c0;
                        if (PUSH) S.ost[osp + r.g[j]] = col | (uint32_t)(uint8_t)buf[col] << 16;
                        buf[col] = (char)(r.chr[j] & 0x7fu);
                    }
                    pend[j] &= ~__ballot(mine);
                    any |= pend[j] != 0;
                }
            }
        }
        if (PUSH) osp += co.total;
    }
}

// Edits of positions [p_lo, p_hi): plain and overriding counts (uniform).
__device__ __forceinline__ void dfs_counts(DfsLds& S, int32_t p_lo, int32_t p_hi, int lane, int32_t& np, int32_t& no) {
    np = no = 0;
    for (int32_t q = p_lo; q < p_hi; q += kWave) {
        int4 b = make_int4(0, 0, 0, 0);
        if (q + lane < p_hi) b = S.bnd[S.cur_u[q + lane]];
        np += (int32_t)wave_inclusive_scan((uint32_t)(b.y - b.x)) ;
        no += (int32_t)wave_inclusive_scan((uint32_t)(b.w - b.z));
        np = __builtin_amdgcn_readlane(np, kWave - 1);
        no = __builtin_amdgcn_readlane(no, kWave - 1);
    }
}

__device__ __forceinline__ void dfs_copy_in(const ReplayDev& d, DfsLds& S, int64_t c0, int64_t n, int lane) {
    const uint4* src = reinterpret_cast<const uint4*>(d.cons_row + c0);
    for (int64_t b = 0; b < n / 16; b += kWave) {
        const int64_t k = b + lane;
        if (k < n / 16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + k),
                                             (__attribute__((address_space(3))) void*)(S.tile + b), 16, 0, 0);
    }
}

// Small transitions (the common case: at most kFastNodes entering nodes, each with at most
// kFastEdits plain and overriding edits in the tile): lane = (node k, edit j) with k = lane /
// kFastEdits, so the edits come with one load per lane and no prefix scan or binary search
// (the general path, dfs_apply, costs ~100 VALU instructions per round; the kernel is issue-
// bound: r05 SQ counters, 27 % of wave cycles issuing at ~4 waves per SIMD).
constexpr int kFastEdits = 16, kFastNodes = kWave / kFastEdits;

struct DfsFast {
    bool on;                  // (uniform) this transition is small
    int4 b;                   // this lane's node's bounds
    uint32_t cp, hp, co, ho;  // this lane's plain / overriding edit (column, char); kNoCol: none
};
constexpr uint32_t kNoCol = ~0u;

__device__ __forceinline__ void dfs_fast_prefetch(const ReplayDev& d, const DfsLds& S, int32_t u_lo, int32_t cnt, int lane,
                                                  DfsFast& x) {
    const int k = lane / kFastEdits, j = lane % kFastEdits;
    x.b = make_int4(0, 0, 0, 0);
    if (k < cnt) x.b = S.bnd[u_lo + k];
    x.on = cnt <= kFastNodes && !__ballot(k < cnt && (x.b.y - x.b.x > kFastEdits || x.b.w - x.b.z > kFastEdits));
    x.cp = x.co = kNoCol;
    x.hp = x.ho = 0;
    if (!x.on) return;
    if (j < x.b.y - x.b.x) {
        x.cp = d.edit_col[x.b.x + j];
        x.hp = d.edit_chr[x.b.x + j];
    }
    if (j < x.b.w - x.b.z) {
        x.co = d.edit_col[x.b.z + j];
        x.ho = d.edit_chr[x.b.z + j];
    }
}

// Per-node counts of a small transition (lane k * kFastEdits holds node k's): the exclusive
// prefix for this lane's node and the totals.
__device__ __forceinline__ void fast_prefix(int32_t len, int lane, int32_t& pre, int32_t& total) {
    const int32_t l0 = __builtin_amdgcn_readlane(len, 0), l1 = __builtin_amdgcn_readlane(len, kFastEdits),
                  l2 = __builtin_amdgcn_readlane(len, 2 * kFastEdits), l3 = __builtin_amdgcn_readlane(len, 3 * kFastEdits);
    const int k = lane / kFastEdits;
    pre = k == 0 ? 0 : k == 1 ? l0 : k == 2 ? l0 + l1 : l0 + l1 + l2;
    total = l0 + l1 + l2 + l3;
}

// Apply a small transition's entering positions [lp, lp + cnt): plain edits (pushed), then the
// overriding ones node by node in path order (pushed).
__device__ __forceinline__ void dfs_fast_apply(DfsLds& S, const DfsFast& x, int32_t lp, int32_t cnt, int64_t c0, int lane,
                                               int32_t& psp, int32_t& osp) {
    char* buf = reinterpret_cast<char*>(S.tile);
    const int k = lane / kFastEdits, j = lane % kFastEdits;
    int32_t pre, tot, opre, otot;
    fast_prefix(k < cnt ? x.b.y - x.b.x : 0, lane, pre, tot);
    fast_prefix(k < cnt ? x.b.w - x.b.z : 0, lane, opre, otot);
    if (j == 0 && k < cnt) {
        S.psp_at[lp + k] = (uint16_t)(psp + pre);
        S.osp_at[lp + k] = (uint16_t)(osp + opre);
    }
    if (x.cp != kNoCol) {
        const uint32_t col = x.cp - (uint32_t)c0;
        S.pst[psp + pre + j] = col | (uint32_t)(uint8_t)buf[col] << 16;
        buf[col] = (char)(x.hp & 0x7fu);
    }
    psp += tot;
    if (otot > 0) {   // (uniform) in path order: node k after node k - 1
        for (int kk = 0; kk < cnt; ++kk) {
            if (k == kk && x.co != kNoCol) {
                const uint32_t col = x.co - (uint32_t)c0;
                S.ost[osp + opre + j] = col | (uint32_t)(uint8_t)buf[col] << 16;
                buf[col] = (char)(x.ho & 0x7fu);
            }
        }
        osp += otot;
    }
}

struct DfsState {
    int32_t psp, osp, prev_len, next_u, len, lp;   // stacks, previous path length, next group node, this leaf's path
    bool rebuild;
    int32_t gc;   // the path prefix every leaf of the group shares (never undone inside the group)
};

// Leaf i of the group: its transition (cur: the fast one, prefetched two leaves ahead; or f:
// the general one, prefetched one leaf ahead), its write-out; meanwhile leaf i + 1's general
// prefetch (when nxt, its fast one, does not apply) and leaf i + 2's fast one (into cur).
__device__ __forceinline__ void dfs_leaf(const ReplayDev& d, DfsLds& S, DfsState& st, int32_t i, int32_t i0, int32_t i1,
                                         int32_t t, int64_t c0, int64_t n, int lane, DfsPrefetch& f, DfsFast& cur,
                                         const DfsFast& nxt) {
    const int32_t len = st.len, lp = st.lp;
    // the path positions [lp, len) are new group nodes next_u ..
    for (int32_t p = lp + lane; p < len; p += kWave) S.cur_u[p] = (uint8_t)(st.next_u + (p - lp));
    st.next_u += len - lp;
    char* buf = reinterpret_cast<char*>(S.tile);
#ifndef PM_DFS_NOEDITS
    int32_t np = 0, no = 0;
    // the group's first leaf: its positions [0, gc) are every leaf's and never undone inside
    // the group, so they are applied without pushes (with the prefetched first chunk) and the
    // stacks hold only what later leaves undo -- a deep tree's long shared stem would otherwise
    // overflow them and make every leaf of the group rebuild its row
    int32_t lo = lp;
    if (i == i0 && st.gc > 0 && !st.rebuild) {
        lo = min(st.gc, len);
        dfs_apply<false>(d, S, 0, lo, c0, lane, st.psp, st.osp, true, f);
    }
    if (!st.rebuild) {
        if (cur.on) {   // (the counts from the prefetched bounds)
            int32_t pre;
            fast_prefix(lane / kFastEdits < len - lp ? cur.b.y - cur.b.x : 0, lane, pre, np);
            fast_prefix(lane / kFastEdits < len - lp ? cur.b.w - cur.b.z : 0, lane, pre, no);
        } else {
            dfs_counts(S, lo, len, lane, np, no);
        }
        const int32_t psp_x = lo < st.prev_len ? (int32_t)S.psp_at[lo] : st.psp;
        const int32_t osp_x = lo < st.prev_len ? (int32_t)S.osp_at[lo] : st.osp;
        st.rebuild = psp_x + np > kDfsPCap || osp_x + no > kDfsOCap;
    }
    if (!st.rebuild) {
        // exit: overriding frames deepest first, then the plain entries above lp
        if (lp < st.prev_len) {
            for (int32_t p = st.prev_len - 1; p >= lp && st.osp > (int32_t)S.osp_at[lp]; --p) {
                const int32_t a = S.osp_at[p];
                for (int32_t k = a + lane; k < st.osp; k += kWave) {
                    const uint32_t e = S.ost[k];
                    buf[e & 0xffffu] = (char)(e >> 16);
                }
                st.osp = a;
            }
            st.osp = S.osp_at[lp];
            const int32_t a = S.psp_at[lp];
            for (int32_t k = a + lane; k < st.psp; k += kWave) {
                const uint32_t e = S.pst[k];
                buf[e & 0xffffu] = (char)(e >> 16);
            }
            st.psp = a;
        }
        if (cur.on) dfs_fast_apply(S, cur, lp, len - lp, c0, lane, st.psp, st.osp);
        else dfs_apply<true>(d, S, lo, len, c0, lane, st.psp, st.osp, lo == lp, f);
    } else {
        // rebuild: the consensus again, the whole path, nothing pushed
        if (lane == 0) atomicAdd(d.dfs_rebuilds, 1);   // (rare; counted for the tests)
        dfs_copy_in(d, S, c0, n, lane);
        __syncthreads();
        dfs_apply<false>(d, S, 0, len, c0, lane, st.psp, st.osp, false, f);
    }
#endif
    st.prev_len = len;
    if (i + 1 < i1) {
        st.len = S.llen[i + 1 - i0];
        st.lp = S.llp[i + 1 - i0];
        if (!nxt.on) dfs_prefetch(d, S, st.next_u, min(kWave, st.len - st.lp), c0, lane, f);
        if (i + 2 < i1) dfs_fast_prefetch(d, S, st.next_u + (st.len - st.lp), S.llen[i + 2 - i0] - S.llp[i + 2 - i0], lane, cur);
    }
    dfs_write_out(d, S, i - i0, t, c0, n, lane);
}

// waves per SIMD (the second __launch_bounds__ argument is amdgpu_waves_per_eu): 4 = 128 VGPRs
#ifndef PM_DFS_WAVES
#define PM_DFS_WAVES 4
#endif
__global__ __launch_bounds__(kWave, PM_DFS_WAVES) void k_replay_dfs(ReplayDev d) {
    __shared__ DfsLds S;
    const int lane = (int)threadIdx.x;
#ifdef PM_DFS_TILE_MAJOR   // (A/B) concurrent waves = many groups' rows at one tile
    const int32_t t = (int32_t)(blockIdx.x / (uint32_t)d.groups), g = (int32_t)(blockIdx.x % (uint32_t)d.groups);
#else
    // concurrent waves = consecutive tiles of few groups: their writes are adjacent pieces of
    // the same few rows (DRAM pages, translations) instead of one piece of thousands of rows
    const int32_t g = (int32_t)(blockIdx.x / (uint32_t)d.tiles), t = (int32_t)(blockIdx.x % (uint32_t)d.tiles);
#endif
    const int64_t c0 = (int64_t)t * kDfsTile;
    const int64_t n = min(kDfsTile, d.row_stride - c0);   // multiple of 16
    const int32_t i0 = d.g_leaf_off[g], i1 = d.g_leaf_off[g + 1];
    const int32_t u0 = d.g_union_off[g], nu = d.g_union_off[g + 1] - u0;
    // the group's node bounds for this tile, and the consensus tile
    for (int32_t u = lane; u < nu; u += kWave) {
        const int2* te = d.tile2 + (size_t)d.g_union[u0 + u] * (d.tiles + 1) + t;
        const int2 a = te[0], b = te[1];
        S.bnd[u] = make_int4(a.x, b.x, a.y, b.y);
    }
    dfs_copy_in(d, S, c0, n, lane);
    dfs_leaf_tables(d, S, i0, i1 - i0, t, c0, n, lane);
    __syncthreads();   // (one wave: the copy-in and the tables landed)
    int32_t gc = S.llen[0];   // (a one-leaf group: its whole path)
    for (int32_t k = 1; k < i1 - i0; ++k) gc = min(gc, (int32_t)S.llp[k]);
    DfsState st{0, 0, 0, 0, S.llen[0], 0, false, gc};
    DfsPrefetch f;
    DfsFast xa, xb;
    xa.on = false;   // (the first leaf: its whole path, the general path)
    // (its first chunk: of the shared prefix when there is one, applied first)
    dfs_prefetch(d, S, 0, min(kWave, gc > 0 ? gc : st.len), c0, lane, f);
    xb.on = false;
    if (i0 + 1 < i1) dfs_fast_prefetch(d, S, st.len, S.llen[1] - S.llp[1], lane, xb);
    // two leaves per trip, the roles of the two transition buffers swapped by the code rather
    // than by register moves (a move of a load's destination would wait for the load)
    for (int32_t i = i0; i < i1; i += 2) {
        dfs_leaf(d, S, st, i, i0, i1, t, c0, n, lane, f, xa, xb);
        if (i + 1 < i1) dfs_leaf(d, S, st, i + 1, i0, i1, t, c0, n, lane, f, xb, xa);
    }
}

// getCodeFromNucleotide (src/panman.cpp:78-113) for the replayed characters; the reroot
// driver turns '-' and the 'x' sentinel into state 1 = code 0 (src/reroot.cpp:176-181).
__device__ __forceinline__ uint32_t code_of_char(char ch) {
    switch (ch) {
        case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
        case 'R': return 5;  case 'Y': return 10; case 'S': return 6;  case 'W': return 9;
        case 'K': return 12; case 'M': return 3;  case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7;  case 'N': return 15;
        default: return 0;
    }
}

// One thread per output byte (two columns); row reads and code writes are coalesced.
__global__ __launch_bounds__(256) void k_rows_to_codes(const char* rows, int64_t row_stride, int32_t leaves, int64_t c0,
                                                       int64_t n, uint8_t* out, int64_t out_stride) {
    const int64_t per_row = (n + 1) / 2;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= per_row * leaves) return;
    const int64_t leaf = t / per_row, b = t % per_row;
    const char* r = rows + leaf * row_stride + c0 + 2 * b;
    uint32_t v = code_of_char(r[0]);
    if (2 * b + 1 < n) v |= code_of_char(r[1]) << 4;
    out[leaf * out_stride + b] = (uint8_t)v;
}

__device__ __forceinline__ char complement_of(char c) {   // getComplementCharacter (src/panman.cpp:171-204)
    switch (c) {
        case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
        case 'R': return 'Y'; case 'Y': return 'R'; case 'S': return 'S'; case 'W': return 'W';
        case 'K': return 'M'; case 'M': return 'K'; case 'B': return 'V'; case 'D': return 'H';
        case 'H': return 'D'; case 'V': return 'B';
        default: return 'N';
    }
}

__device__ __forceinline__ bool fmt_keep(char ch, bool aligned) { return ch != 'x' && (aligned || ch != '-'); }

// Block-wide sum / exclusive scan over 256 threads (4 waves).
__device__ __forceinline__ int64_t block_sum(int64_t v, int64_t* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const int64_t t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}

// chars each (leaf, print position) segment prints
__global__ __launch_bounds__(256) void k_fmt_count(FmtArgs f) {
    __shared__ int64_t red[4];
    const int32_t leaf = blockIdx.y, pos = blockIdx.x;
    const size_t k = (size_t)leaf * f.positions + pos;
    const FmtSeg sg = f.seg[k];
    if (sg.src < 0) {
        if (threadIdx.x == 0) f.seg_len[k] = f.aligned ? sg.width : 0;
        return;
    }
    const char* row = f.rows + (size_t)leaf * f.row_stride + sg.src;
    int64_t n = 0;
    for (int64_t j = threadIdx.x; j < sg.width; j += blockDim.x) n += fmt_keep(row[j], f.aligned);
    n = block_sum(n, red);
    if (threadIdx.x == 0) f.seg_len[k] = n;
}

// write every segment's chars at their wrapped, rotated place in the leaf's record
__global__ __launch_bounds__(256) void k_fmt_write(FmtArgs f) {
    __shared__ int64_t red[4];
    __shared__ int64_t wsum[4];
    const int32_t leaf = blockIdx.y, pos = blockIdx.x;
    const size_t k = (size_t)leaf * f.positions + pos;
    const FmtSeg sg = f.seg[k];
    const int64_t L = f.line_len[leaf], st = f.start[leaf];
    const int64_t n0 = f.name_off[leaf], n1 = f.name_off[leaf + 1];
    char* rec = f.text + f.text_off[leaf];
    const int64_t hdr = (n1 - n0) + 2;   // '>' name '\n'
    if (pos == 0) {
        if (threadIdx.x == 0) {
            rec[0] = '>';
            rec[hdr - 1] = '\n';
            rec[hdr + L + L / 70] = '\n';   // the caller's final newline (src/fasta.cpp:2094)
        }
        for (int64_t j = threadIdx.x; j < n1 - n0; j += blockDim.x) rec[1 + j] = f.names[n0 + j];
    }
    auto place = [&](int64_t p, char ch) {
        const int64_t q = L ? (p - st + L) % L : 0;
        const int64_t o = hdr + q + q / 70;
        rec[o] = ch;
        if (q % 70 == 69) rec[o + 1] = '\n';
    };
    const int64_t base = f.seg_off[k];
    if (sg.src < 0) {
        if (!f.aligned) return;
        for (int64_t j = threadIdx.x; j < sg.width; j += blockDim.x) place(base + j, '-');
        return;
    }
    const char* row = f.rows + (size_t)leaf * f.row_stride + sg.src;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t done = 0;
    for (int64_t j0 = 0; j0 < sg.width; j0 += blockDim.x) {
        const int64_t j = j0 + threadIdx.x;
        char ch = 0;
        bool keep = false;
        if (j < sg.width) {
            ch = sg.rev ? row[sg.width - 1 - j] : row[j];
            keep = fmt_keep(ch, f.aligned);
            if (sg.rev && ch != '-') ch = complement_of(ch);
        }
        const uint64_t m = __ballot(keep);
        const int64_t below = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int64_t before = 0;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        const int64_t chunk = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (keep) place(base + done + before + below, ch);
        done += chunk;
        __syncthreads();
    }
    (void)red;
}

}  // namespace

hipError_t launch_rows_to_codes(pm_ctx* c, const char* rows, int64_t row_stride, int32_t leaves, int64_t c0, int64_t n,
                                uint8_t* out, int64_t out_stride) {
    const int64_t total = (n + 1) / 2 * leaves;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rows_to_codes, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream, rows, row_stride,
                       leaves, c0, n, out, out_stride);
    return hipGetLastError();
}

hipError_t launch_fmt_count(pm_ctx* c, const FmtArgs& f, int32_t leaves) {
    if (leaves == 0 || f.positions == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fmt_count, dim3((unsigned)f.positions, (unsigned)leaves), dim3(256), 0, c->stream, f);
    return hipGetLastError();
}

hipError_t launch_fmt_write(pm_ctx* c, const FmtArgs& f, int32_t leaves) {
    if (leaves == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fmt_write, dim3((unsigned)std::max(f.positions, 1), (unsigned)leaves), dim3(256), 0, c->stream, f);
    return hipGetLastError();
}

hipError_t launch_replay(pm_ctx* c, const ReplayDev& d) {
    if (d.leaves == 0) return hipSuccess;
    timer_begin(c, 3);
    const unsigned groups = (unsigned)((d.tiles + kReplayGroup - 1) / kReplayGroup);
    if (d.dfs) {
        hipLaunchKernelGGL(k_replay_dfs, dim3((unsigned)((int64_t)d.groups * d.tiles)), dim3(kWave), 0, c->stream, d);
    } else {
        const size_t ring_bytes = (size_t)3 * d.ring * sizeof(int2);
        hipLaunchKernelGGL(k_replay, dim3((unsigned)d.leaves, groups), dim3(256), ring_bytes, c->stream, d);
    }
    timer_end(c, 3);
    return hipGetLastError();
}

// This file's code object, loaded ahead of its first launch (pm_warmup).
hipError_t warm_replay() {
    hipFuncAttributes at;
    return hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_fmt_count));
}

}  // namespace pm
