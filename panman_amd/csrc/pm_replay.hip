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

__device__ __forceinline__ void absent_ranges(const ReplayDev& d, int32_t leaf, int32_t t, int32_t* rng) {
    const int64_t c0 = (int64_t)t * kReplayTile, c1 = min(c0 + kReplayTile, d.row_stride);
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

// A workgroup barrier that orders LDS only: each wave's LDS accesses are complete (lgkmcnt)
// and visible to the others, while its global stores and loads stay in flight.  __syncthreads()
// is a workgroup release / acquire over global memory too, which on gfx950 waits for every
// outstanding vector memory operation (vmcnt(0)): behind the write-out that is a full HBM
// write round trip per tile, and before it the next tile's prefetched edit loads.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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
            if (k < n / 16) dst[k] = tile_buf[k];
        }
        lds_barrier();   // the tile buffer is refilled next
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
    const size_t ring_bytes = (size_t)3 * d.ring * sizeof(int2);
    hipLaunchKernelGGL(k_replay, dim3((unsigned)d.leaves, groups), dim3(256), ring_bytes, c->stream, d);
    timer_end(c, 3);
    return hipGetLastError();
}

}  // namespace pm
