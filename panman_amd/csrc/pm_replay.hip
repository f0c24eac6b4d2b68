// pm_replay.hip -- root-to-leaf mutation replay for FASTA extraction (gfx950).
//
// Restates the per-leaf sequence reconstruction of Tree::printFASTAUltraFast
// (src/fasta.cpp:1993-2089) and printFASTAUltraFastHelper's mutation pass (:1795-1935):
// every leaf starts from the expanded block consensus (gap slots as '-') and applies the
// nucleotide mutations of each node on its root->leaf path in order, only for blocks that
// are present at the leaf (blockSequence, :1766-1787, :1842).
//
//   k_replay_piped  one workgroup per (leaf, 8 column tiles of 16 KiB): consensus tile -> LDS,
//                   the path nodes' edits inside the tile applied root first by all four
//                   waves, 64 path nodes (one chunk) at a time (edits of one node are unique
//                   per column and sorted by column on the host, so a per-(node, tile) offset
//                   table bounds each node's slice), absent blocks restored, one coalesced
//                   write of the tile: 1 B per leaf-column to HBM, the replay roofline of
//                   SURVEY.md §8d.  Any depth: a SARS-like tree's 280-node paths are 5 chunks.
#include "pm_bits.h"
#include "pm_internal.h"

namespace pm {
namespace {

// The path's edits that fall in column tile t, applied to the LDS tile by ONE wave.  Only
// an edit that overwrites an ancestor's edit of the same column (kEditOverrides, marked on
// the host) needs ordering: the others touch distinct columns along any one path and are
// written in any order, the overriding ones after them node by node, root first -- the
// LDS writes of a wave take effect in issue order, so a descendant's edit wins without a
// barrier.  A chunk is up to 64 path nodes: their slice bounds (one load per lane) and a
// wave prefix sum of the slice lengths; a round gathers up to kEditsPerLane x 64 of the
// chunk's edits at once (one memory round trip).
#ifndef PM_REPLAY_EPL
#define PM_REPLAY_EPL 4
#endif
constexpr int kEditsPerLane = PM_REPLAY_EPL;

struct EditChunk {
    int cnt;
    int64_t lo;       // this lane's node: first edit of its slice
    int32_t len;      // this lane's node: slice length
    int32_t excl;     // exclusive prefix of the lengths
    int32_t total;    // edits in the chunk
};

// A round in flight: col / chr straight from their loads (not combined with anything
// until edit_write, so a prefetched round does not wait for its loads), node8 = path
// position << 8, kNoEdit: none.
struct EditRound {
    uint32_t col[kEditsPerLane];
    uint32_t chr[kEditsPerLane];
    uint32_t node8[kEditsPerLane];
};
constexpr uint32_t kNoEdit = ~0u;

__device__ __forceinline__ void edit_round(const ReplayDev& d, const EditChunk& c, int32_t base, int64_t c0, int lane,
                                           EditRound& r) {
    int64_t e[kEditsPerLane];
    int32_t node[kEditsPerLane];
    const uint32_t lo_lo = (uint32_t)c.lo, lo_hi = (uint32_t)(c.lo >> 32);
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        // edit g of the chunk belongs to the last path node whose slice starts at or
        // before g: a binary search over the lanes' prefix sums (64 nodes: 6 steps)
        const int32_t g = base + lane + j * kWave;
        int k_lo = 0, k_hi = c.cnt - 1;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const int mid = (k_lo + k_hi + 1) >> 1;
            if (__shfl(c.excl, mid) <= g) k_lo = mid;
            else k_hi = mid - 1;
        }
        const int32_t ek = __shfl(c.excl, k_lo);
        const int64_t lok = (int64_t)(((uint64_t)(uint32_t)__shfl((int)lo_hi, k_lo) << 32) |
                                      (uint32_t)__shfl((int)lo_lo, k_lo));
        node[j] = g < c.total ? k_lo : -1;
        e[j] = lok + (g - ek);
    }
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        r.col[j] = (uint32_t)c0;
        r.chr[j] = 0;
        if (node[j] >= 0) {
            r.col[j] = d.edit_col[e[j]];
            r.chr[j] = d.edit_chr[e[j]];
        }
        r.node8[j] = node[j] >= 0 ? (uint32_t)node[j] << 8 : kNoEdit;
    }
}

// A round's edits in two halves: the ones that overwrite no ancestor's edit (returns whether
// the round holds any overriding one, wave-uniform) ...
__device__ __forceinline__ bool edit_write_plain(const EditRound& r, char* buf, int64_t c0) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        const bool ok = r.node8[j] != kNoEdit;
        const bool ovr = ok && (r.chr[j] & kEditOverrides);
        if (ok && !ovr) buf[r.col[j] - c0] = (char)(r.chr[j] & 0x7fu);
        any |= __ballot(ovr) != 0;
    }
    return any;
}

// ... and its overriding ones, node by node in path order: the first pending edit (edits are
// in path order) names the next node
__device__ __forceinline__ void edit_write_overrides(const EditRound& r, char* buf, int64_t c0) {
    const int lane = (int)threadIdx.x & (kWave - 1);
    uint64_t pend[kEditsPerLane];
    bool any = false;
#pragma unroll
    for (int j = 0; j < kEditsPerLane; ++j) {
        pend[j] = __ballot(r.node8[j] != kNoEdit && (r.chr[j] & kEditOverrides));
        any |= pend[j] != 0;
    }
    while (any) {
        uint32_t k = 0;
        bool found = false;
#pragma unroll
        for (int j = 0; j < kEditsPerLane; ++j)
            if (!found && pend[j]) {
                k = (uint32_t)__builtin_amdgcn_readlane(r.node8[j], (int)__builtin_ctzll(pend[j])) >> 8;
                found = true;
            }
        any = false;
#pragma unroll
        for (int j = 0; j < kEditsPerLane; ++j) {
            const bool mine = ((pend[j] >> lane) & 1ull) && (r.node8[j] >> 8) == k;
            if (mine) buf[r.col[j] - c0] = (char)(r.chr[j] & 0x7fu);
            pend[j] &= ~__ballot(mine);
            any |= pend[j] != 0;
        }
    }
}

// A chunk from slice bounds already in registers (the short-path pipeline below).
__device__ __forceinline__ EditChunk edit_chunk_from(int cnt, int64_t lo, int64_t hi, int lane) {
    EditChunk c;
    c.cnt = cnt;
    c.lo = lo;
    c.len = lane < cnt ? (int32_t)(hi - lo) : 0;
    const int32_t incl = (int32_t)wave_inclusive_scan((uint32_t)c.len);
    c.total = __builtin_amdgcn_readlane(incl, kWave - 1);
    c.excl = incl - c.len;
    return c;
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

#ifndef PM_REPLAY_PIPED_WAVES
#define PM_REPLAY_PIPED_WAVES 6
#endif
// PM_REPLAY_DB: two LDS tile buffers -- tile t + 1's consensus copy-in is issued as tile t's
// edits start, so it lands behind them instead of heading tile t + 1's critical path.  Off:
// the second 16 KiB buffer takes the kernel from 6 to 4 workgroups per CU (LDS), and C5 went
// 1.75 -> 2.04 ms (r04i, interleaved).
#ifndef PM_REPLAY_DB
#define PM_REPLAY_DB 0
#endif
constexpr int kReplayBufs = PM_REPLAY_DB ? 2 : 1;

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

// One chunk's edits of a tile, all four waves: every wave holds the chunk's slice bounds
// (lane = path node) and takes every fourth round (a super-round = 4 x kEditsPerLane x 64
// edits; a C5 tile has ~800).  Edits that overwrite no ancestor's edit touch distinct columns
// along the path, so the waves write them in any order; the overriding ones (kEditOverrides,
// rare) follow wave by wave -- the rounds are in path order -- with a barrier between, and
// only in a super-round that has any.  Every super-round ends in a barrier, so the next
// chunk's (deeper nodes') overriding edits land after this chunk's writes.  `r` holds the
// wave's first round, already issued.
__device__ __forceinline__ void chunk_edits(const ReplayDev& d, const EditChunk& ch, EditRound& r, char* buf,
                                            int64_t c0, int wave, int lane) {
    constexpr int32_t R = kEditsPerLane * kWave;
    for (int32_t sr = 0; sr < ch.total; sr += 4 * R) {   // (uniform: every wave holds the same chunk)
        const int32_t base = sr + wave * R;
        if (sr > 0 && base < ch.total) edit_round(d, ch, base, c0, lane, r);   // (super-round 0: prefetched)
        const bool ovr = base < ch.total && edit_write_plain(r, buf, c0);
        if (__syncthreads_or(ovr)) {
            for (int w = 0; w < 4; ++w) {
                if (wave == w && base < ch.total) edit_write_overrides(r, buf, c0);
                __syncthreads();
            }
        }
    }
}

// Slice bounds of chunk [q, q + 64) of the path at tile t (lane = path node); the path ids
// and the bounds are two dependent loads, issued for chunk k + 1 before chunk k's rounds.
struct ChunkBounds {
    int cnt;
    int64_t lo, hi;
};

__device__ __forceinline__ ChunkBounds chunk_bounds(const ReplayDev& d, int64_t q, int64_t p1, int32_t t, int lane) {
    ChunkBounds b{(int)min((int64_t)kWave, p1 - q), 0, 0};
    if (lane < b.cnt) {
        const int64_t* te = d.tile_edit + (size_t)d.path[q + lane] * (d.tiles + 1) + t;
        b.lo = te[0];
        b.hi = te[1];
    }
    return b;
}

// Each wave prefetches its first round of the next tile's first chunk while the tile is
// restored and written out, so a tile's edits cost LDS writes, not a chain of memory round
// trips in one wave (round 3's single-editor kernel: ~10 us per 16 KiB tile at C5).  Paths
// deeper than 64 nodes walk their further chunks after the first, each chunk's bounds loaded
// while the previous chunk's rounds run.
__global__ __launch_bounds__(256, PM_REPLAY_PIPED_WAVES) void k_replay_piped(ReplayDev d) {
    __shared__ uint4 tile_buf[kReplayBufs][kReplayTile / 16];
    __shared__ int32_t rng[2][2 + 2 * kRestoreRanges];
    const int32_t leaf = blockIdx.x;
    const int32_t t_begin = (int32_t)blockIdx.y * kReplayGroup;
    const int32_t t_end = min(d.tiles, t_begin + kReplayGroup);
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & (kWave - 1);
    constexpr int32_t R = kEditsPerLane * kWave;   // edits per wave-round
    const int64_t p0 = d.path_off[leaf], p1 = d.path_off[leaf + 1];
    const int cnt = (int)min((int64_t)kWave, p1 - p0);
    const int64_t* te = nullptr;
    int64_t te_next = 0, te_next2 = 0;   // this lane's node: slice starts of tiles t+1, t+2
    EditChunk ch{};
    EditRound r{};
    if (cnt > 0) {
        const int32_t node = lane < cnt ? d.path[p0 + lane] : d.path[p0];
        te = d.tile_edit + (size_t)node * (d.tiles + 1);
        const int64_t te_cur = te[t_begin];
        te_next = te[t_begin + 1];
        if (t_begin + 2 <= d.tiles) te_next2 = te[t_begin + 2];
        ch = edit_chunk_from(cnt, te_cur, te_next, lane);
        if (wave * R < ch.total) edit_round(d, ch, wave * R, (int64_t)t_begin * kReplayTile, lane, r);
    }
    if (tid == kWave) absent_ranges(d, leaf, t_begin, rng[0]);
    if (kReplayBufs == 2) tile_copy_in(d, t_begin, tile_buf[0], wave, lane);
    for (int32_t t = t_begin; t < t_end; ++t) {
        const int64_t c0 = (int64_t)t * kReplayTile;
        const int64_t n = min(kReplayTile, d.row_stride - c0);   // multiple of 16
        uint4* cur = tile_buf[kReplayBufs == 2 ? (t - t_begin) & 1 : 0];
        char* buf = reinterpret_cast<char*>(cur);
        if (kReplayBufs == 1) tile_copy_in(d, t, cur, wave, lane);
        __syncthreads();   // tile t's copy-in landed; (two buffers) tile t - 1's write-out read its buffer
        if (kReplayBufs == 2 && t + 1 < t_end) tile_copy_in(d, t + 1, tile_buf[(t + 1 - t_begin) & 1], wave, lane);
        if (p1 - p0 <= kWave) {
            chunk_edits(d, ch, r, buf, c0, wave, lane);
        } else {
            ChunkBounds nb = chunk_bounds(d, p0 + kWave, p1, t, lane);
            chunk_edits(d, ch, r, buf, c0, wave, lane);
            for (int64_t q = p0 + kWave; q < p1; q += kWave) {
                const EditChunk cq = edit_chunk_from(nb.cnt, nb.lo, nb.hi, lane);
                if (wave * R < cq.total) edit_round(d, cq, wave * R, c0, lane, r);
                if (q + kWave < p1) nb = chunk_bounds(d, q + kWave, p1, t, lane);
                chunk_edits(d, cq, r, buf, c0, wave, lane);
            }
        }
        restore_absent(d, leaf, t, rng[(t - t_begin) & 1], buf, tid, blockDim.x);
        if (cnt > 0 && t + 1 < t_end) {
            // the next tile's first rounds, in flight through the restore / write / copy
            ch = edit_chunk_from(cnt, te_next, te_next2, lane);
            te_next = te_next2;
            if (t + 3 <= d.tiles) te_next2 = te[t + 3];
            if (wave * R < ch.total) edit_round(d, ch, wave * R, c0 + kReplayTile, lane, r);
        }
        if (tid == kWave && t + 1 < t_end) absent_ranges(d, leaf, t + 1, rng[(t + 1 - t_begin) & 1]);
        __syncthreads();
        uint4* dst = reinterpret_cast<uint4*>(d.rows + (size_t)leaf * d.row_stride + c0);
        for (int64_t k = tid; k < n / 16; k += blockDim.x) dst[k] = cur[k];
        if (kReplayBufs == 1) __syncthreads();   // the tile buffer is refilled next
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
    hipLaunchKernelGGL(k_replay_piped, dim3((unsigned)d.leaves, groups), dim3(256), 0, c->stream, d);
    timer_end(c, 3);
    return hipGetLastError();
}

}  // namespace pm
