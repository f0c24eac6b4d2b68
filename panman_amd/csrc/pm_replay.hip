// pm_replay.hip -- root-to-leaf mutation replay for FASTA extraction (gfx950).
//
// Restates the per-leaf sequence reconstruction of Tree::printFASTAUltraFast
// (src/fasta.cpp:1993-2089) and printFASTAUltraFastHelper's mutation pass (:1795-1935):
// every leaf starts from the expanded block consensus (gap slots as '-') and applies the
// nucleotide mutations of each node on its root->leaf path in order, only for blocks that
// are present at the leaf (blockSequence, :1766-1787, :1842).
//
//   k_replay_tile   one workgroup per (leaf, 32 KiB column tile): consensus tile -> LDS,
//                   the path nodes' edits inside the tile applied root first (edits of one
//                   node are unique per column and sorted by column on the host, so a
//                   per-(node, tile) offset table bounds each node's slice), one coalesced
//                   write of the tile: 1 B per leaf-column to HBM, the replay roofline of
//                   SURVEY.md §8d.
#include "pm_internal.h"

namespace pm {
namespace {

// One workgroup = (leaf, tile of kReplayTile columns): the tile of the leaf's row is
// assembled in LDS -- consensus copy, then each path node's edits that fall in the tile,
// root first, one barrier per node with edits (a descendant's write wins) -- and leaves as
// one coalesced write.  Each row byte is written to HBM once.
__global__ __launch_bounds__(256) void k_replay_tile(ReplayDev d) {
    __shared__ uint4 tile_buf[kReplayTile / 16];
    char* buf = reinterpret_cast<char*>(tile_buf);
    const int32_t leaf = blockIdx.x;
    const int32_t t = blockIdx.y;
    const int64_t c0 = (int64_t)t * kReplayTile;
    const int64_t n = min(kReplayTile, d.row_stride - c0);   // multiple of 16
    const uint4* src = reinterpret_cast<const uint4*>(d.cons_row + c0);
    for (int64_t k = threadIdx.x; k < n / 16; k += blockDim.x) tile_buf[k] = src[k];
    __syncthreads();
    const uint32_t* pres = d.presence + (size_t)leaf * d.presence_words;
    const int64_t p0 = d.path_off[leaf], p1 = d.path_off[leaf + 1];
    // The path's edit slices for this tile, 256 nodes at a time: slice bounds and their
    // prefix sums in LDS, then every thread loads its share of ALL the chunk's edits at
    // once (one round of memory latency instead of one per node), then the edits are
    // written node by node, root first, with a barrier between nodes.
    constexpr int kPer = 8;   // edits per thread per round
    __shared__ int64_t lo[256], pre[257];
    for (int64_t q = p0; q < p1; q += 256) {
        const int cnt = (int)min((int64_t)256, p1 - q);
        if ((int)threadIdx.x < cnt) {
            const int64_t* te = d.tile_edit + (size_t)d.path[q + threadIdx.x] * (d.tiles + 1) + t;
            lo[threadIdx.x] = te[0];
            pre[threadIdx.x + 1] = te[1] - te[0];
        }
        if (threadIdx.x == 0) pre[0] = 0;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 1; k <= cnt; ++k) pre[k] += pre[k - 1];
        __syncthreads();
        const int64_t total = pre[cnt];
        for (int64_t base = 0; base < total; base += (int64_t)kPer * blockDim.x) {
            int node[kPer];
            uint32_t col[kPer];
            char chr[kPer];
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                node[j] = -1;
                const int64_t g = base + threadIdx.x + (int64_t)j * blockDim.x;
                if (g >= total) continue;
                int lo_k = 0, hi_k = cnt - 1;   // last node with pre[k] <= g
                while (lo_k < hi_k) {
                    const int mid = (lo_k + hi_k + 1) >> 1;
                    if (pre[mid] <= g) lo_k = mid;
                    else hi_k = mid - 1;
                }
                const int64_t e = lo[lo_k] + (g - pre[lo_k]);
                node[j] = lo_k;
                col[j] = d.edit_col[e];
                chr[j] = (char)d.edit_chr[e];
            }
            const int64_t hi_g = min(total, base + (int64_t)kPer * blockDim.x);
#ifdef PM_EXP_NOBARRIERS   // timing experiment: edits written in one pass (conflicts unordered)
#pragma unroll
            for (int j = 0; j < kPer; ++j)
                if (node[j] >= 0) buf[col[j] - c0] = chr[j];
            __syncthreads();
            if (hi_g >= 0) continue;
#endif
            for (int k = 0; k < cnt; ++k) {   // root first
                if (pre[k + 1] <= base || pre[k] >= hi_g) continue;   // uniform: no edits this round
#pragma unroll
                for (int j = 0; j < kPer; ++j)
                    if (node[j] == k) buf[col[j] - c0] = chr[j];
                __syncthreads();
            }
        }
        __syncthreads();   // lo / pre are reused by the next chunk
    }
    // blocks absent at the leaf keep the consensus (their edits are not applied: :1842)
    for (int32_t id = d.tile_blk[t]; id < d.blocks; ++id) {
        const int64_t b_lo = d.blk_lo[id];
        if (b_lo >= c0 + n) break;
        if ((pres[id >> 5] >> (id & 31)) & 1u) continue;
        const int64_t a = max(b_lo, c0), b = min(d.blk_hi[id], c0 + n);
        for (int64_t k = a + threadIdx.x; k < b; k += blockDim.x) buf[k - c0] = d.cons_row[k];
    }
    __syncthreads();
    uint4* dst = reinterpret_cast<uint4*>(d.rows + (size_t)leaf * d.row_stride + c0);
    for (int64_t k = threadIdx.x; k < n / 16; k += blockDim.x) dst[k] = tile_buf[k];
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
    hipLaunchKernelGGL(k_replay_tile, dim3((unsigned)d.leaves, (unsigned)d.tiles), dim3(256), 0, c->stream, d);
    timer_end(c, 3);
    return hipGetLastError();
}

}  // namespace pm
