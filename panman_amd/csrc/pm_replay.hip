// pm_replay.hip -- root-to-leaf mutation replay for FASTA extraction (gfx950).
//
// Restates the per-leaf sequence reconstruction of Tree::printFASTAUltraFast
// (src/fasta.cpp:1993-2089) and printFASTAUltraFastHelper's mutation pass (:1795-1935):
// every leaf starts from the expanded block consensus (gap slots as '-') and applies the
// nucleotide mutations of each node on its root->leaf path in order, only for blocks that
// are present at the leaf (blockSequence, :1766-1787, :1842).
//
//   k_replay_fill   rows[leaf][col] = consensus row; 16 B per lane, HBM-write bound
//                   (1 B per leaf-column, the replay roofline of SURVEY.md §8d).
//   k_replay_apply  one workgroup per leaf: the path (parent pointers) is staged in LDS,
//                   then each path node's edits are written by all lanes, one barrier per
//                   node so a descendant's write wins (edits of one node are unique per
//                   column, resolved on the host in list order).
#include "pm_internal.h"

namespace pm {
namespace {

__global__ __launch_bounds__(256) void k_replay_fill(char* rows, const char* cons_row, int64_t stride, int32_t leaves) {
    const int64_t vec = stride / 16;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= vec * leaves) return;
    const int64_t leaf = t / vec, k = t % vec;
    reinterpret_cast<uint4*>(rows + leaf * stride)[k] = reinterpret_cast<const uint4*>(cons_row)[k];
}

constexpr int kMaxDepth = 8192;

__global__ __launch_bounds__(256) void k_replay_apply(ReplayDev d) {
    __shared__ int32_t path[kMaxDepth];
    __shared__ int32_t depth;
    const int32_t leaf = blockIdx.x;
    if (threadIdx.x == 0) {
        int32_t n = d.leaf_node[leaf], k = 0;
        while (n >= 0 && k < kMaxDepth) {
            path[k++] = n;
            n = d.parent[n];
        }
        depth = k;
    }
    __syncthreads();
    const uint32_t* pres = d.presence + (size_t)leaf * d.presence_words;
    char* row = d.rows + (size_t)leaf * d.row_stride;
    for (int32_t k = depth - 1; k >= 0; --k) {   // root first
        const int32_t n = path[k];
        const int64_t e0 = d.edit_off[n], e1 = d.edit_off[n + 1];
        if (e0 == e1) continue;   // uniform: no barrier needed
        for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
            const int32_t b = d.edit_blk[e];
            if ((pres[b >> 5] >> (b & 31)) & 1u) row[d.edit_col[e]] = (char)d.edit_chr[e];
        }
        __syncthreads();
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

}  // namespace

hipError_t launch_rows_to_codes(pm_ctx* c, const char* rows, int64_t row_stride, int32_t leaves, int64_t c0, int64_t n,
                                uint8_t* out, int64_t out_stride) {
    const int64_t total = (n + 1) / 2 * leaves;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rows_to_codes, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream, rows, row_stride,
                       leaves, c0, n, out, out_stride);
    return hipGetLastError();
}

hipError_t launch_replay(pm_ctx* c, const ReplayDev& d) {
    if (d.leaves == 0) return hipSuccess;
    if (d.max_depth > kMaxDepth) return hipErrorNotSupported;
    const int64_t n = d.row_stride / 16 * d.leaves;
    timer_begin(c, 3);
    hipLaunchKernelGGL(k_replay_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, d.rows, d.cons_row,
                       d.row_stride, d.leaves);
    hipLaunchKernelGGL(k_replay_apply, dim3(d.leaves), dim3(256), 0, c->stream, d);
    timer_end(c, 3);
    return hipGetLastError();
}

}  // namespace pm
