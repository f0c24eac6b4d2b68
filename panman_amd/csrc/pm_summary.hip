// pm_summary.hip -- `panmanUtils --summary` over a loaded PanMAT (src/summary.cpp).
//
// Tree::printSummary (src/summary.cpp:257-273) is a set of reductions over every node's
// mutation lists (getTotalParsimonyParallelHelper :3-59, getBlockMutationsParallelHelper
// :61-109, tbb::parallel_reduce over a recursion in the reference).  Here the lists are
// flat CSR arrays, so one kernel reduces them all at once: every thread classifies one
// NucMut and one block mutation, a wave sums with DPP-free shuffles and one lane per wave
// adds into 7 counters.  What is sequential by definition stays on the host: the leaf depths
// (the reference sums them into a float in Newick leaf order, src/panman.cpp:386-394 -- an
// order-dependent rounding) and the duplication / translocation walk (:111-193, a DFS
// carrying the block-presence vector).
#include <map>
#include <tuple>
#include <vector>

#include "pm_internal.h"

namespace pm {
namespace {

enum SumIdx { kNS, kNI, kND, kBI, kBD, kInv, kBDInv, kSumCount };

__global__ __launch_bounds__(kBlock) void k_summary(const uint8_t* nuc_info, int64_t nuc_n, const uint8_t* bm_info,
                                                    const uint8_t* bm_inv, int64_t bm_n,
                                                    unsigned long long* out) {
    uint32_t c[kSumCount] = {0, 0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nuc_n || i < bm_n; i += stride) {
        if (i < nuc_n) {   // NucMut::type() = mutInfo & 7, length() = mutInfo >> 4 (src/panman.hpp:251-258)
            const uint32_t info = nuc_info[i], type = info & 7u;
            c[kNS] += type == PM_MUT_NS ? info >> 4 : 0u;
            c[kNI] += type == PM_MUT_NI;
            c[kND] += type == PM_MUT_ND;
        }
        if (i < bm_n) {    // BlockMut: blockMutInfo 1 = BI, 0 = BD; inversion flag
            const bool ins = bm_info[i] != 0, inv = bm_inv[i] != 0;
            c[kBI] += ins;
            c[kBD] += !ins && !inv;
            c[kInv] += inv;
            c[kBDInv] += !ins && inv;
        }
    }
#pragma unroll
    for (int k = 0; k < kSumCount; ++k) {
        uint32_t v = c[k];
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & (kWave - 1)) == 0 && v) atomicAdd(&out[k], (unsigned long long)v);
    }
}

template <class T>
hipError_t to_device(const T* src, int64_t n, T** dst, hipStream_t s) {
    *dst = nullptr;
    if (n <= 0) return hipSuccess;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), sizeof(T) * n);
    if (e == hipSuccess) e = hipMemcpyAsync(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice, s);
    return e;
}

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" int pm_summary_compute(pm_ctx* c, const pm_panmat* p, pm_summary* out) {
    if (!c || !p || !out || p->num_nodes < 1 || p->root < 0 || p->root >= p->num_nodes || !p->child_offsets)
        return c ? fail(c, PM_ERR_ARG, "bad PanMAT") : PM_ERR_ARG;
    (void)hipSetDevice(c->device);
    const int32_t N = p->num_nodes;
    const int64_t nuc_n = p->nuc_mut_offsets ? p->nuc_mut_offsets[N] : 0;
    const int64_t bm_n = p->block_mut_offsets ? p->block_mut_offsets[N] : 0;
    uint8_t *d_nuc = nullptr, *d_bi = nullptr, *d_binv = nullptr;
    unsigned long long* d_out = nullptr;
    unsigned long long h[kSumCount] = {0, 0, 0, 0, 0, 0, 0};
    hipError_t e = to_device(p->nuc_mut_info, nuc_n, &d_nuc, c->stream);
    if (e == hipSuccess) e = to_device(p->block_mut_info, bm_n, &d_bi, c->stream);
    if (e == hipSuccess) e = to_device(p->block_mut_inversion, bm_n, &d_binv, c->stream);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_out), sizeof h);
    if (e == hipSuccess) e = hipMemsetAsync(d_out, 0, sizeof h, c->stream);
    if (e == hipSuccess && (nuc_n > 0 || bm_n > 0)) {
        const int64_t n = std::max(nuc_n, bm_n);
        const unsigned blocks = (unsigned)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_summary, dim3(blocks), dim3(kBlock), 0, c->stream, d_nuc, nuc_n, d_bi, d_binv, bm_n, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, d_out, sizeof h, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_nuc);
    (void)hipFree(d_bi);
    (void)hipFree(d_binv);
    (void)hipFree(d_out);
    if (e != hipSuccess) return hip_fail(c, e, "summary reduction");

    // leaf depths in Newick leaf order (pre-order, children in list order), float sum as the
    // Newick parser does (src/panman.cpp:386-394); internal node count = m_currInternalNode
    int64_t internal = 0, leaves = 0;
    size_t max_depth = 0;
    float mean = 0.f;
    std::vector<std::pair<int32_t, size_t>> stack{{p->root, 0}};
    std::vector<int32_t> order;   // pre-order, for the block walk
    order.reserve(N);
    while (!stack.empty()) {
        const auto [v, depth] = stack.back();
        stack.pop_back();
        order.push_back(v);
        const int32_t a = p->child_offsets[v], b = p->child_offsets[v + 1];
        if (a == b) {
            ++leaves;
            max_depth = std::max(max_depth, depth);
            mean += depth;
        } else {
            ++internal;
        }
        for (int32_t k = b - 1; k >= a; --k) stack.push_back({p->child_index[k], depth + 1});
    }
    if ((int32_t)order.size() != N) return fail(c, PM_ERR_ARG, "PanMAT is not one tree");
    mean /= (float)leaves;

    // duplications / translocations (src/summary.cpp:111-193, 203-250): blocks grouped by
    // identical consensusSeq; a DFS carrying block presence, undone on the way back up
    const int32_t B = p->num_blocks;
    std::map<std::vector<uint32_t>, std::vector<int32_t>> by_seq;
    for (int32_t i = 0; i < B; ++i)
        by_seq[std::vector<uint32_t>(p->block_seq + p->block_seq_offsets[i], p->block_seq + p->block_seq_offsets[i + 1])]
            .push_back(p->block_primary[i]);
    std::vector<int32_t> group_of(B, 0);
    std::vector<std::vector<int32_t>> groups;
    for (auto& kv : by_seq) {
        for (int32_t b : kv.second)
            if (b >= 0 && b < B) group_of[b] = (int32_t)groups.size();
        groups.push_back(kv.second);
    }
    int64_t dup = 0, trans = 0;
    if (bm_n > 0) {
        std::vector<uint8_t> exists(B, 0), strand(B, 1);
        // a block's presence before the current node's mutations: `prior` for the blocks
        // this node touches (first old value), `exists` for the others -- no O(B) copy per node
        constexpr uint8_t kUntouched = 0xff;
        std::vector<uint8_t> prior(B, kUntouched);
        struct Frame {
            int32_t v;
            int32_t next_child;
            std::vector<std::tuple<int32_t, uint8_t, uint8_t>> undo;
        };
        std::vector<Frame> st;
        auto enter = [&](int32_t v) {
            Frame f{v, p->child_offsets[v], {}};
            for (int64_t k = p->block_mut_offsets[v]; k < p->block_mut_offsets[v + 1]; ++k) {
                const int32_t b = p->block_mut_primary[k];
                if (b < 0 || b >= B) continue;
                if (prior[b] == kUntouched) prior[b] = exists[b];
                f.undo.emplace_back(b, exists[b], strand[b]);
                const bool inv = p->block_mut_inversion[k] != 0;
                if (p->block_mut_info[k]) {
                    exists[b] = 1;
                    strand[b] = !inv;
                } else if (inv) {
                    strand[b] = !strand[b];
                } else {
                    exists[b] = 0;
                    strand[b] = 1;
                }
            }
            for (int64_t k = p->block_mut_offsets[v]; k < p->block_mut_offsets[v + 1]; ++k) {
                const int32_t b = p->block_mut_primary[k];
                if (!p->block_mut_info[k] || b < 0 || b >= B) continue;
                for (int32_t d : groups[group_of[b]]) {
                    if (d == b || d < 0 || d >= B) continue;
                    const bool before = prior[d] != kUntouched ? prior[d] != 0 : exists[d] != 0;
                    if (exists[d] && before) { ++dup; break; }
                    if (!exists[d] && before) { ++trans; break; }
                }
            }
            for (const auto& u : f.undo) prior[std::get<0>(u)] = kUntouched;
            st.push_back(std::move(f));
        };
        enter(p->root);
        while (!st.empty()) {
            Frame& f = st.back();
            if (f.next_child < p->child_offsets[f.v + 1]) {
                enter(p->child_index[f.next_child++]);
                continue;
            }
            for (auto it = f.undo.rbegin(); it != f.undo.rend(); ++it) {
                exists[std::get<0>(*it)] = std::get<1>(*it);
                strand[std::get<0>(*it)] = std::get<2>(*it);
            }
            st.pop_back();
        }
    }

    out->nodes = internal + leaves;
    out->samples = leaves;
    out->substitutions = (int64_t)h[kNS];
    out->insertions = (int64_t)(h[kNI] + h[kBI]);
    out->deletions = (int64_t)(h[kND] + h[kBD]);
    out->inversions = (int64_t)h[kInv];
    out->max_depth = (int64_t)max_depth;
    out->mean_depth = mean;
    out->block_insertions = (int64_t)h[kBI];
    out->block_deletions = (int64_t)h[kBD];
    out->block_inversions = (int64_t)h[kBDInv];
    out->block_duplications = dup;
    out->block_translocations = trans;
    return PM_OK;
}
