// pm_measure.hip -- measurement helpers for the roofline the bench reports.
//
//   pm_stream_copy_rate  the achievable-HBM reference: a 16-B-per-lane streaming copy
//                        (read + write bytes / s), the access pattern of the level kernels'
//                        leaf-row and record streams.
//   pm_design_bytes      the bytes THIS design must move in one pm_run, counted from the
//                        record masks of the run just made: leaf words, compressed set
//                        records written and read, compact finals, dirty-lane leaf reads,
//                        8 B per mutation record -- each at the 16-B-per-lane granularity the
//                        kernels load and store (cache-resident consensus words excluded).
//                        `achieved` = these bytes / kernel time can therefore not exceed
//                        what the kernels really draw from HBM (PMC FETCH / WRITE sizes).
#include <algorithm>
#include <vector>

#include "pm_kernels.h"

namespace pm {
namespace {

constexpr int kCopyUnroll = 4;

__global__ __launch_bounds__(kBlock) void k_stream_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * kCopyUnroll + threadIdx.x;
    uint4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n) dst[i] = v[u];
    }
}

// Write-only streaming: 16 B per lane, kCopyUnroll non-temporal stores per thread (the
// replay's row stores).
__global__ __launch_bounds__(kBlock) void k_stream_write(uint4* __restrict__ dst, int64_t n, uint32_t tag) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * kCopyUnroll + threadIdx.x;
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
        const int64_t i = base + (int64_t)u * kBlock;
        if (i < n) store_stream(dst + i, make_uint4((uint32_t)i, tag, (uint32_t)(i >> 32), ~tag));
    }
}

// FETCH_SIZE calibration for scattered 16-B-per-lane reads (the pre-order's parent finals and
// dirty-lane leaf words): thread i reads 16 B at i * stride, (i + n) * stride, ... (kGather
// reads, each lane its own 16 B of a stride-spaced slot) and writes one coalesced 16-B XOR.
constexpr int kGather = 4;

__global__ __launch_bounds__(kBlock) void k_gather_probe(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         int64_t n, int64_t stride_q) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kGather; ++u) {
        const uint4 v = src[(i + (int64_t)u * n) * stride_q];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    dst[i] = acc;
}

inline int popc(uint64_t x) { return __builtin_popcountll(x); }

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" {

int pm_stream_copy_rate(int device, int64_t bytes, int reps, double* gbs) {
    if (!gbs || bytes < (1 << 20) || reps < 1) return PM_ERR_ARG;
    *gbs = 0.0;
    if (hipSetDevice(device) != hipSuccess) return PM_ERR_HIP;
    const int64_t n = bytes / (int64_t)sizeof(uint4);
    uint4 *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = PM_OK;
    if (hipMalloc(reinterpret_cast<void**>(&a), n * sizeof(uint4)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&b), n * sizeof(uint4)) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess) {
        rc = PM_ERR_OOM;
    } else {
        const dim3 grid((unsigned)((n + (int64_t)kBlock * kCopyUnroll - 1) / ((int64_t)kBlock * kCopyUnroll)));
        (void)hipMemsetAsync(a, 1, n * sizeof(uint4), s);
        hipLaunchKernelGGL(k_stream_copy, grid, dim3(kBlock), 0, s, a, b, n);   // warm-up
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_stream_copy, grid, dim3(kBlock), 0, s, a, b, n);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.f)
            rc = PM_ERR_HIP;
        else
            *gbs = 2.0 * (double)n * sizeof(uint4) * reps / (ms * 1e-3) / 1e9;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return rc;
}

int pm_stream_write_rate(int device, int64_t bytes, int reps, double* gbs) {
    if (!gbs || bytes < (1 << 20) || reps < 1) return PM_ERR_ARG;
    *gbs = 0.0;
    if (hipSetDevice(device) != hipSuccess) return PM_ERR_HIP;
    const int64_t n = bytes / (int64_t)sizeof(uint4);
    uint4* a = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = PM_OK;
    if (hipMalloc(reinterpret_cast<void**>(&a), n * sizeof(uint4)) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess) {
        rc = PM_ERR_OOM;
    } else {
        const dim3 grid((unsigned)((n + (int64_t)kBlock * kCopyUnroll - 1) / ((int64_t)kBlock * kCopyUnroll)));
        hipLaunchKernelGGL(k_stream_write, grid, dim3(kBlock), 0, s, a, n, 0u);   // warm-up (first touch)
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_stream_write, grid, dim3(kBlock), 0, s, a, n, (uint32_t)r + 1);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.f)
            rc = PM_ERR_HIP;
        else
            *gbs = (double)n * sizeof(uint4) * reps / (ms * 1e-3) / 1e9;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    return rc;
}

int pm_gather_probe(int device, int64_t lanes, int stride_bytes, int reps, double* ms_per_launch) {
    if (!ms_per_launch || lanes < kBlock || stride_bytes < 16 || stride_bytes % 16 || reps < 1) return PM_ERR_ARG;
    *ms_per_launch = 0.0;
    if (hipSetDevice(device) != hipSuccess) return PM_ERR_HIP;
    const int64_t sq = stride_bytes / 16, n = lanes;
    const size_t src_q = (size_t)(n * kGather) * sq;
    uint4 *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = PM_OK;
    if (hipMalloc(reinterpret_cast<void**>(&a), src_q * sizeof(uint4)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&b), n * sizeof(uint4)) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess) {
        rc = PM_ERR_OOM;
    } else {
        const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
        (void)hipMemsetAsync(a, 1, src_q * sizeof(uint4), s);
        hipLaunchKernelGGL(k_gather_probe, grid, dim3(kBlock), 0, s, a, b, n, sq);   // warm-up
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_gather_probe, grid, dim3(kBlock), 0, s, a, b, n, sq);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.f)
            rc = PM_ERR_HIP;
        else
            *ms_per_launch = (double)ms / reps;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return rc;
}

int pm_design_bytes(pm_ctx* c, double* out, int n) {
    if (!c || !out || n < 5) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    const int mode = c->last_mode;
    if (mode != PM_MODE_FITCH && mode != PM_MODE_SANKOFF)
        return fail(c, PM_ERR_UNSUPPORTED, "design bytes are modelled for the nucleotide modes");
    int64_t records = 0;
    int rc = pm_mutation_count(c, &records);
    if (rc != PM_OK) return rc;
    const HostTree& ht = c->ht;
    const int32_t I = c->dt.num_internal, L = c->dt.num_leaves;
    const int32_t tiles = (c->words + kWave - 1) / kWave;
    std::vector<uint64_t> m((size_t)I * tiles * kMaskWords);
    hipError_t e = hipMemcpyAsync(m.data(), c->cmask, m.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "record masks");
    const bool virt = c->virtual_leaf_parents;
    const bool sub = virt && (mode == PM_MODE_FITCH || mode == PM_MODE_SANKOFF) && c->subtree_form && c->leaves_all_present &&
                     ht.num_sshape > 0;
    const int32_t root = c->dt.root_dense;
    // virtual nodes as pm_tree_upload forms them (leaf-parents: not the root, one or two
    // children, all leaves; subtree form: S2 / S3 too): vnode = the leaves their parent reads
    std::vector<uint8_t> vnode(I, 0);
    if (virt)
        for (int32_t d = 0; d < I; ++d) {
            const int32_t deg = ht.child_off[d + 1] - ht.child_off[d];
            bool all = d != root && deg <= 2;
            for (int32_t k = ht.child_off[d]; k < ht.child_off[d + 1] && all; ++k) all = ht.child_enc[k] < 0;
            vnode[d] = all ? (uint8_t)deg : 0;
            if (sub && ht.sshape[d]) vnode[d] = (uint8_t)(ht.sshape[d] + 2);
        }
    const double lane = 16.0, word_row = lane * kWave;   // one lane's code planes; one wave's leaf word
    const bool leaf_rule = mode == PM_MODE_FITCH && c->leaves_all_present;
    const double cx_full = mode == PM_MODE_FITCH ? 64.0 : 128.0;   // complex lane: 16 planes / Z0 + Z1
    const double cx_read_up = 64.0;                                // the parent reads Fitch planes / Z0
    double up = 0.0, down = 0.0;
    // components: up leaf words, up child records, up own records + pushes, down own records,
    // down parent finals, down dirty leaf words (a node's first two children: k_down), down
    // finals written, down tail items (descriptor, parent masks and finals: k_tail), down tail
    // items' dirty leaf words (k_tail)
    double part[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    // The pre-order's reads at the memory's granularity: every load draws whole 128-B lines
    // (tools/calib_fetch.hip: one TCC read request per line touched, for 16-B and 64-B reads at
    // any stride and for scattered ones), so a dirty lane's 16-B word costs a line unless a
    // neighbour in the same line is read too.  The level kernels: line[0] descriptors, masks and
    // own records, [1] parent finals, [2] dirty-lane leaf words; the tail: [3] descriptors and
    // masks, [4] dirty-lane leaf words, [5] parent finals.
    double line[6] = {0, 0, 0, 0, 0, 0};
    const double LB = 128.0;
    const int cx_areas = mode == PM_MODE_FITCH ? 4 : 8;   // complex planes read by the own-record load
    auto groups8 = [](uint64_t v) {   // lines of a per-lane 16-B row (8 lanes a line)
        int k = 0;
        for (int b = 0; b < 8; ++b) k += ((v >> (8 * b)) & 0xFFull) != 0;
        return k;
    };
    auto pairs = [](uint64_t v) { return popc((v | (v >> 1)) & 0x5555555555555555ull); };   // 64-B per-lane rows
    auto ceil8 = [](int v) { return (v + 7) / 8; };

    // lines of a record's area 0 read at lanes dm: simple lanes at their rank, complex lanes'
    // finals after the simple codes (final_slot); consensus lanes read the cached consensus
    auto rank_lines = [](uint64_t dm, uint64_t s, uint64_t x) {
        const int ns = popc(s);
        uint32_t seen = 0;
        for (uint64_t r = dm & (s | x); r; r &= r - 1) {
            const int l = __builtin_ctzll(r);
            const uint64_t below = l ? (~0ull >> (64 - l)) : 0ull;
            const int pos = ((s >> l) & 1ull) ? popc(s & below) : ns + popc(x & below);
            seen |= 1u << (pos >> 3);
        }
        return popc(seen);
    };
    auto mk = [&](int32_t d, int t) { return &m[((size_t)d * tiles + t) * kMaskWords]; };
    // LDS-staged sweeps: a node whose parent is in its cluster hands its set (post-order) and
    // receives its parent's final (pre-order sweeps) through LDS
    // (post-order sweeps: Fitch, and Sankoff when they cover every height with <= 255-child
    // nodes, as launch_sankoff takes them; pre-order sweeps: both modes)
    const bool planned = sub && c->cluster && ht.cl.band_wg.size() > 1 && !ht.cl.slot_of.empty();
    const bool clu = planned && (mode == PM_MODE_FITCH || (ht.cl.h0 == 0 && ht.cl.max_degree <= 255));
    auto in_cluster = [&](int32_t d) { return planned && ht.cl.slot_of[d] >= 0; };
    auto in_lds = [&](int32_t d) { return clu && in_cluster(d); };
    const bool down_lds = planned && ht.cl.down && (mode == PM_MODE_SANKOFF || !c->sub_down);
    for (int32_t d = 0; d < I; ++d) {
        if (vnode[d]) continue;
        const int32_t e0 = ht.child_off[d], e1 = ht.child_off[d + 1];
        line[0] += 64.0;   // descriptor (a node's tiles run in adjacent waves)
        for (int t = 0; t < tiles; ++t) {
            const uint64_t* q = mk(d, t);
            // level kernels: mask record (half a line), own record (simple codes by rank, then
            // the complex areas), parent finals (every non-consensus lane)
            line[0] += 64.0 + LB * (ceil8(popc(q[1])) + cx_areas * ceil8(popc(q[0])));
            if (d != root && !(down_lds && in_cluster(d))) line[1] += LB * rank_lines(q[3] | q[4], q[4], q[3]);
            const uint64_t dirty_m = d == root ? ~0ull : q[2];
            const uint64_t dleaf_m = leaf_rule && d != root ? q[0] : dirty_m;
            const double rec = 64.0 + lane * popc(q[1]) + cx_full * popc(q[0]);
            // post-order: children in, own record + masks out, parent masks pushed to children
            up += rec;
            part[2] += rec;
            const double dirty = d == root ? kWave : popc(q[2]);
            // Fitch, every leaf present: leaf children are read at complex lanes only, an
            // S2 / S3 child at the lanes its parent pushed into its record (leaf_rule)
            const double dirty_leaf = leaf_rule && d != root ? popc(q[0]) : dirty;
            // words 6 / 7 follow the pre-order descriptor, which drops S2 / S3 children
            auto s_child = [&](int32_t e) { return sub && ht.child_enc[e] >= 0 && vnode[ht.child_enc[e]] > 2; };
            for (int32_t k = e0; k < e1; ++k) {
                const int32_t ch = ht.child_enc[k];
                // k_tail item (a leaf-ish child beyond the second, or an S2 / S3 child in the
                // subtree form)
                const bool tail = (k >= e0 + 2 && (ch < 0 || vnode[ch])) || (sub && ch >= 0 && vnode[ch] > 2);
                // a k_tail item's dirty lanes (as below)
                const uint64_t tdm = d == root ? ~0ull
                                     : ch >= 0 && vnode[ch] > 2 ? mk(ch, t)[5]
                                     : ch < 0 && leaf_rule ? q[0] : q[2];
                if (ch < 0) {
                    up += word_row;
                    down += lane * dirty_leaf;
                    part[0] += word_row;
                    part[tail ? 8 : 5] += lane * dirty_leaf;
                    line[tail ? 4 : 2] += LB * groups8(tail ? tdm : dleaf_m);
                } else if (vnode[ch]) {
                    const int32_t nl = vnode[ch];
                    // (Fitch, all present: the first two children's own masks, words 6 / 7)
                    const double dv = vnode[ch] > 2 ? popc(mk(ch, t)[5])
                                      : leaf_rule && d != root && k < e0 + 2 ? popc(q[6 + (k - e0) - (k > e0 && s_child(e0))])
                                                                             : dirty;
                    up += word_row * nl;
                    down += lane * dv * nl;
                    part[0] += word_row * nl;
                    part[tail ? 8 : 5] += lane * dv * nl;
                    const uint64_t dv_m = vnode[ch] > 2 ? mk(ch, t)[5]
                                          : leaf_rule && d != root && k < e0 + 2 ? q[6 + (k - e0) - (k > e0 && s_child(e0))]
                                                                                 : dirty_m;
                    // an S2 / S3 item: its leaves side by side (64 B a lane, sub_planes); a
                    // leaf-parent: one row per leaf
                    line[tail ? 4 : 2] += vnode[ch] > 2 ? LB * pairs(dv_m) : LB * groups8(tail ? tdm : dv_m) * nl;
                } else if (!in_lds(ch)) {
                    const uint64_t* r = mk(ch, t);
                    const double b = 64.0 + lane * popc(r[1]) + cx_read_up * popc(r[0]) + lane;   // + pushed masks
                    up += b;
                    part[1] += b;
                }
                // a k_tail item: descriptor + parent masks (64 B each), the parent's final on its
                // dirty non-consensus lanes
                if (tail) {
                    const uint64_t dm = tdm;
                    const double b = 128.0 + lane * popc((q[0] | q[1]) & dm);
                    down += b;
                    part[7] += b;
                    // descriptor (adjacent tiles: once per item), masks; the parent's final at
                    // the dirty lanes (by rank in its record, or the root's row)
                    line[3] += (t == 0 ? 64.0 : 0.0) + 64.0;
                    if (dm) line[5] += LB * (d == root ? groups8(dm) : rank_lines(dm, q[1], q[0]));
                }
            }
            // pre-order: own record, parent final (non-consensus lanes), compact final out
            down += rec;
            part[3] += rec;
            if (d == root) {
                down += 2.0 * word_row;   // forced / root final
            } else {
                const double pf = down_lds && in_cluster(d) ? 0.0 : lane * popc(q[3] | q[4]);
                down += pf + lane * popc(q[0]);
                part[4] += pf;
                part[6] += lane * popc(q[0]);
            }
        }
    }
    down += 8.0 * (double)records;
    out[0] = up;
    out[1] = down;
    out[2] = 8.0 * (double)records + 4.0 * (double)c->num_sites;   // score histogram
    out[3] = 0.5 * (double)L * (double)c->num_sites + 8.0 * (double)records;   // floor: leaf codes once + records
    out[4] = (double)records;
    for (int k = 0; k < 9 && 5 + k < n; ++k) out[5 + k] = part[k];
    for (int k = 0; k < 6 && 14 + k < n; ++k) out[14 + k] = line[k];
    return PM_OK;
}

}  // extern "C"
