// pm_host.cpp -- host side of the C-ABI: context, tree flattening, uploads, results.
//
// The reference keeps the tree as Node* with children vectors and rebuilds an
// unordered_map<string,int> per column (src/panman.cpp:1409-1417).  Here the topology is
// flattened once (pm_tree_upload): dense internal indices, height levels for the
// post-order and depth levels for the pre-order, children encoded for the kernels.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "pm_internal.h"

namespace pm {

int fail(pm_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(pm_ctx* c, hipError_t e, const char* what) {
    return fail(c, PM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

namespace {

template <class T>
hipError_t dev_alloc(T** p, size_t count) {
    if (count == 0) count = 1;
    return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * count);
}

template <class T>
void dev_free(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

template <class T>
hipError_t upload(T** dst, const std::vector<T>& v, hipStream_t s) {
    hipError_t e = dev_alloc(dst, v.size());
    if (e != hipSuccess || v.empty()) return e;
    e = hipMemcpyAsync(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);   // host vectors may die after return
}

void free_tree(DevTree& t) {
    dev_free(t.child_off);
    dev_free(t.child_enc);
    dev_free(t.parent_dense);
    dev_free(t.internal_id);
    dev_free(t.leaf_id);
    dev_free(t.up_order);
    dev_free(t.down_order);
    dev_free(t.leaf_parent);
    dev_free(t.leaf_down);
    dev_free(t.child_enc_v);
    dev_free(t.up_order_v);
    dev_free(t.down_order_v);
    dev_free(t.down_desc);
    dev_free(t.up_desc);
    dev_free(t.up_desc_v);
    dev_free(t.down_desc_v);
    dev_free(t.tail_desc);
    dev_free(t.tail_desc_v);
    dev_free(t.vleaf);
    dev_free(t.part_desc);
    dev_free(t.part_desc_v);
    dev_free(t.part_desc_k);
    dev_free(t.part_desc_gs);
    dev_free(t.child_enc_k);
    dev_free(t.up_desc_k);
    dev_free(t.up_desc_g);
    dev_free(t.up_desc_gs);
    dev_free(t.down_desc_k);
    dev_free(t.down_desc_ks);
    dev_free(t.pslot_k);
    dev_free(t.pslot_g);
    dev_free(t.pslot_gs);
    dev_free(t.vinner);
    dev_free(t.tail_desc_k);
    dev_free(t.lvl);
    dev_free(t.cl_items);
    dev_free(t.cl_down_items);
    dev_free(t.cl_wg_off);
    dev_free(t.cl_slot_of);
    dev_free(t.pslot_kc);
    dev_free(t.pslot_gc);
    dev_free(t.cl_pslot);
    t = DevTree{};
}

void drop_graph(pm_ctx* c) {
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    c->graph_exec = nullptr;
    c->graph_key = 0;
}

void free_columns(pm_ctx* c) {
    drop_graph(c);
    dev_free(c->leaf_planes);
    dev_free(c->leaf_present);
    dev_free(c->leaf_flag);
    dev_free(c->cons);
    dev_free(c->forced);
    dev_free(c->score);
    dev_free(c->root_code);
    dev_free(c->root_final);
    dev_free(c->sub_planes);
    c->sub_planes_bytes = 0;
    c->sub_planes_ok = false;
    c->has_leaves = c->has_sites = c->has_forced = false;
    c->ran = false;
}

void free_work(pm_ctx* c) {
    drop_graph(c);
    dev_free(c->sets);
    dev_free(c->cmask);
    dev_free(c->upm);
    c->upm_bytes = 0;
    dev_free(c->finals);
    dev_free(c->sk_parts);
    dev_free(c->recs);
    dev_free(c->shard_cnt);
    c->sets_bytes = c->finals_bytes = c->cmask_bytes = c->sk_parts_bytes = 0;
    c->shard_cap = 0;
}

int64_t wpad_of(const pm_ctx* c) { return (int64_t)((c->words + kWave - 1) / kWave) * kWave; }

// Allocate per-shard column buffers (leaf planes, consensus, outputs) for S sites.
int alloc_columns(pm_ctx* c, int64_t sites) {
    free_columns(c);
    c->num_sites = sites;
    c->words = (int32_t)((sites + 31) / 32);
    const int64_t wpad = wpad_of(c);
    hipError_t e;
    if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->leaf_planes), sizeof(uint4) * (size_t)c->dt.num_leaves * wpad)) != hipSuccess ||
        (e = dev_alloc(&c->leaf_flag, (size_t)c->dt.num_leaves)) != hipSuccess ||
        (e = dev_alloc(&c->cons, (size_t)std::max<int64_t>(wpad, 4 * kWave))) != hipSuccess ||   // cx_base reads 4 tiles
        (e = dev_alloc(&c->forced, (size_t)wpad)) != hipSuccess ||
        (e = dev_alloc(&c->score, (size_t)sites)) != hipSuccess ||
        (e = dev_alloc(&c->root_code, (size_t)sites)) != hipSuccess ||
        (e = dev_alloc(&c->root_final, (size_t)wpad)) != hipSuccess) {
        free_columns(c);
        return fail(c, PM_ERR_OOM, std::string("column buffers: ") + hipGetErrorString(e));
    }
    (void)hipMemsetAsync(c->cons, 0, sizeof(uint4) * std::max<int64_t>(wpad, 4 * kWave), c->stream);
    return PM_OK;
}

// Work buffers sized for the current shard and mode; records get a first-guess capacity
// that pm_mutation_count grows on overflow.
int alloc_work(pm_ctx* c, int mode) {
    const int64_t wpad = wpad_of(c);
    const bool fitch = mode == PM_MODE_FITCH || mode == PM_MODE_BLOCK_FITCH;
    const size_t planes = fitch ? 4 * kFitchRecQuads : 36;   // records of kFitchRec / kSankoffRec uint4 per tile
    const size_t need_sets = (size_t)c->dt.num_internal * wpad * planes * 4;
    const size_t need_mask = (size_t)c->dt.num_internal * (wpad / kWave) * kMaskWords * sizeof(uint64_t);
    hipError_t e;
    if (need_sets > c->sets_bytes) {
        dev_free(c->sets);
        if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->sets), need_sets)) != hipSuccess)
            return fail(c, PM_ERR_OOM, std::string("state sets: ") + hipGetErrorString(e));
        c->sets_bytes = need_sets;
    }
    if (need_mask > c->cmask_bytes) {
        dev_free(c->cmask);
        if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->cmask), need_mask)) != hipSuccess)
            return fail(c, PM_ERR_OOM, std::string("set masks: ") + hipGetErrorString(e));
        c->cmask_bytes = need_mask;
    }
    // up slots: Fitch / Sankoff, subtree form (every leaf present, some S2 / S3 node)
    if ((mode == PM_MODE_FITCH || mode == PM_MODE_SANKOFF) && c->subtree_form && c->ht.num_sshape > 0) {
        const size_t items = (size_t)std::max(c->ht.cl.upm_base + c->ht.cl.n_items,
                                              std::max(c->ht.up_items_k, std::max(c->ht.up_items_g, c->ht.up_items_gs)));
        const size_t need = items * (wpad / kWave) * 4 * sizeof(uint64_t);
        if (need > c->upm_bytes) {
            dev_free(c->upm);
            c->upm_bytes = 0;
            if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->upm), need)) != hipSuccess)
                return fail(c, PM_ERR_OOM, std::string("up slots: ") + hipGetErrorString(e));
            c->upm_bytes = need;
        }
    }
    if (!fitch) {   // Sankoff nodes of out-degree > 255: part counters
        const size_t parts = (size_t)std::max(c->ht.part_off.empty() ? 0 : c->ht.part_off.back(),
                                              std::max(c->ht.part_off_v.empty() ? 0 : c->ht.part_off_v.back(),
                                                       std::max(c->ht.part_off_k.empty() ? 0 : c->ht.part_off_k.back(),
                                                                c->ht.part_off_gs.empty() ? 0 : c->ht.part_off_gs.back())));
        const size_t need = parts * kPartPlanes * wpad * sizeof(uint32_t);
        if (need > c->sk_parts_bytes) {
            dev_free(c->sk_parts);
            if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->sk_parts), need)) != hipSuccess)
                return fail(c, PM_ERR_OOM, std::string("Sankoff part counters: ") + hipGetErrorString(e));
            c->sk_parts_bytes = need;
        }
    }
    if (!c->shard_cnt && (e = dev_alloc(&c->shard_cnt, kShards)) != hipSuccess)
        return fail(c, PM_ERR_OOM, "shard counters");
    if (c->shard_cap == 0) {
        const double nodes = (double)c->dt.num_internal + c->dt.num_leaves;
        const double guess = std::max(65536.0, 0.01 * nodes * (double)c->num_sites);
        const int64_t cap = c->record_cap > 0 ? c->record_cap : (int64_t)(guess * 1.5 / kShards) + 256;
        if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->recs), sizeof(pm_mut) * (size_t)cap * kShards)) != hipSuccess)
            return fail(c, PM_ERR_OOM, std::string("mutation records: ") + hipGetErrorString(e));
        c->shard_cap = cap;
    }
    return PM_OK;
}

// Non-temporal set-record loads (pm_fitch_nt.hip / pm_sankoff_nt.hip) when the tree has a
// level of at least 64k (node, tile) waves: there the records a wave reads have left the
// caches anyway (N* Fitch 14.7 -> 14.06 ms); a tree of small levels (C3: <= ~900 nodes x 15
// tiles) reads them back from cache and keeps ordinary loads (C3 Fitch 4.42 -> 4.30 ms).
bool nt_policy(const pm_ctx* c) {
    if (c->nt_loads >= 0) return c->nt_loads != 0;
    const std::vector<int32_t>& off = c->ht.down_level_off;
    int64_t widest = 0;
    for (size_t l = 0; l + 1 < off.size(); ++l) widest = std::max<int64_t>(widest, off[l + 1] - off[l]);
    return widest * (wpad_of(c) / kWave) >= 65536;
}

hipError_t launch_all(pm_ctx* c, int mode) {
    const bool sankoff = mode == PM_MODE_SANKOFF || mode == PM_MODE_BLOCK_SANKOFF;
    const bool block = mode == PM_MODE_BLOCK_FITCH || mode == PM_MODE_BLOCK_SANKOFF;
    const bool nt = nt_policy(c);
    phase_add("run.nt_loads", nt ? 1.0 : 0.0);   // which build of the passes a launch sequence took
    hipError_t e = sankoff ? (nt ? launch_sankoff_nt(c, block) : launch_sankoff(c, block))
                           : (nt ? launch_fitch_nt(c, block) : launch_fitch(c, block));
    if (e == hipSuccess) e = launch_score(c);
    return e;
}

// Everything a captured run depends on: a different value means a different graph.
uint64_t graph_key_of(const pm_ctx* c, int mode) {
    const uint64_t parts[] = {(uint64_t)mode, (uint64_t)c->virtual_leaf_parents, (uint64_t)c->subtree_form,
                              (uint64_t)c->narrow_max, (uint64_t)c->group_waves, (uint64_t)c->group_levels, (uint64_t)c->up_group,
                              (uint64_t)c->sub_down, (uint64_t)c->plain_up, (uint64_t)c->plain_min_waves, (uint64_t)c->cluster,
                              (uint64_t)(uintptr_t)c->upm,
                              (uint64_t)(uintptr_t)c->sk_parts,
                              (uint64_t)c->leaves_all_present, (uint64_t)c->has_forced, (uint64_t)c->num_sites,
                              (uint64_t)c->shard_cap, (uint64_t)(uintptr_t)c->recs, (uint64_t)(uintptr_t)c->sets,
                              (uint64_t)(uintptr_t)c->cmask, (uint64_t)(uintptr_t)c->root_final,
                              (uint64_t)(uintptr_t)c->leaf_planes, (uint64_t)(uintptr_t)c->leaf_present,
                              (uint64_t)(uintptr_t)c->leaf_flag, (uint64_t)(uintptr_t)c->cons,
                              (uint64_t)(uintptr_t)c->forced, (uint64_t)(uintptr_t)c->score,
                              (uint64_t)(uintptr_t)c->root_code, (uint64_t)(uintptr_t)c->shard_cnt,
                              (uint64_t)(uintptr_t)c->sub_planes, (uint64_t)nt_policy(c),
                              (uint64_t)(uintptr_t)c->dt.child_off, (uint64_t)(uintptr_t)c->stream};
    uint64_t h = 1469598103934665603ull;
    for (uint64_t v : parts) h = (h ^ v) * 1099511628211ull;
    return h | 1;
}

int run_once(pm_ctx* c, int mode) {
    hipError_t e;
    if (!c->use_graph) {
        e = launch_all(c, mode);
        if (e != hipSuccess) return hip_fail(c, e, "parsimony launch");
    } else {
        const uint64_t key = graph_key_of(c, mode);
        if (key != c->graph_key) {
            drop_graph(c);
            const bool prof = c->profiling;
            c->profiling = false;   // per-kernel events are not part of the graph
            hipGraph_t g = nullptr;
            e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
            if (e == hipSuccess) {
                const hipError_t le = launch_all(c, mode);
                e = hipStreamEndCapture(c->stream, &g);
                if (e == hipSuccess) e = le;
            }
            c->profiling = prof;
            if (e == hipSuccess) e = hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0);
            if (g) (void)hipGraphDestroy(g);
            if (e != hipSuccess) {
                drop_graph(c);
                return hip_fail(c, e, "graph capture");
            }
            c->graph_key = key;
        }
        timer_begin(c, 4);
        e = hipGraphLaunch(c->graph_exec, c->stream);
        timer_end(c, 4);
        if (e != hipSuccess) return hip_fail(c, e, "graph launch");
    }
    c->ran = true;
    c->last_mode = mode;
    return PM_OK;
}

// Synchronise; if any shard overflowed, grow the record buffer to fit and run again.
int settle(pm_ctx* c, std::vector<uint32_t>& counts) {
    for (int attempt = 0; attempt < 2; ++attempt) {
        counts.assign(kShards, 0);
        hipError_t e = hipMemcpyAsync(counts.data(), c->shard_cnt, sizeof(uint32_t) * kShards,
                                      hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "result sync");
        const uint32_t worst = *std::max_element(counts.begin(), counts.end());
        if ((int64_t)worst <= c->shard_cap) return PM_OK;
        dev_free(c->recs);
        const int64_t cap = (int64_t)worst + worst / 8 + 256;
        if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->recs), sizeof(pm_mut) * (size_t)cap * kShards)) != hipSuccess)
            return fail(c, PM_ERR_OOM, std::string("mutation records: ") + hipGetErrorString(e));
        c->shard_cap = cap;
        int rc = run_once(c, c->last_mode);
        if (rc != PM_OK) return rc;
    }
    return fail(c, PM_ERR_STATE, "mutation record buffer still overflowing");
}

}  // namespace

int settle_run(pm_ctx* c) {
    std::vector<uint32_t> counts;
    return settle(c, counts);
}

hipError_t side_fork(pm_ctx* c) {
    hipError_t e = hipEventRecord(c->ev_fork, c->stream);
    return e == hipSuccess ? hipStreamWaitEvent(c->side, c->ev_fork, 0) : e;
}

hipError_t side_join(pm_ctx* c) {
    hipError_t e = hipEventRecord(c->ev_join, c->side);
    return e == hipSuccess ? hipStreamWaitEvent(c->stream, c->ev_join, 0) : e;
}

void timer_begin(pm_ctx* c, int cls) {
    if (!c->profiling) return;
    auto& v = c->timers[cls];
    if (c->timers_used[cls] == v.size()) {
        Timer t;
        (void)hipEventCreate(&t.a);
        (void)hipEventCreate(&t.b);
        v.push_back(t);
    }
    (void)hipEventRecord(v[c->timers_used[cls]].a, c->stream);
}

void timer_end(pm_ctx* c, int cls) {
    if (!c->profiling) return;
    (void)hipEventRecord(c->timers[cls][c->timers_used[cls]].b, c->stream);
    ++c->timers_used[cls];
}

}  // namespace pm

using namespace pm;

namespace pm {

int build_sub_planes(pm_ctx* c) {
    // (only the subtree form reads it, and that form needs every leaf present)
    if (c->sub_planes_ok || !c->has_tree || !c->has_leaves || !c->leaves_all_present) return PM_OK;
    hipError_t e = hipSuccess;
    if (c->ht.num_tail_s == 0) {
        c->sub_planes_ok = true;
        return PM_OK;
    }
    const size_t need = (size_t)c->ht.num_tail_s * (size_t)wpad_of(c) * 4 * sizeof(uint4);
    if (need > c->sub_planes_bytes) {
        dev_free(c->sub_planes);
        c->sub_planes_bytes = 0;
        if ((e = malloc_or_release(c, reinterpret_cast<void**>(&c->sub_planes), need)) != hipSuccess)
            return fail(c, PM_ERR_OOM, std::string("subtree leaf layout: ") + hipGetErrorString(e));
        c->sub_planes_bytes = need;
    }
    PhaseClock clock;
    if ((e = launch_sub_planes(c)) != hipSuccess) return hip_fail(c, e, "subtree leaf layout");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "subtree leaf layout");
    clock.lap("upload.sub_planes");
    c->sub_planes_ok = true;
    return PM_OK;
}

// Leaf columns already on the device (packed codes, [row][row_stride]); every leaf with a
// row is fully present.  Used by drivers that produce the columns on the GPU (reroot).
int leaves_install(pm_ctx* c, int64_t S, const uint8_t* d_codes4, int64_t row_stride, const int32_t* node_row) {
    if (!c->has_tree) return fail(c, PM_ERR_STATE, "upload the tree first");
    if (S <= 0 || S >= (int64_t)1 << 24 || row_stride < (S + 1) / 2) return fail(c, PM_ERR_ARG, "bad leaf columns");
    const int32_t L = c->dt.num_leaves;
    std::vector<int32_t> row_of_leaf(L);
    std::vector<uint8_t> flag(L);
    for (int32_t l = 0; l < L; ++l) {
        row_of_leaf[l] = node_row[c->ht.leaf_id[l]];
        flag[l] = row_of_leaf[l] < 0 ? kLeafAbsent : kLeafPresent;
    }
    int rc = alloc_columns(c, S);
    if (rc != PM_OK) return rc;
    int32_t* d_rows = nullptr;
    hipError_t e = upload(&d_rows, row_of_leaf, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(c->leaf_flag, flag.data(), L, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_pack_codes(c, d_codes4, row_stride, d_rows, nullptr, 0);
    c->leaves_all_present = std::all_of(flag.begin(), flag.end(), [](uint8_t f) { return f == kLeafPresent; });
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(d_rows);
    if (e != hipSuccess) return hip_fail(c, e, "leaf install");
    c->has_leaves = true;
    c->sub_planes_ok = false;
    return build_sub_planes(c);
}

}  // namespace pm

extern "C" {

int pm_create(int device, pm_ctx** out) {
    if (!out) return PM_ERR_ARG;
    *out = nullptr;
    PhaseClock clock;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return PM_ERR_HIP;
    if (device < 0 || device >= n) return PM_ERR_ARG;
    if ((e = hipSetDevice(device)) != hipSuccess) return PM_ERR_HIP;
    pm_ctx* c = new pm_ctx();
    c->device = device;
    if ((e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming)) != hipSuccess) {
        if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
        if (c->side) (void)hipStreamDestroy(c->side);
        if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
        delete c;
        return PM_ERR_HIP;
    }
    c->stream = c->own_stream;
    *out = c;
    clock.lap("hip.create_context");
    return PM_OK;
}

int pm_warmup(int device) {
    PhaseClock clock;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return PM_ERR_HIP;
    if (device < 0 || device >= n) return PM_ERR_ARG;
    if ((e = hipSetDevice(device)) != hipSuccess) return PM_ERR_HIP;
    for (auto warm : {warm_fitch, warm_sankoff, warm_fitch_nt, warm_sankoff_nt, warm_replay, warm_synth, warm_sort})
        if ((e = warm()) != hipSuccess) return PM_ERR_HIP;
    // the runtime's first allocation and staged copies
    void* d = nullptr;
    uint8_t h[4096] = {0};
    if ((e = hipMalloc(&d, sizeof h)) != hipSuccess) return PM_ERR_HIP;
    e = hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    clock.lap("hip.warmup");
    return e == hipSuccess ? PM_OK : PM_ERR_HIP;
}

void pm_destroy(pm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_work(c);
    free_columns(c);
    free_tree(c->dt);
    free_replay(c);
    comm_release(c);
    free_hostio(c);
    for (auto& v : c->timers)
        for (auto& t : v) {
            (void)hipEventDestroy(t.a);
            (void)hipEventDestroy(t.b);
        }
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* pm_last_error(const pm_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pm_set_stream(pm_ctx* c, void* s) {
    if (!c) return PM_ERR_ARG;
    c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
    return PM_OK;
}

int pm_set_option(pm_ctx* c, int option, int64_t value) {
    if (!c) return PM_ERR_ARG;
    if (option == PM_OPT_SUBTREE) {
        c->subtree_form = value != 0;
        return PM_OK;
    }
    if (option == PM_OPT_VIRTUAL) {
        c->virtual_leaf_parents = value != 0;
        return PM_OK;
    }
    if (option == PM_OPT_NARROW) {
        if (value < 0 || value > 1024) return fail(c, PM_ERR_ARG, "PM_OPT_NARROW: 0..1024 items per level");
        c->narrow_max = (int32_t)value;
        return PM_OK;
    }
    if (option == PM_OPT_UP_GROUP) {
        c->up_group = value != 0;
        return PM_OK;
    }
    if (option == PM_OPT_PLAIN_UP) {   // 0 off, 1 on (default threshold), >= 2: on from that many waves
        if (value < 0) return fail(c, PM_ERR_ARG, "PM_OPT_PLAIN_UP: 0, 1 or a wave threshold >= 2");
        c->plain_up = value != 0;
        c->plain_min_waves = value >= 2 ? value : 0;
        return PM_OK;
    }
    if (option == PM_OPT_SUB_DOWN) {
        c->sub_down = value != 0;
        return PM_OK;
    }
    if (option == PM_OPT_GROUP_WAVES) {
        if (value < 0) return fail(c, PM_ERR_ARG, "PM_OPT_GROUP_WAVES: >= 0 waves");
        c->group_waves = value;
        return PM_OK;
    }
    if (option == PM_OPT_GROUP_LEVELS) {
        if (value < 2 || value > 4) return fail(c, PM_ERR_ARG, "PM_OPT_GROUP_LEVELS: 2 to 4");
        c->group_levels = (int32_t)value;
        return PM_OK;
    }
    if (option == PM_OPT_RECORD_CAP) {
        if (value < 1 || value > ((int64_t)1 << 31)) return fail(c, PM_ERR_ARG, "PM_OPT_RECORD_CAP: 1 .. 2^31 records per shard");
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        drop_graph(c);
        dev_free(c->recs);
        c->shard_cap = 0;   // the next run allocates record_cap per shard
        c->record_cap = value;
        c->ran = false;
        return PM_OK;
    }
    if (option == PM_OPT_NT_LOADS) {
        if (value < -1 || value > 1) return fail(c, PM_ERR_ARG, "PM_OPT_NT_LOADS: -1 (by level size), 0 or 1");
        c->nt_loads = (int32_t)value;
        return PM_OK;
    }
    // 0 off (and no plan at the next tree upload: the grouped post-order covers every level);
    // 1 on (the default plan); >= 2 on, that level threshold and no bushiness test (next tree upload)
    if (option == PM_OPT_CLUSTER) {
        if (value < 0 || value > ((int64_t)1 << 30)) return fail(c, PM_ERR_ARG, "PM_OPT_CLUSTER: 0, 1 or a level size >= 2");
        c->cluster = value != 0;
        c->cluster_max_level = value == 0 ? 0 : value == 1 ? kClMaxLevel : (int32_t)value;
        c->cluster_chain = value == 1;
        return PM_OK;
    }
    if (option == PM_OPT_GRAPH) {
        c->use_graph = value != 0;
        if (!c->use_graph) drop_graph(c);
        return PM_OK;
    }
    return fail(c, PM_ERR_ARG, "unknown option");
}

int pm_set_profiling(pm_ctx* c, int enable) {
    if (!c) return PM_ERR_ARG;
    c->profiling = enable != 0;
    for (auto& u : c->timers_used) u = 0;
    return PM_OK;
}

int pm_tree_upload(pm_ctx* c, const pm_tree* t) {
    // PM_UPLOAD_TIMING=1: host phase durations on stderr
    const bool timing = std::getenv("PM_UPLOAD_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto upload_phase = [&](const char* what) {
        const auto now = std::chrono::steady_clock::now();
        phase_add(std::string("tree.") + what, std::chrono::duration<double>(now - t_last).count());
        if (!timing) {
            t_last = now;
            return;
        }
        std::fprintf(stderr, "[pm_tree_upload] %-16s %8.2f s\n", what, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
    if (!c || !t || !t->child_offsets || t->num_nodes < 2) return fail(c, PM_ERR_ARG, "bad tree");
    (void)hipSetDevice(c->device);
    c->sub_planes_ok = false;   // its S2 / S3 nodes are this tree's
    const int32_t N = t->num_nodes;
    const int32_t* off = t->child_offsets;
    const int32_t* idx = t->child_index;
    if (off[0] != 0 || t->root < 0 || t->root >= N) return fail(c, PM_ERR_ARG, "bad tree header");
    for (int32_t i = 0; i < N; ++i)
        if (off[i + 1] < off[i]) return fail(c, PM_ERR_ARG, "child offsets not monotone");
    const int32_t E = off[N];
    if (E != N - 1) return fail(c, PM_ERR_ARG, "a tree on N nodes has N-1 edges");
    std::vector<int32_t> parent(N, -2);
    parent[t->root] = -1;
    for (int32_t i = 0; i < N; ++i)
        for (int32_t e = off[i]; e < off[i + 1]; ++e) {
            const int32_t ch = idx[e];
            if (ch < 0 || ch >= N || parent[ch] != -2) return fail(c, PM_ERR_ARG, "child index invalid or repeated");
            parent[ch] = i;
        }
    if (off[t->root + 1] == off[t->root]) return fail(c, PM_ERR_ARG, "root must be internal");
    // a child's encoding keeps the dense internal index in its low kShapeShift bits (the
    // subtree shape above them): more internal nodes would mix shape bits into indices
    int64_t internal = 0;
    for (int32_t i = 0; i < N; ++i) internal += off[i + 1] > off[i];
    if (internal > kDenseMask) return fail(c, PM_ERR_ARG, "too many internal nodes (limit 2^28 - 1)");
    // BFS from the root: depth + connectivity.
    std::vector<int32_t> bfs;
    bfs.reserve(N);
    std::vector<int32_t> depth(N, -1);
    bfs.push_back(t->root);
    depth[t->root] = 0;
    for (size_t h = 0; h < bfs.size(); ++h) {
        const int32_t u = bfs[h];
        for (int32_t e = off[u]; e < off[u + 1]; ++e) {
            depth[idx[e]] = depth[u] + 1;
            bfs.push_back(idx[e]);
        }
    }
    if ((int32_t)bfs.size() != N) return fail(c, PM_ERR_ARG, "tree is not connected");
    std::vector<int32_t> height(N, 0);
    for (int32_t k = N - 1; k >= 0; --k) {
        const int32_t u = bfs[k];
        int32_t h = 0;
        for (int32_t e = off[u]; e < off[u + 1]; ++e) h = std::max(h, height[idx[e]] + 1);
        height[u] = off[u + 1] > off[u] ? h : 0;
    }

    HostTree ht;
    ht.num_nodes = N;
    ht.root = t->root;
    ht.dense_of.assign(N, 0);
    // Dense internal indices and leaf ranks in DFS pre-order: a subtree's leaf rows and
    // records are contiguous, and the nodes of one level (bucketed in dense order below)
    // run in tree order, so neighbouring waves read neighbouring rows.
    std::vector<int32_t> dfs;
    dfs.reserve(N);
    {
        std::vector<int32_t> stack{t->root};
        while (!stack.empty()) {
            const int32_t u = stack.back();
            stack.pop_back();
            dfs.push_back(u);
            for (int32_t e = off[u + 1] - 1; e >= off[u]; --e) stack.push_back(idx[e]);
        }
    }
    // Internal nodes: the materialised ones (every internal node but the virtual
    // leaf-parents, see below) by depth, then the virtual ones; DFS order within a depth.
    // A pre-order level of the virtual-leaf-parent form is then a contiguous range of
    // dense indices, so its waves know their node -- and its record masks -- without
    // reading the level descriptor first (DevTree::down_dense).
    auto virtual_id = [&](int32_t u) {
        if (u == t->root || off[u + 1] == off[u] || off[u + 1] - off[u] > 2) return false;
        for (int32_t e = off[u]; e < off[u + 1]; ++e)
            if (off[idx[e] + 1] > off[idx[e]]) return false;
        return true;
    };
    // Subtree form (Fitch, every leaf present): a node whose two children are leaves or
    // two-leaf cherries, at least one a cherry, under a parent of out-degree <= 2, is also
    // evaluated inline by its parent (shapes S2 = (cherry, leaf), S3 = (cherry, cherry)).
    auto cherry2 = [&](int32_t u) {
        return u != t->root && off[u + 1] - off[u] == 2 && off[idx[off[u]] + 1] == off[idx[off[u]]] &&
               off[idx[off[u] + 1] + 1] == off[idx[off[u] + 1]];
    };
    auto sshape_id = [&](int32_t u) {
        if (u == t->root || off[u + 1] - off[u] != 2 || parent[u] < 0 || off[parent[u] + 1] - off[parent[u]] > 2)
            return 0;
        int cherries = 0;
        for (int32_t e = off[u]; e < off[u + 1]; ++e) {
            const int32_t ch = idx[e];
            if (off[ch + 1] == off[ch]) continue;
            if (!cherry2(ch)) return 0;
            ++cherries;
        }
        return cherries;   // 1: S2, 2: S3
    };
    {
        std::vector<int32_t> inner;
        for (const int32_t i : dfs) {
            if (off[i + 1] > off[i]) {
                inner.push_back(i);
            } else {
                ht.dense_of[i] = -(int32_t)ht.leaf_id.size() - 1;
                ht.leaf_id.push_back(i);
            }
        }
        // stable counting sort by key: DFS order kept within a key
        int32_t maxd = 0;
        for (const int32_t i : inner) maxd = std::max(maxd, depth[i]);
        // key: the materialised nodes by (depth, has an S2 / S3 child) -- a subtree-form
        // pre-order level, and each half of it, is one contiguous range of dense indices --
        // then the S2 / S3 nodes by depth -- the order of the subtree form's tail items, so a
        // tail wave knows its S2 / S3 node, and the masks its parent pushed there, from its
        // item index alone -- then the virtual leaf-parents.  (The leaf-parent form's levels,
        // which include the S2 / S3 nodes, are then two ranges: its pre-order kernels read
        // the node from the descriptor.)
        auto has_sub_child = [&](int32_t u) {
            for (int32_t e = off[u]; e < off[u + 1]; ++e)
                if (sshape_id(idx[e])) return true;
            return false;
        };
        const int32_t D1 = maxd + 1, nk = 4 * D1;
        std::vector<int32_t> key(inner.size()), start(nk + 1, 0);
        for (size_t k = 0; k < inner.size(); ++k) {
            const int32_t u = inner[k];
            key[k] = virtual_id(u) ? 3 * D1 + depth[u] : sshape_id(u) ? 2 * D1 + depth[u]
                                                       : 2 * depth[u] + (has_sub_child(u) ? 1 : 0);
            ++start[key[k] + 1];
        }
        for (int32_t k = 0; k < nk; ++k) start[k + 1] += start[k];
        ht.internal_id.assign(inner.size(), 0);
        for (size_t k = 0; k < inner.size(); ++k) ht.internal_id[start[key[k]]++] = inner[k];
        for (size_t k = 0; k < ht.internal_id.size(); ++k) ht.dense_of[ht.internal_id[k]] = (int32_t)k;
    }
    const int32_t I = (int32_t)ht.internal_id.size();
    const int32_t L = (int32_t)ht.leaf_id.size();
    // child encodings keep the dense index in the low kShapeShift bits (shape and virtual
    // flags above it)
    if (I >= (1 << kShapeShift)) return fail(c, PM_ERR_ARG, "trees of 2^28 or more internal nodes are not supported");
    ht.child_off.assign(I + 1, 0);
    ht.child_enc.reserve(E);
    std::vector<int32_t> parent_dense(I, -1), leaf_parent(L, -1);
    for (int32_t d = 0; d < I; ++d) {
        const int32_t u = ht.internal_id[d];
        for (int32_t e = off[u]; e < off[u + 1]; ++e) {
            const int32_t ch = idx[e];
            ht.child_enc.push_back(ht.dense_of[ch]);
            if (ht.dense_of[ch] >= 0) parent_dense[ht.dense_of[ch]] = d;
            else leaf_parent[-ht.dense_of[ch] - 1] = d;
        }
        ht.child_off[d + 1] = (int32_t)ht.child_enc.size();
    }
    // post-order levels: internal nodes by height 1..H
    int32_t H = 0, D = 0;
    for (int32_t d = 0; d < I; ++d) {
        H = std::max(H, height[ht.internal_id[d]]);
        D = std::max(D, depth[ht.internal_id[d]]);
    }
    int32_t DL = 0;
    for (int32_t l = 0; l < L; ++l) DL = std::max(DL, depth[ht.leaf_id[l]]);
    auto bucket = [](int32_t levels, int32_t count, auto key, std::vector<int32_t>& offs, std::vector<int32_t>& order) {
        offs.assign(levels + 1, 0);
        for (int32_t i = 0; i < count; ++i) ++offs[key(i) + 1];
        for (int32_t k = 0; k < levels; ++k) offs[k + 1] += offs[k];
        order.assign(count, 0);
        std::vector<int32_t> cur(offs.begin(), offs.end() - 1);
        for (int32_t i = 0; i < count; ++i) order[cur[key(i)]++] = i;
    };
    std::vector<int32_t> up_order, down_order, leaf_down;
    bucket(H * kDegreeClasses, I,
           [&](int32_t d) {
               return (height[ht.internal_id[d]] - 1) * kDegreeClasses +
                      degree_class(ht.child_off[d + 1] - ht.child_off[d]);
           },
           ht.up_class_off, up_order);
    ht.up_level_off.assign(H + 1, 0);
    for (int32_t h = 0; h <= H; ++h) ht.up_level_off[h] = ht.up_class_off[h * kDegreeClasses];
    bucket(D + 1, I, [&](int32_t d) { return depth[ht.internal_id[d]]; }, ht.down_level_off, down_order);
    bucket(DL + 1, L, [&](int32_t l) { return depth[ht.leaf_id[l]]; }, ht.leaf_level_off, leaf_down);

    upload_phase("topology+levels");
    // heavy child first: the internal child with the largest subtree (a materialised one
    // on ties) leads its parent's child list, so it is the next node down the parent's
    // chain in both the plain and the virtual-leaf-parent form (children order is free:
    // every pass combines children commutatively and records are sorted on fetch)
    auto is_virtual = [&](int32_t d) {
        if (ht.internal_id[d] == t->root) return false;
        const int32_t deg = ht.child_off[d + 1] - ht.child_off[d];
        if (deg > 2) return false;
        for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
            if (ht.child_enc[e] >= 0) return false;
        return true;
    };
    {
        std::vector<int64_t> sub(N, 1);
        for (int32_t k = N - 1; k >= 0; --k) {
            const int32_t u = bfs[k];
            for (int32_t e = off[u]; e < off[u + 1]; ++e) sub[u] += sub[idx[e]];
        }
        for (int32_t d = 0; d < I; ++d) {
            int32_t best = -1;
            int64_t best_key = -1;
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e) {
                const int32_t x = ht.child_enc[e];
                if (x < 0) continue;
                const int64_t key = sub[ht.internal_id[x]] * 2 + (is_virtual(x) ? 0 : 1);
                if (key > best_key) { best_key = key; best = e; }
            }
            if (best > ht.child_off[d]) std::swap(ht.child_enc[best], ht.child_enc[ht.child_off[d]]);
        }
    }

    upload_phase("heavy child");
    // virtual leaf-parents (Fitch level kernels)
    std::vector<int32_t> child_enc_v(ht.child_enc), up_order_v, down_order_v, vleaf((size_t)I * 4, -1);
    std::vector<uint8_t> virt(I, 0);
    {
        for (int32_t d = 0; d < I; ++d) {
            if (ht.internal_id[d] == t->root) continue;
            const int32_t deg = ht.child_off[d + 1] - ht.child_off[d];
            bool all_leaves = deg <= 2;   // one or two leaves: Fitch and Sankoff evaluate them inline
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1] && all_leaves; ++e) all_leaves = ht.child_enc[e] < 0;
            virt[d] = all_leaves;
            ht.num_virtual += all_leaves;
        }
        for (auto& x : child_enc_v)
            if (x >= 0 && virt[x]) x |= kVirtualBit;
        for (int32_t d = 0; d < I; ++d)
            if (virt[d])
                for (int32_t e = ht.child_off[d], k = 0; e < ht.child_off[d + 1]; ++e, ++k)
                    vleaf[(size_t)d * 4 + k] = -ht.child_enc[e] - 1;
        // levels keep their (height, degree class) buckets; virtual nodes are dropped
        auto drop = [&](std::vector<int32_t>& order, std::vector<int32_t>& offs) {
            std::vector<int32_t> o2, f2{0};
            for (size_t k = 0; k + 1 < offs.size(); ++k) {
                for (int32_t i = offs[k]; i < offs[k + 1]; ++i)
                    if (!virt[order[i]]) o2.push_back(order[i]);
                f2.push_back((int32_t)o2.size());
            }
            order.swap(o2);
            offs.swap(f2);
        };
        bucket(H * kDegreeClasses, I,
               [&](int32_t d) {
                   return (height[ht.internal_id[d]] - 1) * kDegreeClasses +
                          degree_class(ht.child_off[d + 1] - ht.child_off[d]);
               },
               ht.up_class_off_v, up_order_v);
        drop(up_order_v, ht.up_class_off_v);
        ht.up_level_off_v.assign(H + 1, 0);
        for (int32_t h = 0; h <= H; ++h) ht.up_level_off_v[h] = ht.up_class_off_v[h * kDegreeClasses];
        // levels whose nodes of out-degree <= 3 have only leaf / virtual children
        ht.up_leafy_v.assign(H, 0);
        for (int32_t h = 0; h < H; ++h) {
            bool leafy = true;
            for (int32_t i = ht.up_class_off_v[h * kDegreeClasses]; i < ht.up_class_off_v[h * kDegreeClasses + 1] && leafy; ++i)
                for (int32_t e = ht.child_off[up_order_v[i]]; e < ht.child_off[up_order_v[i] + 1]; ++e)
                    leafy &= child_enc_v[e] < 0 || (child_enc_v[e] & kVirtualBit) != 0;
            ht.up_leafy_v[h] = leafy;
        }
        bucket(D + 1, I, [&](int32_t d) { return depth[ht.internal_id[d]]; }, ht.down_level_off_v, down_order_v);
        drop(down_order_v, ht.down_level_off_v);
        ht.down_dense_v = true;   // pre-order item k of the virtual form is dense index k
        for (size_t k = 0; k < down_order_v.size(); ++k) ht.down_dense_v &= down_order_v[k] == (int32_t)k;
    }

    upload_phase("virtual form");
    // subtree form (Fitch, all leaves present): S2 / S3 nodes dropped from the levels as well;
    // child encodings carry the shape (kShapeShift), vleaf their leaves (a, b[, c[, d]]) and
    // vinner their cherries (x[, y])
    std::vector<int32_t> child_enc_k(child_enc_v), up_order_k, down_order_k, vinner((size_t)I * 2, -1);
    std::vector<uint8_t> sshape(I, 0);
    {
        for (int32_t d = 0; d < I; ++d) {
            const int sh = sshape_id(ht.internal_id[d]);
            if (!sh) continue;
            sshape[d] = (uint8_t)sh;
            // leaves: the cherries' leaves first, then the lone leaf (S2)
            int32_t nl = 0, ni = 0;
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e) {
                const int32_t x = ht.child_enc[e];
                if (x < 0) continue;
                vinner[(size_t)d * 2 + ni++] = x;
                for (int32_t f = ht.child_off[x]; f < ht.child_off[x + 1]; ++f) vleaf[(size_t)d * 4 + nl++] = -ht.child_enc[f] - 1;
            }
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
                if (ht.child_enc[e] < 0) vleaf[(size_t)d * 4 + nl++] = -ht.child_enc[e] - 1;
            ht.num_sshape += 1;
        }
        for (auto& x : child_enc_k)
            if (x >= 0 && !(x & kVirtualBit) && sshape[x]) x = (x | kVirtualBit) | (sshape[x] << kShapeShift);
        auto keep = [&](std::vector<int32_t>& order, std::vector<int32_t>& offs, const std::vector<int32_t>& src_order,
                        const std::vector<int32_t>& src_offs) {
            order.clear();
            offs.assign(1, 0);
            for (size_t k = 0; k + 1 < src_offs.size(); ++k) {
                for (int32_t i = src_offs[k]; i < src_offs[k + 1]; ++i)
                    if (!sshape[src_order[i]]) order.push_back(src_order[i]);
                offs.push_back((int32_t)order.size());
            }
        };
        keep(up_order_k, ht.up_class_off_k, up_order_v, ht.up_class_off_v);
        ht.up_level_off_k.assign(H + 1, 0);
        for (int32_t h = 0; h <= H; ++h) ht.up_level_off_k[h] = ht.up_class_off_k[h * kDegreeClasses];
        ht.up_leafy_k.assign(H, 0);
        for (int32_t h = 0; h < H; ++h) {
            bool leafy = true;
            for (int32_t i = ht.up_class_off_k[h * kDegreeClasses]; i < ht.up_class_off_k[h * kDegreeClasses + 1] && leafy; ++i)
                for (int32_t e = ht.child_off[up_order_k[i]]; e < ht.child_off[up_order_k[i] + 1]; ++e)
                    leafy &= child_enc_k[e] < 0 || (child_enc_k[e] & kVirtualBit) != 0;
            ht.up_leafy_k[h] = leafy;
        }
        keep(down_order_k, ht.down_level_off_k, down_order_v, ht.down_level_off_v);
        // each subtree-form pre-order level is one dense range (dense key: depth, then S2/S3 last)
        ht.down_dense_base_k.assign(ht.down_level_off_k.size() - 1, -1);
        bool dense = true;
        for (size_t l = 0; l + 1 < ht.down_level_off_k.size(); ++l) {
            const int32_t a = ht.down_level_off_k[l], b = ht.down_level_off_k[l + 1];
            if (a == b) continue;
            for (int32_t i = a; i < b; ++i) dense &= down_order_k[i] == down_order_k[a] + (i - a);
            ht.down_dense_base_k[l] = down_order_k[a];
        }
        ht.down_dense_k = dense;
    }
    ht.sshape = sshape;
    upload_phase("subtree form");
    // LDS-staged post-order sweeps of the subtree form (PM_OPT_CLUSTER, pm_cluster.cpp)
    plan_clusters(ht, up_order_k, child_enc_k, parent_dense, vleaf, c->cluster_max_level, c->cluster_chain, ht.cl);
    upload_phase("clusters");
    // (counts: the sweeps' first level, bands, workgroups per tile, longest workgroup in rounds)
    phase_add("cluster.first_level", (double)ht.cl.h0);
    phase_add("cluster.bands", ht.cl.band_wg.empty() ? 0.0 : (double)(ht.cl.band_wg.size() - 1));
    phase_add("cluster.workgroups", ht.cl.wg_off.empty() ? 0.0 : (double)(ht.cl.wg_off.size() - 1));
    phase_add("cluster.max_rounds", (double)ht.cl.max_rounds);
    auto make_desc = [&](const std::vector<int32_t>& order, const std::vector<int32_t>& enc) {
        std::vector<NodeDesc> desc(order.size());
        for (size_t k = 0; k < order.size(); ++k) {
            const int32_t d = order[k];
            NodeDesc& x = desc[k];
            x = NodeDesc{};
            x.node = d;
            x.parent = parent_dense[d];
            x.e0 = ht.child_off[d];
            x.e1 = ht.child_off[d + 1];
            x.c0 = enc[x.e0];
            x.c1 = x.e1 - x.e0 > 1 ? enc[x.e0 + 1] : 0;
            for (int j = 0; j < 4; ++j) {
                x.vl0[j] = x.c0 >= 0 && (x.c0 & kVirtualBit) ? vleaf[(size_t)(x.c0 & kDenseMask) * 4 + j] : -1;
                x.vl1[j] = x.e1 - x.e0 > 1 && x.c1 >= 0 && (x.c1 & kVirtualBit)
                               ? vleaf[(size_t)(x.c1 & kDenseMask) * 4 + j] : -1;
            }
        }
        return desc;
    };
    // pre-order descriptors carry the grandparent and great-grandparent (k_down level groups
    // recompute the ancestors' finals)
    auto with_gp = [&](std::vector<NodeDesc> desc) {
        for (NodeDesc& x : desc) {
            x.pad0 = x.parent >= 0 ? parent_dense[x.parent] : -1;
            x.pad1 = x.pad0 >= 0 ? parent_dense[x.pad0] : -1;
        }
        return desc;
    };
    const std::vector<NodeDesc> down_desc = with_gp(make_desc(down_order, ht.child_enc));
    const std::vector<NodeDesc> down_desc_v = with_gp(make_desc(down_order_v, child_enc_v));
    const std::vector<NodeDesc> up_desc = make_desc(up_order, ht.child_enc);
    const std::vector<NodeDesc> up_desc_v = make_desc(up_order_v, child_enc_v);
    const std::vector<NodeDesc> up_desc_k = make_desc(up_order_k, child_enc_k);
    // Grouped post-order launches of the subtree form (PM_OPT_UP_GROUP): a node of
    // out-degree <= 3 joins the launch of its latest materialised children when each of
    // those is of out-degree <= max_rc (Fitch 3; Sankoff 2: a recomputed child's Z0 is the
    // AND-else-OR of its children only when it is binary), computed from earlier launches
    // only, and among its first two children -- its wave recomputes them in registers
    // (k_fitch_up / k_sankoff_up <.., GROUP>, the descriptor's pad0 / pad1 = their descriptor
    // indices) -- otherwise the launch after.  Children come before parents in up_order_k
    // (height order).  Only nodes of heights with at most kUpGroupNodes nodes join a child's
    // launch: big levels fill the chip by themselves and pay for the recomputation (measured
    // at N*).
    // `levels`: only the subtree form's first `levels` post-order levels (Fitch with the LDS-staged
    // sweeps: the levels below them; the sweeps take the rest).
    const std::vector<int32_t>& up_order_k_all = up_order_k;
    auto make_groups = [&](int32_t max_rc, std::vector<int32_t>& level_off, std::vector<int32_t>& class_off,
                           std::vector<uint8_t>& leafy_out, std::vector<uint8_t>& recomp_out,
                           std::vector<int32_t>& plain_out, int32_t levels) {
        levels = std::min<int32_t>(levels, (int32_t)ht.up_level_off_k.size() - 1);
        const std::vector<int32_t> up_order_k(up_order_k_all.begin(), up_order_k_all.begin() + ht.up_level_off_k[levels]);
        auto is_mat = [](int32_t x) { return x >= 0 && !(x & kVirtualBit); };
        auto narrow = [&](int32_t d) { return degree_class(ht.child_off[d + 1] - ht.child_off[d]) == 0; };
        auto recomputable = [&](int32_t d) { return ht.child_off[d + 1] - ht.child_off[d] <= max_rc; };
        std::vector<int32_t> lv(I, -1), inl((size_t)I * 2, -1), hsize(I, 0);
        for (int32_t h = 0; h < levels; ++h)
            for (int32_t i = ht.up_level_off_k[h]; i < ht.up_level_off_k[h + 1]; ++i)
                hsize[up_order_k[i]] = ht.up_level_off_k[h + 1] - ht.up_level_off_k[h];
        std::vector<uint8_t> gen(I, 0);
        int32_t G = 0;
        for (int32_t d : up_order_k) {
            int32_t M = -1;
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
                if (is_mat(child_enc_k[e])) M = std::max(M, lv[child_enc_k[e]]);
            if (M < 0) {
                lv[d] = 0;
            } else {
                bool ok = narrow(d) && hsize[d] <= kUpGroupNodes;
                int top = 0, g = 0;   // children in launch M, the deepest recomputation below them
                for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1] && ok; ++e) {
                    const int32_t x = child_enc_k[e];
                    if (is_mat(x) && lv[x] == M) {
                        ok = recomputable(x) && e - ht.child_off[d] < 2 && gen[x] < kUpGroupDepth;
                        ++top;
                        g = std::max(g, (int)gen[x]);
                    }
                }
                ok = ok && (g == 0 || top == 1);   // a chain below: one recomputed child only
                lv[d] = ok ? M : M + 1;
                gen[d] = ok ? (uint8_t)(g + 1) : 0;
                if (ok)
                    for (int32_t e = ht.child_off[d]; e < ht.child_off[d] + 2 && e < ht.child_off[d + 1]; ++e)
                        if (is_mat(child_enc_k[e]) && lv[child_enc_k[e]] == M) inl[(size_t)d * 2 + (e - ht.child_off[d])] = child_enc_k[e];
            }
            G = std::max(G, lv[d] + 1);
        }
        // bucket by (launch, degree class), children-first order kept inside a bucket; in the
        // out-degree <= 3 class the plain nodes first (binary, neither of the children an S2 / S3
        // subtree nor recomputed here): one launch of the lean kernel covers them
        class_off.assign((size_t)G * kDegreeClasses + 1, 0);
        auto key = [&](int32_t d) { return lv[d] * kDegreeClasses + degree_class(ht.child_off[d + 1] - ht.child_off[d]); };
        auto sub_shaped_enc = [](int32_t x) { return x >= 0 && (x & kVirtualBit) && ((x >> kShapeShift) & 3); };
        auto plain = [&](int32_t d) {
            if (ht.child_off[d + 1] - ht.child_off[d] > 2 || inl[(size_t)d * 2] >= 0 || inl[(size_t)d * 2 + 1] >= 0) return false;
            for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
                if (sub_shaped_enc(child_enc_k[e])) return false;
            return true;
        };
        for (int32_t d : up_order_k) ++class_off[key(d) + 1];
        for (size_t k = 0; k + 1 < class_off.size(); ++k) class_off[k + 1] += class_off[k];
        std::vector<int32_t> order(up_order_k.size()), cur(class_off.begin(), class_off.end() - 1), pos(I, -1);
        plain_out.assign(G, 0);
        for (int pass = 0; pass < 2; ++pass)
            for (int32_t d : up_order_k) {
                if (plain(d) != (pass == 0)) continue;
                pos[d] = cur[key(d)]++;
                order[pos[d]] = d;
                if (pass == 0) ++plain_out[lv[d]];
            }
        level_off.assign(G + 1, 0);
        for (int32_t l = 0; l <= G; ++l) level_off[l] = class_off[(size_t)l * kDegreeClasses];
        leafy_out.assign(G, 0);
        for (int32_t l = 0; l < G; ++l) {
            bool leafy = true;
            for (int32_t i = class_off[(size_t)l * kDegreeClasses]; i < class_off[(size_t)l * kDegreeClasses + 1] && leafy; ++i)
                for (int32_t e = ht.child_off[order[i]]; e < ht.child_off[order[i] + 1]; ++e)
                    leafy &= !is_mat(child_enc_k[e]);
            leafy_out[l] = leafy;
        }
        std::vector<NodeDesc> desc = make_desc(order, child_enc_k);
        recomp_out.assign(G, 0);   // launches where some node recomputes a child (the others run the plain kernel)
        for (size_t k = 0; k < order.size(); ++k) {
            const int32_t d = order[k];
            desc[k].pad0 = inl[(size_t)d * 2] >= 0 ? pos[inl[(size_t)d * 2]] : -1;
            desc[k].pad1 = inl[(size_t)d * 2 + 1] >= 0 ? pos[inl[(size_t)d * 2 + 1]] : -1;
            if (desc[k].pad0 >= 0 || desc[k].pad1 >= 0) recomp_out[lv[d]] = 1;
        }
        return std::make_pair(desc, order);
    };
    // (with a sweep plan the grouped Fitch launches stop below its first level: ht.cl.h0)
    const int32_t all_levels = (int32_t)ht.up_level_off_k.size() - 1;
    const auto groups_g = make_groups(3, ht.up_level_off_g, ht.up_class_off_g, ht.up_leafy_g, ht.up_recomp_g, ht.up_plain_g,
                                      ht.cl.band_wg.size() > 1 ? ht.cl.h0 : all_levels);
    const std::vector<NodeDesc>& up_desc_g = groups_g.first;
    // up slots: each descriptor's parent item and child slot (the parent's first / second
    // child) in the same array, for the subtree form's two up orders
    auto make_pslot = [&](const std::vector<int32_t>& order, const std::vector<NodeDesc>& desc) {
        std::vector<int32_t> pos(I, -1), ps(order.size(), -1);
        for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int32_t)k;
        for (size_t k = 0; k < desc.size(); ++k)
            for (int j = 0; j < 2 && j < desc[k].e1 - desc[k].e0; ++j) {
                const int32_t x = j == 0 ? desc[k].c0 : desc[k].c1;
                if (x >= 0 && !(x & kVirtualBit) && pos[x] >= 0) ps[pos[x]] = (int32_t)k * 2 + j;
            }
        return ps;
    };
    const std::vector<int32_t> pslot_k = make_pslot(up_order_k, up_desc_k), pslot_g = make_pslot(groups_g.second, up_desc_g);
    // with the sweeps: a level item (either up order) whose parent is swept pushes into the
    // parent's sweep item's up slot (item cl.upm_base + item); a swept node whose parent is in a
    // later band likewise (a parent in its own cluster reads its LDS slot instead)
    std::vector<int32_t> pslot_kc(pslot_k), pslot_gc(pslot_g), cl_pslot(ht.cl.items.size(), -1);
    ht.cl.upm_base = (int32_t)std::max(up_desc_k.size(), up_desc_g.size());
    {
        std::vector<int32_t> pos_k(I, -1), pos_g(I, -1);
        for (size_t k = 0; k < up_desc_k.size(); ++k) pos_k[up_order_k[k]] = (int32_t)k;
        for (size_t k = 0; k < groups_g.second.size(); ++k) pos_g[groups_g.second[k]] = (int32_t)k;
        for (int32_t p = 0; p < I && !ht.cl.item_of.empty(); ++p) {
            if (ht.cl.item_of[p] < 0) continue;   // swept parents: their first two materialised children
            const int32_t e0 = ht.child_off[p], e1 = ht.child_off[p + 1];
            for (int j = 0; j < 2 && e0 + j < e1; ++j) {
                const int32_t x = child_enc_k[e0 + j];
                if (x < 0 || (x & kVirtualBit)) continue;
                const int32_t to = (ht.cl.upm_base + ht.cl.item_of[p]) * 2 + j;
                if (ht.cl.item_of[x] >= 0) {
                    cl_pslot[ht.cl.item_of[x]] = ht.cl.slot_of[x] >= 0 ? -1 : to;
                } else {
                    if (pos_k[x] >= 0) pslot_kc[pos_k[x]] = to;
                    if (pos_g[x] >= 0) pslot_gc[pos_g[x]] = to;
                }
            }
        }
    }
    ht.up_items_k = (int32_t)up_desc_k.size();
    ht.up_items_g = (int32_t)up_desc_g.size();
    // Sankoff: binary recomputed children; its part descriptors are the subtree form's (nodes
    // above 255 children never group), so pad0 / pad1 here index the grouped array only
    auto groups_gs = make_groups(2, ht.up_level_off_gs, ht.up_class_off_gs, ht.up_leafy_gs, ht.up_recomp_gs, ht.up_plain_gs,
                                 all_levels);
    std::vector<NodeDesc> up_desc_gs = groups_gs.first;
    const std::vector<int32_t> pslot_gs = make_pslot(groups_gs.second, up_desc_gs);
    ht.up_items_gs = (int32_t)up_desc_gs.size();
    // subtree-form pre-order descriptors list only the children the level kernel handles:
    // S2 / S3 children are tail items (k_tail<.., SUB>); a node left with none gets a
    // materialised placeholder (c0 = 0, no loads, no records)
    std::vector<NodeDesc> down_desc_k = with_gp(make_desc(down_order_k, child_enc_k));
    const std::vector<NodeDesc> down_desc_ks = down_desc_k;   // (PM_OPT_SUB_DOWN: S children kept)
    for (NodeDesc& x : down_desc_k) {
        const int32_t deg = x.e1 - x.e0;
        if (deg > 2) continue;   // S2 / S3 nodes have parents of out-degree <= 2
        int32_t keep_enc[2], keep_vl[2][4], nk = 0;
        for (int j = 0; j < deg; ++j) {
            const int32_t enc = j == 0 ? x.c0 : x.c1;
            if (enc >= 0 && (enc & kVirtualBit) && ((enc >> kShapeShift) & 3)) continue;
            keep_enc[nk] = enc;
            for (int q = 0; q < 4; ++q) keep_vl[nk][q] = j == 0 ? x.vl0[q] : x.vl1[q];
            ++nk;
        }
        if (nk == deg) continue;
        x.e0 = 0;
        x.e1 = std::max(nk, 1);
        x.c0 = nk > 0 ? keep_enc[0] : 0;
        x.c1 = nk > 1 ? keep_enc[1] : 0;
        for (int q = 0; q < 4; ++q) {
            x.vl0[q] = nk > 0 ? keep_vl[0][q] : -1;
            x.vl1[q] = nk > 1 ? keep_vl[1][q] : -1;
        }
    }
    // the pre-order over the sweeps' clusters (every level swept only)
    ht.cl.down = plan_cluster_down(ht, down_order_k, down_desc_k, child_enc_k, ht.cl);
    phase_add("cluster.down", ht.cl.down ? 1.0 : 0.0);
    auto make_tail = [&](const std::vector<int32_t>& order, const std::vector<int32_t>& enc) {
        std::vector<TailDesc> tail;
        for (int32_t d : order)
            for (int32_t e = ht.child_off[d] + 2; e < ht.child_off[d + 1]; ++e) {
                const int32_t x = enc[e];
                if (x >= 0 && !(x & kVirtualBit)) continue;   // materialised child: its own wave
                TailDesc t{};
                t.parent = d;
                t.enc = x;
                t.ix = t.iy = -1;
                for (int j = 0; j < 4; ++j) t.vl[j] = x >= 0 ? vleaf[(size_t)(x & kDenseMask) * 4 + j] : -1;
                t.id[0] = x < 0 ? ht.leaf_id[-x - 1] : ht.internal_id[x & kDenseMask];
                for (int j = 0; j < 4; ++j) t.id[1 + j] = t.vl[j] >= 0 ? ht.leaf_id[t.vl[j]] : -1;
                tail.push_back(t);
            }
        return tail;
    };
    upload_phase("descriptors");
    std::vector<TailDesc> tail_desc = make_tail(down_order, ht.child_enc);
    std::vector<TailDesc> tail_desc_v = make_tail(down_order_v, child_enc_v);
    ht.num_tail = (int32_t)tail_desc.size();
    ht.num_tail_v = (int32_t)tail_desc_v.size();
    // subtree form: every S2 / S3 node, in dense order (item k = dense index sbase + k), then
    // the leaf-parent form's items
    std::vector<TailDesc> tail_desc_k;
    ht.sbase = -1;
    for (int32_t d = 0; d < I; ++d) {
        if (!sshape[d]) continue;
        if (ht.sbase < 0) ht.sbase = d;
        TailDesc t{};
        t.parent = parent_dense[d];
        t.enc = (d | kVirtualBit) | (sshape[d] << kShapeShift);
        for (int j = 0; j < 4; ++j) t.vl[j] = vleaf[(size_t)d * 4 + j];
        t.ix = ht.internal_id[vinner[(size_t)d * 2]];
        t.iy = vinner[(size_t)d * 2 + 1] >= 0 ? ht.internal_id[vinner[(size_t)d * 2 + 1]] : -1;
        t.id[0] = ht.internal_id[d];
        for (int j = 0; j < 4; ++j) t.id[1 + j] = t.vl[j] >= 0 ? ht.leaf_id[t.vl[j]] : -1;
        tail_desc_k.push_back(t);
    }
    ht.num_tail_s = (int32_t)tail_desc_k.size();
    for (int32_t k = 0; k < ht.num_tail_s; ++k)
        if (ht.sbase + k >= I || !sshape[ht.sbase + k]) return fail(c, PM_ERR_STATE, "S2 / S3 nodes not one dense range");
    // tail items by their parent's pre-order level (the subtree form's levels are the leaf-
    // parent form's, S2 / S3 nodes removed): neighbouring waves read neighbouring parents
    {
        auto by_level = [&](std::vector<TailDesc>& tail, const std::vector<int32_t>& order,
                            const std::vector<int32_t>& offs) {
            std::vector<int32_t> lvl_of(I, 0);
            for (size_t l = 0; l + 1 < offs.size(); ++l)
                for (int32_t i = offs[l]; i < offs[l + 1]; ++i) lvl_of[order[i]] = (int32_t)l;
            std::stable_sort(tail.begin(), tail.end(),
                             [&](const TailDesc& x, const TailDesc& y) { return lvl_of[x.parent] < lvl_of[y.parent]; });
        };
        by_level(tail_desc, down_order, ht.down_level_off);
        by_level(tail_desc_v, down_order_v, ht.down_level_off_v);
    }
    tail_desc_k.insert(tail_desc_k.end(), tail_desc_v.begin(), tail_desc_v.end());
    ht.num_tail_k = (int32_t)tail_desc_k.size();

    // Sankoff parts: nodes of out-degree > 255, children cut into kPartChildren-wide parts
    std::vector<PartDesc> part_desc[4];
    for (int v = 0; v < 4; ++v) {
        const std::vector<NodeDesc>& ud = v == 3 ? up_desc_gs : v == 2 ? up_desc_k : v ? up_desc_v : up_desc;
        std::vector<int32_t>& po = v == 3 ? ht.part_off_gs : v == 2 ? ht.part_off_k : v ? ht.part_off_v : ht.part_off;
        po.assign(ud.size() + 1, 0);
        ht.up_degree[v].assign(ud.size(), 0);
        for (size_t k = 0; k < ud.size(); ++k) {
            const int32_t deg = ud[k].e1 - ud[k].e0;
            ht.up_degree[v][k] = deg;
            const int32_t np = deg > 255 ? (deg + kPartChildren - 1) / kPartChildren : 0;
            for (int32_t j = 0; j < np; ++j) part_desc[v].push_back(PartDesc{(int32_t)k, j, po[k] + j, 0});
            po[k + 1] = po[k] + np;
        }
    }
    // pad0 = the first part (Sankoff up descriptors; the Fitch level kernels do not read it)
    std::vector<NodeDesc> up_desc_p = up_desc, up_desc_vp = up_desc_v, up_desc_kp = up_desc_k;
    for (size_t k = 0; k < up_desc_p.size(); ++k) up_desc_p[k].pad0 = ht.part_off[k];
    for (size_t k = 0; k < up_desc_vp.size(); ++k) up_desc_vp[k].pad0 = ht.part_off_v[k];
    for (size_t k = 0; k < up_desc_kp.size(); ++k) up_desc_kp[k].pad0 = ht.part_off_k[k];
    for (size_t k = 0; k < up_desc_gs.size(); ++k)   // (grouped nodes have out-degree <= 3: pad0 / pad1 stay theirs)
        if (up_desc_gs[k].e1 - up_desc_gs[k].e0 > 255) up_desc_gs[k].pad0 = ht.part_off_gs[k];
    upload_phase("parts");
    std::vector<int32_t> lvl;
    {
        const std::vector<int32_t>* up[5] = {&ht.up_class_off, &ht.up_class_off_v, &ht.up_class_off_k, &ht.up_class_off_g,
                                             &ht.up_class_off_gs};
        const std::vector<int32_t>* dn[3] = {&ht.down_level_off, &ht.down_level_off_v, &ht.down_level_off_k};
        for (int f = 0; f < 5; ++f) {
            ht.lvl_up[f] = (int64_t)lvl.size();
            lvl.insert(lvl.end(), up[f]->begin(), up[f]->end());
            if (f >= 3) continue;
            ht.lvl_down[f] = (int64_t)lvl.size();
            lvl.insert(lvl.end(), dn[f]->begin(), dn[f]->end());
        }
        ht.lvl_base_k = (int64_t)lvl.size();
        lvl.insert(lvl.end(), ht.down_dense_base_k.begin(), ht.down_dense_base_k.end());
    }

    free_work(c);
    free_columns(c);
    free_tree(c->dt);
    DevTree dt;
    dt.num_internal = I;
    dt.num_leaves = L;
    dt.root_dense = ht.dense_of[t->root];
    hipError_t e;
    size_t tree_bytes = 0;   // (pm_memory_footprint)
    auto up = [&](auto** dst, const auto& v) {
        tree_bytes += sizeof(v[0]) * v.size();
        return upload(dst, v, c->stream);
    };
    if ((e = up(&dt.child_off, ht.child_off)) != hipSuccess ||
        (e = up(&dt.child_enc, ht.child_enc)) != hipSuccess ||
        (e = up(&dt.parent_dense, parent_dense)) != hipSuccess ||
        (e = up(&dt.internal_id, ht.internal_id)) != hipSuccess ||
        (e = up(&dt.leaf_id, ht.leaf_id)) != hipSuccess ||
        (e = up(&dt.up_order, up_order)) != hipSuccess ||
        (e = up(&dt.down_order, down_order)) != hipSuccess ||
        (e = up(&dt.leaf_parent, leaf_parent)) != hipSuccess ||
        (e = up(&dt.leaf_down, leaf_down)) != hipSuccess ||
        (e = up(&dt.child_enc_v, child_enc_v)) != hipSuccess ||
        (e = up(&dt.up_order_v, up_order_v)) != hipSuccess ||
        (e = up(&dt.down_order_v, down_order_v)) != hipSuccess ||
        (e = up(&dt.down_desc, down_desc)) != hipSuccess ||
        (e = up(&dt.up_desc, up_desc_p)) != hipSuccess ||
        (e = up(&dt.up_desc_v, up_desc_vp)) != hipSuccess ||
        (e = up(&dt.down_desc_v, down_desc_v)) != hipSuccess ||
        (e = up(&dt.vleaf, vleaf)) != hipSuccess ||
        (e = up(&dt.tail_desc, tail_desc)) != hipSuccess ||
        (e = up(&dt.tail_desc_v, tail_desc_v)) != hipSuccess ||
        (e = up(&dt.part_desc, part_desc[0])) != hipSuccess ||
        (e = up(&dt.part_desc_v, part_desc[1])) != hipSuccess ||
        (e = up(&dt.part_desc_k, part_desc[2])) != hipSuccess ||
        (e = up(&dt.part_desc_gs, part_desc[3])) != hipSuccess ||
        (e = up(&dt.child_enc_k, child_enc_k)) != hipSuccess ||
        (e = up(&dt.up_desc_k, up_desc_kp)) != hipSuccess ||
        (e = up(&dt.up_desc_g, up_desc_g)) != hipSuccess ||
        (e = up(&dt.up_desc_gs, up_desc_gs)) != hipSuccess ||
        (e = up(&dt.down_desc_k, down_desc_k)) != hipSuccess ||
        (e = up(&dt.down_desc_ks, down_desc_ks)) != hipSuccess ||
        (e = up(&dt.pslot_k, pslot_k)) != hipSuccess ||
        (e = up(&dt.pslot_g, pslot_g)) != hipSuccess ||
        (e = up(&dt.pslot_gs, pslot_gs)) != hipSuccess ||
        (e = up(&dt.vinner, vinner)) != hipSuccess ||
        (e = up(&dt.tail_desc_k, tail_desc_k)) != hipSuccess ||
        (e = up(&dt.lvl, lvl)) != hipSuccess ||
        (e = up(&dt.cl_items, ht.cl.items)) != hipSuccess ||
        (e = up(&dt.cl_down_items, ht.cl.down_items)) != hipSuccess ||
        (e = up(&dt.cl_wg_off, ht.cl.wg_off)) != hipSuccess ||
        (e = up(&dt.cl_slot_of, ht.cl.slot_of)) != hipSuccess ||
        (e = up(&dt.pslot_kc, pslot_kc)) != hipSuccess ||
        (e = up(&dt.pslot_gc, pslot_gc)) != hipSuccess ||
        (e = up(&dt.cl_pslot, cl_pslot)) != hipSuccess) {
        free_tree(dt);
        return hip_fail(c, e, "tree upload");
    }
    for (const NodeDesc& x : ht.cl.items) ht.cl.max_degree = std::max(ht.cl.max_degree, x.e1 - x.e0);
    ht.cl.items.clear();   // (device only)
    ht.cl.items.shrink_to_fit();
    ht.cl.down_items.clear();
    ht.cl.down_items.shrink_to_fit();
    ht.cl.item_of.clear();
    ht.cl.item_of.shrink_to_fit();
    c->dt = dt;
    c->tree_bytes = tree_bytes;
    c->ht = std::move(ht);
    c->max_degree = 0;
    for (int32_t d = 0; d < I; ++d) c->max_degree = std::max(c->max_degree, c->ht.child_off[d + 1] - c->ht.child_off[d]);
    c->has_tree = true;
    upload_phase("device upload");
    return PM_OK;
}

int pm_leaves_upload(pm_ctx* c, int64_t S, const uint8_t* codes4, int64_t row_stride, const int32_t* node_row,
                     const uint8_t* present, int64_t present_stride) {
    if (!c) return PM_ERR_ARG;
    if (!c->has_tree) return fail(c, PM_ERR_STATE, "upload the tree first");
    if (S <= 0 || S >= (int64_t)1 << 24 || !codes4 || !node_row || row_stride < (S + 1) / 2)
        return fail(c, PM_ERR_ARG, "bad leaf matrix arguments (0 < sites < 2^24)");
    if (present && present_stride < (S + 7) / 8) return fail(c, PM_ERR_ARG, "bad presence stride");
    (void)hipSetDevice(c->device);
    const int32_t L = c->dt.num_leaves;
    std::vector<int32_t> row_of_leaf(L);
    std::vector<uint8_t> flag(L);
    int32_t rows = 0;
    for (int32_t l = 0; l < L; ++l) {
        row_of_leaf[l] = node_row[c->ht.leaf_id[l]];
        flag[l] = row_of_leaf[l] < 0 ? kLeafAbsent : (present ? kLeafPartial : kLeafPresent);
        rows = std::max(rows, row_of_leaf[l] + 1);
    }
    int rc = alloc_columns(c, S);
    if (rc != PM_OK) return rc;
    const int64_t wpad = wpad_of(c);
    hipError_t e;
    if (present && (e = dev_alloc(&c->leaf_present, (size_t)L * wpad)) != hipSuccess)
        return fail(c, PM_ERR_OOM, "presence planes");
    uint8_t* d_codes = nullptr;
    uint8_t* d_present = nullptr;
    int32_t* d_rows = nullptr;
    const size_t code_bytes = (size_t)rows * row_stride;
    const size_t pres_bytes = present ? (size_t)rows * present_stride : 0;
    if ((e = dev_alloc(&d_codes, code_bytes)) != hipSuccess || (e = upload(&d_rows, row_of_leaf, c->stream)) != hipSuccess ||
        (present && (e = dev_alloc(&d_present, pres_bytes)) != hipSuccess)) {
        dev_free(d_codes);
        dev_free(d_rows);
        dev_free(d_present);
        return fail(c, PM_ERR_OOM, "leaf staging");
    }
    e = hipMemcpyAsync(d_codes, codes4, code_bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && present) e = hipMemcpyAsync(d_present, present, pres_bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(c->leaf_flag, flag.data(), L, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_pack_codes(c, d_codes, row_stride, d_rows, d_present, present_stride);
    c->leaves_all_present = std::all_of(flag.begin(), flag.end(), [](uint8_t f) { return f == kLeafPresent; });
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(d_codes);
    dev_free(d_rows);
    dev_free(d_present);
    if (e != hipSuccess) return hip_fail(c, e, "leaf upload");
    c->has_leaves = true;
    c->sub_planes_ok = false;
    return build_sub_planes(c);
}

int pm_sites_upload(pm_ctx* c, const uint8_t* consensus4, const uint8_t* forced4) {
    if (!c || !consensus4) return fail(c, PM_ERR_ARG, "consensus required");
    if (!c->has_leaves) return fail(c, PM_ERR_STATE, "upload the leaves first");
    (void)hipSetDevice(c->device);
    const size_t bytes = (size_t)(c->num_sites + 1) / 2;
    uint8_t* d = nullptr;
    hipError_t e = dev_alloc(&d, bytes);
    if (e != hipSuccess) return fail(c, PM_ERR_OOM, "site staging");
    e = hipMemcpyAsync(d, consensus4, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_pack_sites(c, d, c->cons);
    if (e == hipSuccess && forced4) {
        e = hipMemcpyAsync(d, forced4, bytes, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = launch_pack_sites(c, d, c->forced);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(d);
    if (e != hipSuccess) return hip_fail(c, e, "site upload");
    c->has_forced = forced4 != nullptr;
    c->has_sites = true;
    return PM_OK;
}

int pm_run(pm_ctx* c, int mode) {
    if (!c) return PM_ERR_ARG;
    if (mode < PM_MODE_FITCH || mode > PM_MODE_BLOCK_SANKOFF) return fail(c, PM_ERR_ARG, "unknown mode");
    if (!c->has_tree || !c->has_leaves || !c->has_sites) return fail(c, PM_ERR_STATE, "tree, leaves and sites first");
    (void)hipSetDevice(c->device);
    int rc = alloc_work(c, mode);
    if (rc == PM_OK) rc = build_sub_planes(c);   // (current after every upload; a new tree resets it)
    if (rc != PM_OK) return rc;
    return run_once(c, mode);
}

int pm_mutation_count(pm_ctx* c, int64_t* count) {
    if (!c || !count) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    std::vector<uint32_t> counts;
    int rc = settle(c, counts);
    if (rc != PM_OK) return rc;
    int64_t n = 0;
    for (uint32_t k : counts) n += k;
    *count = n;
    return PM_OK;
}

int pm_mutations_fetch(pm_ctx* c, pm_mut* out, int64_t cap, int64_t* count) {
    if (!c || !count) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    std::vector<uint32_t> counts;
    int rc = settle(c, counts);
    if (rc != PM_OK) return rc;
    int64_t n = 0;
    for (uint32_t k : counts) n += k;
    *count = n;
    if (!out) return PM_OK;
    if (cap < n) return fail(c, PM_ERR_ARG, "output capacity too small");
    if (n <= INT32_MAX) {   // device radix sort (pm_sort.hip), one D2H copy
        const hipError_t e = sort_records_to_host(c, counts, n, out);
        return e == hipSuccess ? PM_OK : hip_fail(c, e, "record sort");
    }
    int64_t at = 0;
    for (int s = 0; s < kShards; ++s) {
        if (!counts[s]) continue;
        hipError_t e = hipMemcpyAsync(out + at, c->recs + (size_t)s * c->shard_cap, sizeof(pm_mut) * counts[s],
                                      hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "record download");
        at += counts[s];
    }
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "record download");
    std::sort(out, out + n, [](const pm_mut& a, const pm_mut& b) {
        return a.node != b.node ? a.node < b.node : a.site_info < b.site_info;
    });
    return PM_OK;
}

int pm_site_results(pm_ctx* c, int32_t* score, uint8_t* root_code) {
    if (!c) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    std::vector<uint32_t> counts;
    int rc = settle(c, counts);
    if (rc != PM_OK) return rc;
    hipError_t e = hipSuccess;
    if (score) e = hipMemcpyAsync(score, c->score, sizeof(int32_t) * c->num_sites, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && root_code)
        e = hipMemcpyAsync(root_code, c->root_code, c->num_sites, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "site results");
}

int pm_site_results_device(pm_ctx* c, void* score_device, void* root_device) {
    if (!c) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    const int rc = settle_run(c);
    if (rc != PM_OK) return rc;
    hipError_t e = hipSuccess;
    if (score_device)
        e = hipMemcpyAsync(score_device, c->score, sizeof(int32_t) * c->num_sites, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess && root_device)
        e = hipMemcpyAsync(root_device, c->root_code, c->num_sites, hipMemcpyDeviceToDevice, c->stream);
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "site results (device)");
}

int pm_kernel_times(pm_ctx* c, double* ms, int64_t* launches, int classes) {
    if (!c || !ms || !launches) return PM_ERR_ARG;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "timer sync");
    for (int k = 0; k < classes; ++k) {
        ms[k] = 0.0;
        launches[k] = 0;
        if (k >= kClasses) continue;
        for (size_t i = 0; i < c->timers_used[k]; ++i) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, c->timers[k][i].a, c->timers[k][i].b) == hipSuccess) ms[k] += t;
        }
        launches[k] = (int64_t)c->timers_used[k];
        c->timers_used[k] = 0;
    }
    return PM_OK;
}

int pm_synth_columns(pm_ctx* c, int64_t site_begin, int64_t S, uint64_t seed) {
    if (!c) return PM_ERR_ARG;
    if (!c->has_tree) return fail(c, PM_ERR_STATE, "upload the tree first");
    if (S <= 0 || S >= (int64_t)1 << 24 || site_begin < 0) return fail(c, PM_ERR_ARG, "bad site range");
    (void)hipSetDevice(c->device);
    int rc = alloc_columns(c, S);
    if (rc != PM_OK) return rc;
    // the generator stages internal sequences in `finals` ([I][W] uint4), scratch freed after it
    // (15 GB at 1M leaves x 30k sites that a run does not need)
    hipError_t e = dev_alloc(&c->finals, (size_t)c->dt.num_internal * wpad_of(c));
    if (e != hipSuccess) return fail(c, PM_ERR_OOM, std::string("generator scratch: ") + hipGetErrorString(e));
    c->finals_bytes = sizeof(uint4) * (size_t)c->dt.num_internal * wpad_of(c);
    std::vector<uint8_t> flag(c->dt.num_leaves, kLeafPresent);
    e = hipMemcpyAsync(c->leaf_flag, flag.data(), flag.size(), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_synth(c, site_begin, seed);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(c->finals);
    c->finals_bytes = 0;
    if (e != hipSuccess) return hip_fail(c, e, "synthetic columns");
    c->has_leaves = c->has_sites = true;
    c->leaves_all_present = true;
    c->has_forced = false;
    c->sub_planes_ok = false;
    return build_sub_planes(c);
}

int pm_leaf_codes_fetch(pm_ctx* c, int64_t s0, int64_t ns, uint8_t* out) {
    if (!c || !out || s0 < 0 || ns <= 0) return fail(c, PM_ERR_ARG, "bad range");
    if (!c->has_leaves || s0 + ns > c->num_sites) return fail(c, PM_ERR_STATE, "range outside the uploaded sites");
    (void)hipSetDevice(c->device);
    uint8_t* d = nullptr;
    const size_t bytes = (size_t)c->dt.num_leaves * ns;
    hipError_t e = dev_alloc(&d, bytes);
    if (e != hipSuccess) return fail(c, PM_ERR_OOM, "fetch staging");
    e = launch_unpack_leaf_codes(c, s0, ns, d);
    std::vector<uint8_t> by_rank(bytes);
    if (e == hipSuccess) e = hipMemcpyAsync(by_rank.data(), d, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(d);
    if (e != hipSuccess) return hip_fail(c, e, "leaf fetch");
    // rows by leaf rank (tree order) -> rows in increasing node-id order
    std::vector<int32_t> ranks(c->dt.num_leaves);
    std::iota(ranks.begin(), ranks.end(), 0);
    std::sort(ranks.begin(), ranks.end(), [&](int32_t x, int32_t y) { return c->ht.leaf_id[x] < c->ht.leaf_id[y]; });
    for (size_t k = 0; k < ranks.size(); ++k)
        std::memcpy(out + k * ns, by_rank.data() + (size_t)ranks[k] * ns, (size_t)ns);
    return PM_OK;
}

int pm_consensus_fetch(pm_ctx* c, int64_t s0, int64_t ns, uint8_t* out) {
    if (!c || !out || s0 < 0 || ns <= 0) return fail(c, PM_ERR_ARG, "bad range");
    if (!c->has_sites || s0 + ns > c->num_sites) return fail(c, PM_ERR_STATE, "range outside the uploaded sites");
    (void)hipSetDevice(c->device);
    uint8_t* d = nullptr;
    hipError_t e = dev_alloc(&d, (size_t)ns);
    if (e != hipSuccess) return fail(c, PM_ERR_OOM, "fetch staging");
    e = launch_unpack_sites(c, c->cons, s0, ns, d);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, ns, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dev_free(d);
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "consensus fetch");
}

int pm_synth_tree_random_join(int64_t leaves, uint64_t seed, int32_t* child_offsets, int32_t* child_index,
                              int32_t* root) {
    // SURVEY.md §8d family T1: repeatedly join two uniformly chosen pool items.
    if (leaves < 2 || leaves > (int64_t)1 << 30 || !child_offsets || !child_index || !root) return PM_ERR_ARG;
    std::mt19937_64 rng(seed);
    std::vector<int32_t> pool(leaves);
    std::iota(pool.begin(), pool.end(), 0);
    const int64_t N = 2 * leaves - 1;
    for (int64_t i = 0; i <= leaves; ++i) child_offsets[i] = 0;
    int32_t next = (int32_t)leaves;
    int64_t e = 0;
    while (pool.size() > 1) {
        size_t m = pool.size();
        size_t a = rng() % m;
        std::swap(pool[a], pool[m - 1]);
        const int32_t x = pool[m - 1];
        pool.pop_back();
        --m;
        size_t b = rng() % m;
        std::swap(pool[b], pool[m - 1]);
        const int32_t y = pool[m - 1];
        pool.pop_back();
        child_index[e++] = x;
        child_index[e++] = y;
        child_offsets[next + 1] = (int32_t)e;
        pool.push_back(next++);
    }
    (void)N;
    *root = pool[0];
    return PM_OK;
}

int pm_synth_tree_sars_like(int64_t leaves, uint64_t seed, int32_t* child_offsets, int32_t* child_index,
                            int32_t* root, int64_t* num_nodes) {
    // SURVEY.md §8d family T2: ladderised sequential insertion -- leaf i splits the pendant
    // edge of leaf i-1 with p = 0.9, else of a uniform earlier leaf -- then 10 % of the
    // internal nodes are merged away (edge contraction) into polytomies of 3-64 children.
    if (leaves < 2 || leaves > (int64_t)1 << 29 || !child_offsets || !child_index || !root || !num_nodes)
        return PM_ERR_ARG;
    std::mt19937_64 rng(seed);
    auto uniform = [&](uint64_t n) { return (uint64_t)((unsigned __int128)rng() * n >> 64); };
    auto coin = [&](double p) { return (double)(rng() >> 11) * 0x1.0p-53 < p; };
    const int64_t L = leaves, N0 = 2 * leaves - 1;
    std::vector<int32_t> par(N0, -1);
    std::vector<std::vector<int32_t>> kids(N0);
    int32_t next = (int32_t)L;
    const int32_t r = next++;
    kids[r] = {0, 1};
    par[0] = par[1] = r;
    for (int64_t i = 2; i < L; ++i) {
        const int32_t t = coin(0.9) ? (int32_t)(i - 1) : (int32_t)uniform((uint64_t)i);
        const int32_t q = par[t], v = next++;
        for (int32_t& k : kids[q])
            if (k == t) k = v;
        par[v] = q;
        kids[v] = {t, (int32_t)i};
        par[t] = par[i] = v;
    }
    // polytomies: visit internal non-root nodes in random order; a visited node absorbs
    // internal children (its own kids first) until it has k ~ U[3,64] children, never more
    // than 64, until 10 % of the internal nodes are gone
    std::vector<int32_t> perm;
    for (int32_t v = (int32_t)L + 1; v < next; ++v) perm.push_back(v);
    for (size_t i = perm.size(); i > 1; --i) std::swap(perm[i - 1], perm[uniform(i)]);
    std::vector<uint8_t> dead(N0, 0);
    int64_t budget = (int64_t)(0.1 * (double)(next - L));
    for (int32_t v : perm) {
        if (budget <= 0) break;
        if (dead[v]) continue;
        const size_t k = 3 + (size_t)uniform(62);
        size_t scan = 0;
        while (kids[v].size() < k && budget > 0 && scan < kids[v].size()) {
            const int32_t c = kids[v][scan];
            if (c < L || kids[v].size() - 1 + kids[c].size() > 64) {
                ++scan;
                continue;
            }
            std::vector<int32_t> g = std::move(kids[c]);
            kids[v].erase(kids[v].begin() + scan);
            kids[v].insert(kids[v].begin() + scan, g.begin(), g.end());
            for (int32_t x : g) par[x] = v;
            dead[c] = 1;
            --budget;
        }
    }
    // compact ids: leaves keep [0, L), surviving internal nodes follow in creation order
    std::vector<int32_t> id(N0, -1);
    int32_t n = 0;
    for (int32_t v = 0; v < next; ++v)
        if (!dead[v]) id[v] = n++;
    int64_t e = 0;
    child_offsets[0] = 0;
    for (int32_t v = 0; v < next; ++v) {
        if (dead[v]) continue;
        for (int32_t c : kids[v]) child_index[e++] = id[c];
        child_offsets[id[v] + 1] = (int32_t)e;
    }
    *root = id[r];
    *num_nodes = n;
    return PM_OK;
}

}  // extern "C"
