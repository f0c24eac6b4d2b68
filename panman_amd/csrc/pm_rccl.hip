// pm_rccl.hip -- column shards over several GPUs with one RCCL all-gather.
//
// The reference's alignment columns are independent (src/panman.cpp:1381 Fitch, :1568
// Sankoff: one parsimony call per column), so each GPU runs the level kernels over its own
// contiguous site range with the tree replicated.  The only exchange is the per-site result
// the north star names -- parsimony score and root code -- gathered with ONE ncclAllGather
// over xGMI: every rank contributes a fixed-size chunk of packed 8-B entries
// {score:int32, root:u8} headed by its (site_begin, count), so ranks may hold uneven or
// even-aligned ranges and nobody needs the others' shard rule.  Mutation records stay on
// their rank (local site indices) and are merged by (node, global site) on the host.
//
// RCCL is opened at run time (dlopen "librccl.so.1"): inside a PyTorch process that is
// torch's already-loaded copy (same soname), so one RCCL instance serves both; the
// single-GPU entry points never load it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "pm_chunk.h"
#include "pm_internal.h"

namespace pm {
namespace {

struct Rccl {
    bool ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.why = std::string("librccl.so.1 not loadable: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all &= fn != nullptr;
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.init_rank, "ncclCommInitRank");
        sym(r.init_all, "ncclCommInitAll");
        sym(r.all_gather, "ncclAllGather");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.destroy, "ncclCommDestroy");
        sym(r.count, "ncclCommCount");
        sym(r.user_rank, "ncclCommUserRank");
        sym(r.error_string, "ncclGetErrorString");
        r.ok = all;
        if (!all) r.why = "librccl.so.1 lacks an expected symbol";
    });
    return r;
}

int rccl_fail(pm_ctx* c, ncclResult_t e, const char* what) {
    return fail(c, PM_ERR_HIP, std::string(what) + ": " + rccl().error_string(e));
}

__global__ void k_pack_results(const int32_t* score, const uint8_t* root, int64_t begin, int64_t count, bool ok,
                               uint64_t* chunk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) chunk[0] = ok ? chunk_head(begin, count) : chunk_failed_head();
    if (ok && i < count) chunk[1 + i] = chunk_entry(score[i], root[i]);
}

__global__ void k_unpack_results(const uint64_t* all, int64_t per, int n, int64_t total, int32_t* score,
                                 uint8_t* root, int32_t* status) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) *status = chunk_check(all, per, n, total);
    if (g < per * n) chunk_unpack_one(all, per, g, total, score, root);
}

}  // namespace

void comm_release(pm_ctx* c) {
    if (c->comm && rccl().ok) (void)rccl().destroy(static_cast<ncclComm_t>(c->comm));
    c->comm = nullptr;
    if (c->gather_buf) (void)hipFree(c->gather_buf);
    c->gather_buf = nullptr;
    c->gather_bytes = 0;
}

}  // namespace pm

using namespace pm;

namespace {

// The gather buffers: [send chunk | ranks x chunk | status].
int ensure_gather(pm_ctx* c, int64_t per) {
    const size_t need = sizeof(uint64_t) * ((size_t)per * (size_t)(c->comm_size + 1) + 1);
    if (need <= c->gather_bytes) return PM_OK;
    if (c->gather_buf) (void)hipFree(c->gather_buf);
    c->gather_buf = nullptr;
    c->gather_bytes = 0;
    const hipError_t e = hipMalloc(&c->gather_buf, need);
    if (e != hipSuccess) return hip_fail(c, e, "gather buffers");
    c->gather_bytes = need;
    return PM_OK;
}

int32_t* gather_status(pm_ctx* c, int64_t per) {
    return reinterpret_cast<int32_t*>(static_cast<uint64_t*>(c->gather_buf) + (size_t)per * (c->comm_size + 1));
}

// A rank's shard in two halves, so that one process driving several GPUs (pm_multi_run)
// queues every rank's pm_run before it waits on any of them.
//
// shard_begin: the send chunk is stamped "failed" first (memset, its error checked: a chunk
// is failed until a successful pack overwrites it, so a rank whose run or pack breaks can
// never hand the others a previous call's healthy results), then pm_run on the shard.
int shard_begin(pm_ctx* c, int mode, int64_t total_sites, int64_t site_begin, int64_t per) {
    uint32_t* head = static_cast<uint32_t*>(c->gather_buf);   // little-endian u64: count low, begin high
    hipError_t e = hipMemsetD32Async(head, kChunkFailed, 1, c->stream);
    if (e == hipSuccess) e = hipMemsetD32Async(head + 1, 0u, 1, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "stamp send chunk");
    if (site_begin < 0 || site_begin > UINT32_MAX || c->num_sites > per - 1 || site_begin + c->num_sites > total_sites)
        return fail(c, PM_ERR_ARG, "shard outside [0, total_sites) or wider than ceil(total / ranks) + 2");
    return pm_run(c, mode);
}

// shard_finish: record-buffer overflow settled (a re-run with a bigger buffer: the score
// counts only stored records), then the packed chunk into the send buffer.  A failed rank's
// chunk keeps the failed head, so the caller still joins the collective and every rank
// learns of it from the heads.
int shard_finish(pm_ctx* c, int rc, int64_t site_begin) {
    if (rc == PM_OK) rc = settle_run(c);
    if (rc != PM_OK) return rc;
    hipLaunchKernelGGL(k_pack_results, dim3((unsigned)((c->num_sites + kBlock) / kBlock)), dim3(kBlock), 0, c->stream,
                       c->score, c->root_code, site_begin, c->num_sites, true, static_cast<uint64_t*>(c->gather_buf));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "pack site results");
}

int enqueue_unpack(pm_ctx* c, const uint64_t* recv, int64_t total_sites, int64_t per, void* score_device,
                   void* root_device) {
    const int64_t n = per * c->comm_size;
    hipLaunchKernelGGL(k_unpack_results, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream, recv,
                       per, c->comm_size, total_sites, static_cast<int32_t*>(score_device),
                       static_cast<uint8_t*>(root_device), gather_status(c, per));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "unpack site results");
}

// Wait for the unpack and turn its head check into a status (every rank sees the same heads,
// so every rank returns the same verdict).
int gathered_status(pm_ctx* c, int64_t per) {
    int32_t st = 0;
    hipError_t e = hipMemcpyAsync(&st, gather_status(c, per), sizeof st, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "gather status");
    if (st > 0) return fail(c, PM_ERR_STATE, "rank " + std::to_string(st - 1) + "'s shard failed");
    if (st < 0) return fail(c, PM_ERR_ARG, "gathered shards do not tile [0, total_sites) (shard rules differ between ranks)");
    return PM_OK;
}

int gather_call(pm_ctx* c, int64_t per) {
    uint64_t* buf = static_cast<uint64_t*>(c->gather_buf);
    const ncclResult_t r = rccl().all_gather(buf, buf + per, (size_t)per, ncclUint64,
                                             static_cast<ncclComm_t>(c->comm), c->stream);
    return r == ncclSuccess ? PM_OK : rccl_fail(c, r, "ncclAllGather");
}

}  // namespace

extern "C" {

int pm_comm_unique_id(uint8_t* id, int64_t len) {
    if (!id || len < PM_COMM_ID_BYTES) return PM_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == PM_COMM_ID_BYTES, "ncclUniqueId size");
    if (!rccl().ok) return PM_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (rccl().get_unique_id(&u) != ncclSuccess) return PM_ERR_HIP;
    std::memcpy(id, &u, sizeof u);
    return PM_OK;
}

int pm_comm_init_rank(pm_ctx* c, const uint8_t* id, int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return PM_ERR_ARG;
    if (!rccl().ok) return fail(c, PM_ERR_UNSUPPORTED, rccl().why);
    (void)hipSetDevice(c->device);
    comm_release(c);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = rccl().init_rank(&comm, nranks, u, rank);
    if (r != ncclSuccess) return rccl_fail(c, r, "ncclCommInitRank");
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_size = nranks;
    return PM_OK;
}

int pm_comm_init_all(pm_ctx* const* ctxs, int n) {
    if (!ctxs || n < 1) return PM_ERR_ARG;
    for (int i = 0; i < n; ++i)
        if (!ctxs[i]) return PM_ERR_ARG;
    if (!rccl().ok) return fail(ctxs[0], PM_ERR_UNSUPPORTED, rccl().why);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        devs[i] = ctxs[i]->device;
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i]) return fail(ctxs[i], PM_ERR_ARG, "one communicator rank per device");
        comm_release(ctxs[i]);
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    const ncclResult_t r = rccl().init_all(comms.data(), n, devs.data());
    if (r != ncclSuccess) return rccl_fail(ctxs[0], r, "ncclCommInitAll");
    for (int i = 0; i < n; ++i) {
        ctxs[i]->comm = comms[i];
        ctxs[i]->comm_rank = i;
        ctxs[i]->comm_size = n;
    }
    return PM_OK;
}

int pm_run_gather(pm_ctx* c, int mode, int64_t total_sites, int64_t site_begin, void* score_device,
                  void* root_device) {
    // arguments every rank passes alike: a failure here fails every rank the same way
    if (!c || total_sites < 1 || !score_device || !root_device) return PM_ERR_ARG;
    if (!c->comm) return fail(c, PM_ERR_STATE, "no communicator: pm_comm_init_rank / pm_comm_init_all first");
    (void)hipSetDevice(c->device);
    const int64_t per = chunk_entries(total_sites, c->comm_size);
    int rc = ensure_gather(c, per);   // (a rank that cannot allocate a few KiB cannot join)
    if (rc != PM_OK) return rc;
    // rank-specific work: a failure is carried in this rank's chunk head, the collective joined
    const int local = shard_finish(c, shard_begin(c, mode, total_sites, site_begin, per), site_begin);
    rc = gather_call(c, per);
    if (rc == PM_OK) rc = enqueue_unpack(c, static_cast<const uint64_t*>(c->gather_buf) + per, total_sites, per,
                                         score_device, root_device);
    if (rc == PM_OK) rc = gathered_status(c, per);
    return local != PM_OK ? local : rc;
}

int pm_pack_site_results(pm_ctx* c, int64_t site_begin, int64_t per, void* chunk_device) {
    if (!c || !chunk_device || per < 2) return PM_ERR_ARG;
    if (!c->ran) return fail(c, PM_ERR_STATE, "nothing ran");
    (void)hipSetDevice(c->device);
    int rc = settle_run(c);
    if (rc != PM_OK) return rc;
    if (site_begin < 0 || site_begin > UINT32_MAX || c->num_sites > per - 1)
        return fail(c, PM_ERR_ARG, "shard wider than the chunk (per - 1 sites)");
    hipLaunchKernelGGL(k_pack_results, dim3((unsigned)((c->num_sites + kBlock) / kBlock)), dim3(kBlock), 0, c->stream,
                       c->score, c->root_code, site_begin, c->num_sites, true, static_cast<uint64_t*>(chunk_device));
    // synchronous: the caller's collective may run on another stream (torch's), which nothing
    // orders after this one
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? PM_OK : hip_fail(c, e, "pack site results");
}

int pm_unpack_site_results(pm_ctx* c, const void* all_device, int64_t per, int ranks, int64_t total_sites,
                           void* score_device, void* root_device) {
    if (!c || !all_device || per < 2 || ranks < 1 || total_sites < 1 || !score_device || !root_device) return PM_ERR_ARG;
    (void)hipSetDevice(c->device);
    int32_t* st = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&st), sizeof(int32_t), c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "unpack status");
    const int64_t n = per * ranks;
    hipLaunchKernelGGL(k_unpack_results, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       static_cast<const uint64_t*>(all_device), per, ranks, total_sites,
                       static_cast<int32_t*>(score_device), static_cast<uint8_t*>(root_device), st);
    int32_t v = 0;
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(&v, st, sizeof v, hipMemcpyDeviceToHost, c->stream);
    (void)hipFreeAsync(st, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "unpack site results");
    if (v > 0) return fail(c, PM_ERR_STATE, "rank " + std::to_string(v - 1) + "'s shard failed");
    if (v < 0) return fail(c, PM_ERR_ARG, "gathered shards do not tile [0, total_sites)");
    return PM_OK;
}

int pm_chunk_entries(int64_t total_sites, int ranks, int64_t* per) {
    if (total_sites < 1 || ranks < 1 || !per) return PM_ERR_ARG;
    *per = chunk_entries(total_sites, ranks);
    return PM_OK;
}

int pm_chunk_pack(int64_t site_begin, int64_t count, const int32_t* score, const uint8_t* root, int64_t per,
                  uint64_t* chunk) {
    if (!chunk || per < 2 || count < 0) return PM_ERR_ARG;
    if (!score || !root) {   // a failed shard: the head alone
        chunk[0] = chunk_failed_head();
        return PM_OK;
    }
    if (site_begin < 0 || site_begin > UINT32_MAX || count > per - 1) return PM_ERR_ARG;
    chunk[0] = chunk_head(site_begin, count);
    for (int64_t i = 0; i < count; ++i) chunk[1 + i] = chunk_entry(score[i], root[i]);
    for (int64_t i = count + 1; i < per; ++i) chunk[i] = 0;
    return PM_OK;
}

int pm_chunk_unpack(const uint64_t* all, int64_t per, int ranks, int64_t total_sites, int32_t* score, uint8_t* root) {
    if (!all || per < 2 || ranks < 1 || total_sites < 1 || !score || !root) return PM_ERR_ARG;
    const int st = chunk_check(all, per, ranks, total_sites);
    if (st > 0) return PM_ERR_STATE;
    if (st < 0) return PM_ERR_ARG;
    for (int64_t g = 0; g < per * ranks; ++g) chunk_unpack_one(all, per, g, total_sites, score, root);
    return PM_OK;
}

int pm_multi_run(pm_ctx* const* ctxs, int n, int mode, const int64_t* site_begin, int64_t total_sites,
                 int32_t* score, uint8_t* root_code) {
    if (!ctxs || n < 1 || !site_begin || total_sites < 1) return PM_ERR_ARG;
    for (int i = 0; i < n; ++i)
        if (!ctxs[i] || !ctxs[i]->comm || ctxs[i]->comm_size != n || ctxs[i]->comm_rank != i)
            return ctxs[i] ? fail(ctxs[i], PM_ERR_STATE, "contexts need one pm_comm_init_all communicator, rank = index")
                           : PM_ERR_ARG;
    const int64_t per = chunk_entries(total_sites, n);
    std::vector<void*> out_s(n, nullptr), out_r(n, nullptr);
    int rc = PM_OK;
    for (int i = 0; i < n && rc == PM_OK; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        if (hipMalloc(&out_s[i], sizeof(int32_t) * total_sites) != hipSuccess ||
            hipMalloc(&out_r[i], (size_t)total_sites) != hipSuccess)
            rc = fail(ctxs[i], PM_ERR_OOM, "gathered results");
        if (rc == PM_OK) rc = ensure_gather(ctxs[i], per);
        if (rc == PM_OK) rc = shard_begin(ctxs[i], mode, total_sites, site_begin[i], per);
    }
    // every rank's run is queued before the first wait: the GPUs run their shards together
    for (int i = 0; i < n && rc == PM_OK; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        rc = shard_finish(ctxs[i], rc, site_begin[i]);
    }
    if (rc == PM_OK) {   // one process drives every rank: the collective is one RCCL group
        (void)rccl().group_start();
        for (int i = 0; i < n && rc == PM_OK; ++i) {
            (void)hipSetDevice(ctxs[i]->device);
            rc = gather_call(ctxs[i], per);
        }
        const ncclResult_t r = rccl().group_end();
        if (rc == PM_OK && r != ncclSuccess) rc = rccl_fail(ctxs[0], r, "ncclGroupEnd");
    }
    for (int i = 0; i < n && rc == PM_OK; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        rc = enqueue_unpack(ctxs[i], static_cast<const uint64_t*>(ctxs[i]->gather_buf) + per, total_sites, per,
                            out_s[i], out_r[i]);
    }
    for (int i = 0; i < n && rc == PM_OK; ++i) {
        (void)hipSetDevice(ctxs[i]->device);
        rc = gathered_status(ctxs[i], per);
    }
    if (rc == PM_OK) {   // every rank holds the full vectors; hand back rank 0's
        (void)hipSetDevice(ctxs[0]->device);
        hipError_t e = hipSuccess;
        if (score) e = hipMemcpyAsync(score, out_s[0], sizeof(int32_t) * total_sites, hipMemcpyDeviceToHost, ctxs[0]->stream);
        if (e == hipSuccess && root_code)
            e = hipMemcpyAsync(root_code, out_r[0], (size_t)total_sites, hipMemcpyDeviceToHost, ctxs[0]->stream);
        for (int i = 0; i < n && e == hipSuccess; ++i) {
            (void)hipSetDevice(ctxs[i]->device);
            e = hipStreamSynchronize(ctxs[i]->stream);
        }
        if (e != hipSuccess) rc = hip_fail(ctxs[0], e, "gathered results");
    }
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) continue;
        (void)hipSetDevice(ctxs[i]->device);
        if (ctxs[i]->stream) (void)hipStreamSynchronize(ctxs[i]->stream);
        if (out_s[i]) (void)hipFree(out_s[i]);
        if (out_r[i]) (void)hipFree(out_r[i]);
    }
    return rc;
}

int pm_shard_range(int rank, int ranks, int64_t total_sites, int64_t* begin, int64_t* end) {
    if (ranks < 1 || rank < 0 || rank >= ranks || total_sites < 0 || !begin || !end) return PM_ERR_ARG;
    *begin = (int64_t)rank * total_sites / ranks;
    *end = (int64_t)(rank + 1) * total_sites / ranks;
    return PM_OK;
}

}  // extern "C"
