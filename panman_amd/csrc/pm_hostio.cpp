// pm_hostio.cpp -- host-side plumbing around the kernels: the phase log every driver writes
// its host / device phase times into (pm_phase_report), large device-to-host downloads
// through pinned staging buffers drained by a pool of host threads (the FASTA text), and
// the grow-only device buffers a context keeps between calls.
//
// Why the download pipeline: printFASTAUltraFast's output at config C5 is ~5 GB of text.
// One pageable hipMemcpy of it runs single-threaded through the runtime's own staging and
// first-touches every page of the destination on one core; here the DMA engine fills
// pinned slots (PCIe rate) while host threads copy the previous slot into the destination
// in parallel, so first-touch faults and the host copy are spread over the cores and
// overlap the transfer.
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "pm_internal.h"

namespace pm {

// ---- phase log ---------------------------------------------------------------------------
namespace {
std::mutex g_phase_mu;
std::vector<std::pair<std::string, double>> g_phases;
constexpr size_t kMaxPhases = 4096;
}  // namespace

void phase_add(const std::string& name, double seconds) {
    std::lock_guard<std::mutex> lock(g_phase_mu);
    if (g_phases.size() < kMaxPhases) g_phases.emplace_back(name, seconds);
}

PhaseClock::PhaseClock() : t(std::chrono::steady_clock::now()) {}

double PhaseClock::lap(const char* name) {
    const auto now = std::chrono::steady_clock::now();
    const double s = std::chrono::duration<double>(now - t).count();
    phase_add(name, s);
    t = now;
    return s;
}

int host_threads() {
    if (const char* e = std::getenv("PM_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= 256) return v;
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hc ? hc : 1u));
}

// ---- a small fork-join pool: run(n, fn) calls fn(0..n-1) on the workers and the caller ----
namespace {
class Pool {
  public:
    explicit Pool(int threads) {
        for (int i = 1; i < threads; ++i) workers_.emplace_back([this]() { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lock(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return (int)workers_.size() + 1; }
    // One generation at a time: run() publishes (job, tasks) only when no worker is inside
    // work(), and returns only when every task is done and every worker has left work(), so a
    // worker never mixes one generation's job with another's counter.  Workers take their
    // (job, tasks) snapshot under the lock.
    template <class F>
    void run(int tasks, F&& fn) {
        std::function<void(int)> f(std::forward<F>(fn));
        {
            std::unique_lock<std::mutex> lock(mu_);
            done_.wait(lock, [this]() { return active_ == 0; });
            job_ = &f;
            tasks_ = tasks;
            next_.store(0);
            pending_ = tasks;
            ++gen_;
        }
        cv_.notify_all();
        work(&f, tasks);
        std::unique_lock<std::mutex> lock(mu_);
        done_.wait(lock, [this]() { return pending_ == 0 && active_ == 0; });
        job_ = nullptr;
    }

  private:
    void work(std::function<void(int)>* job, int tasks) {
        for (int i = next_++; i < tasks; i = next_++) {
            (*job)(i);
            std::lock_guard<std::mutex> lock(mu_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(int)>* job = nullptr;
            int tasks = 0;
            {
                std::unique_lock<std::mutex> lock(mu_);
                cv_.wait(lock, [&]() { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (!job_) continue;   // that generation has finished already
                job = job_;
                tasks = tasks_;
                ++active_;
            }
            work(job, tasks);
            std::lock_guard<std::mutex> lock(mu_);
            if (--active_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::function<void(int)>* job_ = nullptr;
    int tasks_ = 0, pending_ = 0, active_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};
}  // namespace

void host_parallel_for(int tasks, const std::function<void(int)>& fn) {
    if (tasks <= 0) return;
    const int t = std::min(tasks, host_threads());
    if (t <= 1) {
        for (int i = 0; i < tasks; ++i) fn(i);
        return;
    }
    Pool pool(t);
    pool.run(tasks, fn);
}

// ---- large downloads ---------------------------------------------------------------------
constexpr size_t kStageChunk = (size_t)64 << 20;   // bytes per pinned slot
constexpr int kStageSlots = 3;                     // slots in flight

void* host_alloc_large(size_t n) {
    void* p = std::malloc(n);
    if (p && n >= ((size_t)64 << 20)) {
        // transparent huge pages where the kernel allows them on request: 512x fewer faults
        const uintptr_t a = ((uintptr_t)p + 4095) & ~(uintptr_t)4095;
        const uintptr_t b = ((uintptr_t)p + n) & ~(uintptr_t)4095;
        if (b > a) (void)madvise(reinterpret_cast<void*>(a), b - a, MADV_HUGEPAGE);
    }
    return p;
}

hipError_t d2h_large(pm_ctx* c, void* dst, const void* src, size_t n) {
    if (n == 0) return hipSuccess;
    if (n < 2 * kStageChunk) {
        hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream);
        return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
    }
    hipError_t e = hipSuccess;
    if (!c->stage) {
        if ((e = hipHostMalloc(&c->stage, kStageChunk * kStageSlots, hipHostMallocDefault)) != hipSuccess) {
            c->stage = nullptr;
            return e;
        }
        for (int s = 0; s < kStageSlots && e == hipSuccess; ++s)
            e = hipEventCreateWithFlags(&c->stage_ev[s], hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    char* stage = static_cast<char*>(c->stage);
    const char* from = static_cast<const char*>(src);
    char* to = static_cast<char*>(dst);
    const int64_t K = (int64_t)((n + kStageChunk - 1) / kStageChunk);
    auto len = [&](int64_t k) { return std::min(kStageChunk, n - (size_t)k * kStageChunk); };
    auto issue = [&](int64_t k) {
        const int s = (int)(k % kStageSlots);
        hipError_t r = hipMemcpyAsync(stage + (size_t)s * kStageChunk, from + (size_t)k * kStageChunk, len(k),
                                      hipMemcpyDeviceToHost, c->stream);
        return r == hipSuccess ? hipEventRecord(c->stage_ev[s], c->stream) : r;
    };
    for (int64_t k = 0; k < std::min<int64_t>(K, kStageSlots) && e == hipSuccess; ++k) e = issue(k);
    const int T = host_threads();
    Pool pool(T);
    constexpr size_t kPiece = (size_t)2 << 20;   // host copy granule (a huge page)
    for (int64_t k = 0; k < K && e == hipSuccess; ++k) {
        const int s = (int)(k % kStageSlots);
        if ((e = hipEventSynchronize(c->stage_ev[s])) != hipSuccess) break;
        const size_t m = len(k);
        const char* slot = stage + (size_t)s * kStageChunk;
        char* out = to + (size_t)k * kStageChunk;
        const int pieces = (int)((m + kPiece - 1) / kPiece);
        pool.run(pieces, [&](int i) {
            const size_t a = (size_t)i * kPiece;
            std::memcpy(out + a, slot + a, std::min(kPiece, m - a));
        });
        if (k + kStageSlots < K) e = issue(k + kStageSlots);
    }
    if (e != hipSuccess) (void)hipStreamSynchronize(c->stream);
    return e;
}

// The same pinned slots, each chunk handed to `sink` (the caller's file descriptor) as soon as
// it lands instead of copied into a host buffer: the device text streams to its destination
// while the next chunks are in flight.  false from sink: stop (the write failed).
hipError_t d2h_stream(pm_ctx* c, const void* src, size_t n, const std::function<bool(const char*, size_t)>& sink,
                      bool& sink_ok) {
    sink_ok = true;
    if (n == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!c->stage) {
        if ((e = hipHostMalloc(&c->stage, kStageChunk * kStageSlots, hipHostMallocDefault)) != hipSuccess) {
            c->stage = nullptr;
            return e;
        }
        for (int s = 0; s < kStageSlots && e == hipSuccess; ++s)
            e = hipEventCreateWithFlags(&c->stage_ev[s], hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    char* stage = static_cast<char*>(c->stage);
    const char* from = static_cast<const char*>(src);
    const int64_t K = (int64_t)((n + kStageChunk - 1) / kStageChunk);
    auto len = [&](int64_t k) { return std::min(kStageChunk, n - (size_t)k * kStageChunk); };
    auto issue = [&](int64_t k) {
        const int s = (int)(k % kStageSlots);
        hipError_t r = hipMemcpyAsync(stage + (size_t)s * kStageChunk, from + (size_t)k * kStageChunk, len(k),
                                      hipMemcpyDeviceToHost, c->stream);
        return r == hipSuccess ? hipEventRecord(c->stage_ev[s], c->stream) : r;
    };
    for (int64_t k = 0; k < std::min<int64_t>(K, kStageSlots) && e == hipSuccess; ++k) e = issue(k);
    for (int64_t k = 0; k < K && e == hipSuccess; ++k) {
        const int s = (int)(k % kStageSlots);
        if ((e = hipEventSynchronize(c->stage_ev[s])) != hipSuccess) break;
        if (sink_ok) sink_ok = sink(stage + (size_t)s * kStageChunk, len(k));
        if (!sink_ok) break;
        if (k + kStageSlots < K) e = issue(k + kStageSlots);
    }
    (void)hipStreamSynchronize(c->stream);   // (slots still in flight after a failed write)
    return e;
}

bool write_all(int fd, const char* p, size_t n) {
    while (n > 0) {
        const ssize_t w = ::write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        n -= (size_t)w;
    }
    return true;
}

void free_hostio(pm_ctx* c) {
    if (c->stage) (void)hipHostFree(c->stage);
    c->stage = nullptr;
    for (auto& ev : c->stage_ev) {
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
    }
    if (c->text_buf) (void)hipFree(c->text_buf);
    c->text_buf = nullptr;
    c->text_cap = 0;
    if (c->rows_buf) (void)hipFree(c->rows_buf);
    c->rows_buf = nullptr;
    c->rows_cap = 0;
}

// The FASTA text and replay rows stay on the device between calls (grow-only, up to ~10 GB at
// C5).  A large allocation that fails drops them and tries once more, so a context that
// replayed before still runs a pass that needs the room (the rows only when no replay state
// refers to them).
void release_cached(pm_ctx* c) {
    if (c->text_buf) (void)hipFree(c->text_buf);
    c->text_buf = nullptr;
    c->text_cap = 0;
    if (!c->replay && c->rows_buf) {
        (void)hipFree(c->rows_buf);
        c->rows_buf = nullptr;
        c->rows_cap = 0;
    }
}

hipError_t malloc_or_release(pm_ctx* c, void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 1));
    if (e == hipSuccess || (!c->text_buf && (c->replay || !c->rows_buf))) return e;
    (void)hipGetLastError();
    release_cached(c);
    return hipMalloc(p, std::max<size_t>(bytes, 1));
}

hipError_t grow_device(void** buf, size_t* cap, size_t need) {
    if (need <= *cap && *buf) return hipSuccess;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(buf, std::max<size_t>(need, 1));
    if (e == hipSuccess) *cap = std::max<size_t>(need, 1);
    else *buf = nullptr;
    return e;
}

}  // namespace pm

extern "C" {

void pm_phase_reset(void) {
    std::lock_guard<std::mutex> lock(pm::g_phase_mu);
    pm::g_phases.clear();
}

int64_t pm_phase_report(char* buf, int64_t len) {
    std::string s;
    {
        std::lock_guard<std::mutex> lock(pm::g_phase_mu);
        char line[64];
        for (auto& p : pm::g_phases) {
            std::snprintf(line, sizeof line, "\t%.6f\n", p.second);
            s += p.first;
            s += line;
        }
    }
    if (buf && len > 0) {
        const size_t n = std::min<size_t>(s.size(), (size_t)len - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int64_t)s.size() + 1;
}

}  // extern "C"

extern "C" {

int pm_memory_footprint(pm_ctx* c, int64_t* out, int n) {
    if (!c || !out || n < 1) return PM_ERR_ARG;
    const int64_t wpad = (int64_t)((c->words + pm::kWave - 1) / pm::kWave) * pm::kWave;
    const int64_t L = c->dt.num_leaves;
    int64_t v[12] = {0};
    if (c->leaf_planes) v[1] += L * wpad * (int64_t)sizeof(uint4) + L;   // code planes + flags
    if (c->leaf_present) v[1] += L * wpad * (int64_t)sizeof(uint32_t);
    v[2] = (int64_t)c->sub_planes_bytes;
    v[3] = (int64_t)c->sets_bytes;
    v[4] = (int64_t)(c->cmask_bytes + c->upm_bytes);   // (mask records + up slots)
    v[5] = (int64_t)c->sk_parts_bytes;
    if (c->recs) v[6] = c->shard_cap * pm::kShards * (int64_t)sizeof(pm_mut) + pm::kShards * 4;
    v[7] = (int64_t)c->tree_bytes;
    if (c->cons) v[8] = std::max<int64_t>(wpad, 4 * pm::kWave) * 16 + 2 * wpad * 16 + c->num_sites * 5;
    v[9] = (int64_t)c->rows_cap + (int64_t)c->text_cap + (int64_t)c->gather_bytes + (int64_t)c->finals_bytes;
    for (int k = 1; k < 10; ++k) v[0] += v[k];
    for (int k = 0; k < n && k < 10; ++k) out[k] = v[k];
    return PM_OK;
}

}  // extern "C"
