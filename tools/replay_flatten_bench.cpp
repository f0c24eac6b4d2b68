// Host-only timing of the FASTA replay's flattening (pm::replay_flatten) on a .panman file,
// and a checksum of everything it produces (to compare builds):
//   g++ -O2 -std=c++17 -Iinclude -Ipanman_amd/csrc -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
//       tools/replay_flatten_bench.cpp -Lpanman_amd -l:libpanman_amd.so -Wl,-rpath,panman_amd -o /tmp/rfb
//   /tmp/rfb file.panman [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "pm_replay.h"

template <class V>
static uint64_t mix(uint64_t h, const V& v) {
    const unsigned char* p = reinterpret_cast<const unsigned char*>(v.data());
    for (size_t i = 0; i < v.size() * sizeof(v[0]); ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    pm_panman* f = nullptr;
    char err[256] = {0};
    if (pm_panman_load(argv[1], &f, err, sizeof err) != PM_OK) {
        std::fprintf(stderr, "load: %s\n", err);
        return 1;
    }
    pm_panmat v;
    pm_panman_tree(f, 0, &v);
    for (int r = 0; r < reps; ++r) {
        pm::ReplayState st;
        pm::ReplayHost h;
        std::string msg;
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = pm::replay_flatten(&v, st, h, -1, -1, msg);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t x = 1469598103934665603ull;
        x = mix(x, h.cons_row); x = mix(x, h.presence); x = mix(x, h.eoff); x = mix(x, h.ecol); x = mix(x, h.echr);
        x = mix(x, h.tile2); x = mix(x, h.tile_blk); x = mix(x, h.path_off); x = mix(x, h.path_all);
        std::printf("rc %d %s  %.3f s  edits %lld columns %lld  hash %016llx\n", rc, msg.c_str(), s, (long long)st.edits,
                    (long long)st.columns, (unsigned long long)x);
    }
    std::string rep((size_t)pm_phase_report(nullptr, 0), '\0');
    pm_phase_report(&rep[0], (int64_t)rep.size());
    std::printf("%s", rep.c_str());
    pm_panman_free(f);
    return 0;
}
