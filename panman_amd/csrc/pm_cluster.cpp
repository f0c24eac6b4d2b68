// pm_cluster.cpp -- host schedule of the LDS-staged post-order sweeps (PM_OPT_CLUSTER).
//
// The post-order of the subtree form (Fitch, every leaf present) above a height h0 runs in
// BANDS of consecutive heights.  Inside a band the materialised nodes fall into connected
// CLUSTERS (a cluster's root has its parent above the band); one workgroup of kClWaves waves
// owns one (cluster, 64-word tile) and walks the cluster's heights bottom-up in ROUNDS of at
// most kClWaves nodes (a node of out-degree > 3 takes a round of its own, its children dealt
// to every wave), a workgroup barrier between rounds.  A node whose parent is in the same
// cluster keeps its 16-plane set in an LDS SLOT from the round that computes it to the round
// of its parent, so the cluster's inner edges never go through memory: the sets still go to
// HBM as compressed records (the pre-order reads them), but nothing waits for those stores.
// Reference semantics unchanged: src/fitchSankoff.cpp:30-56 per node, children combined
// commutatively.
//
// Slots: interval colouring over rounds -- a set occupies its slot from the round that writes
// it to the round that reads it, inclusive (a slot read in round r is reused by a set written
// in round r + 1 or later, never by one written in round r: the waves of a round run
// concurrently).  A band grows height by height while every cluster fits kClSlots slots and
// the band spans at most kClBandHeights heights.
#include <algorithm>
#include <vector>

#include "pm_internal.h"

namespace pm {

namespace {

struct BandNodes {
    std::vector<int32_t> nodes;   // materialised nodes of the band, descending height
};

}  // namespace

// Heights are the post-order levels of the subtree form (up_level_off_k: level l = height
// l + 1, S2 / S3 and virtual nodes removed).
int plan_clusters(const HostTree& ht, const std::vector<int32_t>& up_order_k, const std::vector<int32_t>& child_enc_k,
                  const std::vector<int32_t>& parent_dense, const std::vector<int32_t>& vleaf, int32_t max_level,
                  ClusterPlan& out) {
    out = ClusterPlan{};
    const int32_t I = (int32_t)ht.child_off.size() - 1;
    const int32_t H = (int32_t)ht.up_level_off_k.size() - 1;
    if (max_level <= 0 || H <= 0) return 0;
    // first level of the cluster range: every level from h0 up holds <= max_level nodes
    int32_t h0 = H;
    while (h0 > 0 && ht.up_level_off_k[h0] - ht.up_level_off_k[h0 - 1] <= max_level) --h0;
    out.h0 = h0;
    if (h0 >= H) return 0;
    std::vector<int32_t> level_of(I, -1);
    for (int32_t l = 0; l < H; ++l)
        for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) level_of[up_order_k[i]] = l;
    auto is_mat = [](int32_t x) { return x >= 0 && !(x & kVirtualBit); };
    auto wide = [&](int32_t d) { return ht.child_off[d + 1] - ht.child_off[d] > 3; };

    out.slot_of.assign(I, -1);
    out.wg_off.assign(1, 0);
    out.band_wg.assign(1, 0);
    std::vector<int32_t> comp(I, -1), round_of(I, -1), slot(I, -1);

    // One band [l0, l1): clusters, rounds and slots; false when a cluster needs more than
    // kClSlots slots.  `commit`: append the band's workgroups and items to the plan.
    auto band = [&](int32_t l0, int32_t l1, bool commit) -> bool {
        // clusters: top-down (descending level), a node joins its parent's cluster when the
        // parent is in the band
        std::vector<int32_t> roots;
        for (int32_t l = l1 - 1; l >= l0; --l)
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) {
                const int32_t d = up_order_k[i];
                const int32_t p = parent_dense[d];
                if (p >= 0 && level_of[p] >= l0 && level_of[p] < l1) {
                    comp[d] = comp[p];
                } else {
                    comp[d] = d;
                    roots.push_back(d);
                }
            }
        // members by level, bottom-up: bucket every band node under its cluster root
        std::vector<int32_t> ridx(I, -1);
        for (size_t k = 0; k < roots.size(); ++k) ridx[roots[k]] = (int32_t)k;
        std::vector<int32_t> cnt(roots.size() + 1, 0);
        for (int32_t l = l0; l < l1; ++l)
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) ++cnt[ridx[comp[up_order_k[i]]] + 1];
        for (size_t k = 0; k < roots.size(); ++k) cnt[k + 1] += cnt[k];
        std::vector<int32_t> mem(cnt.back()), cur(cnt.begin(), cnt.end() - 1);
        for (int32_t l = l0; l < l1; ++l)   // ascending level inside each cluster
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) {
                const int32_t d = up_order_k[i];
                mem[cur[ridx[comp[d]]]++] = d;
            }
        struct Wg {
            int32_t begin, end, rounds;
        };
        std::vector<Wg> wgs(roots.size());
        for (size_t k = 0; k < roots.size(); ++k) {
            // rounds: per level, the narrow nodes kClWaves at a time, then each wide node alone
            int32_t r = 0;
            for (int32_t a = cnt[k]; a < cnt[k + 1];) {
                const int32_t l = level_of[mem[a]];
                int32_t b = a;
                while (b < cnt[k + 1] && level_of[mem[b]] == l) ++b;
                int32_t narrow = 0;
                for (int32_t j = a; j < b; ++j)
                    if (!wide(mem[j])) round_of[mem[j]] = r + narrow++ / kClWaves;
                r += (narrow + kClWaves - 1) / kClWaves;
                for (int32_t j = a; j < b; ++j)
                    if (wide(mem[j])) round_of[mem[j]] = r++;
                a = b;
            }
            wgs[k] = Wg{cnt[k], cnt[k + 1], r};
            // slots: intervals [round_of[d], round_of[parent]] of the nodes whose parent is in
            // the cluster, coloured greedily in round order (interval graphs: optimal)
            std::vector<std::pair<int32_t, int32_t>> iv;   // (start round, node)
            for (int32_t j = cnt[k]; j < cnt[k + 1]; ++j) {
                const int32_t d = mem[j];
                const int32_t p = parent_dense[d];
                slot[d] = -1;
                if (p >= 0 && comp[p] == comp[d]) iv.emplace_back(round_of[d], d);
            }
            std::sort(iv.begin(), iv.end());
            int32_t busy_until[kClSlots];   // last round a slot is read in
            for (int s = 0; s < kClSlots; ++s) busy_until[s] = -1;
            for (const auto& x : iv) {
                const int32_t d = x.second, start = x.first, end = round_of[parent_dense[d]];
                int s = 0;
                while (s < kClSlots && busy_until[s] >= start) ++s;
                if (s == kClSlots) return false;
                busy_until[s] = end;
                slot[d] = s;
            }
        }
        if (!commit) return true;
        // longest clusters first (they bound the launch), items in rounds of kClWaves
        std::vector<int32_t> order(roots.size());
        for (size_t k = 0; k < order.size(); ++k) order[k] = (int32_t)k;
        std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return wgs[x].rounds > wgs[y].rounds; });
        for (const int32_t k : order) {
            const Wg& w = wgs[k];
            const size_t base = out.items.size();
            out.items.resize(base + (size_t)w.rounds * kClWaves);
            for (size_t q = base; q < out.items.size(); ++q) {
                out.items[q] = NodeDesc{};
                out.items[q].node = -1;
            }
            std::vector<int32_t> fill(w.rounds, 0);
            for (int32_t j = w.begin; j < w.end; ++j) {
                const int32_t d = mem[j];
                const int32_t r = round_of[d];
                NodeDesc& x = out.items[base + (size_t)r * kClWaves + fill[r]++];
                x.node = d;
                x.e0 = ht.child_off[d];
                x.e1 = ht.child_off[d + 1];
                x.c0 = child_enc_k[x.e0];
                x.c1 = x.e1 - x.e0 > 1 ? child_enc_k[x.e0 + 1] : 0;
                for (int q = 0; q < 4; ++q) {
                    x.vl0[q] = x.c0 >= 0 && (x.c0 & kVirtualBit) ? vleaf[(size_t)(x.c0 & kDenseMask) * 4 + q] : -1;
                    x.vl1[q] = x.e1 - x.e0 > 1 && x.c1 >= 0 && (x.c1 & kVirtualBit)
                                   ? vleaf[(size_t)(x.c1 & kDenseMask) * 4 + q] : -1;
                }
                // parent: this node's LDS slot (or -1); pad0 / pad1: the first two children's
                x.parent = slot[d];
                x.pad0 = is_mat(x.c0) && comp[x.c0] == comp[d] && level_of[x.c0] >= l0 ? slot[x.c0] : -1;
                x.pad1 = x.e1 - x.e0 > 1 && is_mat(x.c1) && comp[x.c1] == comp[d] && level_of[x.c1] >= l0 ? slot[x.c1] : -1;
                if (wide(d))   // every wave of the round takes a share of the children
                    for (int w2 = 1; w2 < kClWaves; ++w2) out.items[base + (size_t)r * kClWaves + w2] = x;
                out.slot_of[d] = slot[d];
            }
            out.wg_off.push_back((int32_t)out.items.size());
            out.max_rounds = std::max(out.max_rounds, w.rounds);
        }
        out.band_wg.push_back((int32_t)out.wg_off.size() - 1);
        return true;
    };

    for (int32_t l0 = h0; l0 < H;) {
        int32_t l1 = std::min(H, l0 + kClBandHeights);
        while (l1 > l0 + 1 && !band(l0, l1, false)) --l1;   // (a one-level band needs no slot)
        band(l0, l1, true);
        out.band_level.push_back(l0);
        l0 = l1;
    }
    out.band_level.push_back(H);
    return 0;
}

}  // namespace pm
