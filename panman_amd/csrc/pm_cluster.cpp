// pm_cluster.cpp -- host schedule of the LDS-staged post-order sweeps (PM_OPT_CLUSTER).
//
// The post-order of the subtree form (Fitch, every leaf present) from level h0 up -- the
// levels of at most max_level nodes, where a level launch cannot fill the chip and each costs
// a chain of memory round trips -- runs in BANDS of consecutive levels.  Inside a band the
// materialised nodes fall into connected CLUSTERS (a cluster's root has its parent above the
// band).  One wave owns one (cluster, 64-word tile) and walks the cluster's nodes in STEPS,
// one node per step in depth-first post-order: a node's set goes to an LDS SLOT when its
// parent is in the cluster and is read from there at the parent's step, so the cluster's inner
// edges never go through memory (the sets still go to HBM as compressed records, which the
// pre-order reads, but nothing waits for those stores).  A wave's LDS accesses take effect in
// issue order: no barrier.  Every other input of a step (leaf words, earlier launches'
// records, the step's descriptor) is loaded one or two steps ahead (k_fitch_up_cluster).
// Reference semantics unchanged: src/fitchSankoff.cpp:30-56 per node, children combined
// commutatively.
//
// Order and slots: children first, the child with the most in-cluster nodes first (so a chain
// needs one slot: a node's step reads its child's slot and writes its own set there); a slot
// read at step e may be written again from step e on (the read comes first in the step).  A
// band grows level by level while every cluster fits kClSlots slots and kClMaxSteps steps and
// the band spans at most kClBandHeights levels (a one-level band always fits: its clusters are
// single nodes).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pm_internal.h"

namespace pm {

int plan_clusters(const HostTree& ht, const std::vector<int32_t>& up_order_k, const std::vector<int32_t>& child_enc_k,
                  const std::vector<int32_t>& parent_dense, const std::vector<int32_t>& vleaf, int32_t max_level,
                  bool chain_check, ClusterPlan& out) {
    out = ClusterPlan{};
    const int32_t I = (int32_t)ht.child_off.size() - 1;
    const int32_t H = (int32_t)ht.up_level_off_k.size() - 1;
    if (max_level <= 0 || H <= 0) return 0;
    // first level of the sweeps: every level from h0 up holds <= max_level nodes
    int32_t h0 = H;
    while (h0 > 0 && ht.up_level_off_k[h0] - ht.up_level_off_k[h0 - 1] <= max_level) --h0;
    out.h0 = h0;
    if (h0 >= H) return 0;
    std::vector<int32_t> level_of(I, -1);
    for (int32_t l = 0; l < H; ++l)
        for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) level_of[up_order_k[i]] = l;
    auto is_mat = [](int32_t x) { return x >= 0 && !(x & kVirtualBit); };

    out.slot_of.assign(I, -1);
    out.item_of.assign(I, -1);
    out.wg_off.assign(1, 0);
    out.band_wg.assign(1, 0);
    std::vector<int32_t> comp(I, -1), step_of(I, -1), slot(I, -1), size(I, 0);

    // One band [l0, l1): clusters, steps and slots; false when a cluster needs more than
    // kClSlots slots or kClMaxSteps steps.  `commit`: append the band's clusters to the plan.
    auto band = [&](int32_t l0, int32_t l1, bool commit) -> bool {
        auto in_band = [&](int32_t x) { return is_mat(x) && level_of[x] >= l0 && level_of[x] < l1; };
        // clusters, top-down: a node joins its parent's when the parent is in the band
        std::vector<int32_t> roots;
        for (int32_t l = l1 - 1; l >= l0; --l)
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) {
                const int32_t d = up_order_k[i];
                const int32_t p = parent_dense[d];
                if (p >= 0 && in_band(p)) {
                    comp[d] = comp[p];
                } else {
                    comp[d] = d;
                    roots.push_back(d);
                }
            }
        // in-cluster subtree sizes, bottom-up
        for (int32_t l = l0; l < l1; ++l)
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) {
                const int32_t d = up_order_k[i];
                int32_t s = 1;
                for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
                    if (in_band(child_enc_k[e])) s += size[child_enc_k[e]];
                size[d] = s;
            }
        // depth-first post-order of r's cluster into seq, the largest in-cluster child first
        struct Scratch {
            std::vector<int32_t> seq, kids;
            std::vector<std::pair<int32_t, int32_t>> stack;
        };
        auto order = [&](int32_t r, Scratch& w) {
            w.seq.clear();
            w.stack.assign(1, {r, 0});
            while (!w.stack.empty()) {
                const int32_t d = w.stack.back().first;
                if (w.stack.back().second == 0) {   // first visit: the children, the largest pushed last (popped first)
                    w.stack.back().second = 1;
                    w.kids.clear();
                    for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e)
                        if (in_band(child_enc_k[e])) w.kids.push_back(child_enc_k[e]);
                    std::sort(w.kids.begin(), w.kids.end(), [&](int32_t x, int32_t y) { return size[x] < size[y]; });
                    for (const int32_t k : w.kids) w.stack.push_back({k, 0});
                } else {
                    w.seq.push_back(d);
                    w.stack.pop_back();
                }
            }
        };
        for (const int32_t r : roots)
            if (size[r] > kClMaxSteps) return false;
        // steps and slots, clusters in parallel (each writes its own nodes' entries only)
        const int tasks = (int)std::min<size_t>(roots.size(), (size_t)4 * host_threads());
        std::atomic<bool> fits{true};
        host_parallel_for(tasks, [&](int t) {
            Scratch w;
            for (size_t k = (size_t)t; k < roots.size() && fits.load(std::memory_order_relaxed); k += (size_t)tasks) {
                order(roots[k], w);
                for (size_t j = 0; j < w.seq.size(); ++j) step_of[w.seq[j]] = (int32_t)j;
                // slots: [step(d), step(parent)] per in-cluster edge, coloured greedily by start
                int32_t busy_until[kClSlots];   // the step a slot is last read in
                for (int q = 0; q < kClSlots; ++q) busy_until[q] = -1;
                for (const int32_t d : w.seq) {   // (seq is in start order)
                    slot[d] = -1;
                    const int32_t p = parent_dense[d];
                    if (!(p >= 0 && in_band(p))) continue;
                    int q = 0;
                    while (q < kClSlots && busy_until[q] > step_of[d]) ++q;
                    if (q == kClSlots) {
                        fits = false;
                        return;
                    }
                    busy_until[q] = step_of[p];
                    slot[d] = q;
                }
            }
        });
        if (!fits) return false;
        if (!commit) return true;
        // longest clusters first (they bound the launch)
        std::vector<int32_t> wgs(roots);
        std::stable_sort(wgs.begin(), wgs.end(), [&](int32_t x, int32_t y) { return size[x] > size[y]; });
        const size_t base0 = out.items.size();
        std::vector<size_t> base(wgs.size() + 1, base0);
        for (size_t k = 0; k < wgs.size(); ++k) {
            base[k + 1] = base[k] + (size_t)size[wgs[k]];
            out.wg_off.push_back((int32_t)base[k + 1]);
            out.max_rounds = std::max(out.max_rounds, size[wgs[k]]);
        }
        out.items.resize(base.back());
        host_parallel_for(tasks, [&](int t) {
            Scratch w;
            for (size_t k = (size_t)t; k < wgs.size(); k += (size_t)tasks) {
                order(wgs[k], w);
                for (size_t j = 0; j < w.seq.size(); ++j) {
                    const int32_t d = w.seq[j];
                    NodeDesc& x = out.items[base[k] + j];
                    x = NodeDesc{};
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
                    x.pad0 = in_band(x.c0) ? slot[x.c0] : -1;
                    x.pad1 = x.e1 - x.e0 > 1 && in_band(x.c1) ? slot[x.c1] : -1;
                    out.item_of[d] = (int32_t)(base[k] + j);
                    out.slot_of[d] = slot[d];
                }
            }
        });
        out.band_wg.push_back((int32_t)out.wg_off.size() - 1);
        return true;
    };

    // Bands bottom-up, each as tall as fits (a taller band only merges clusters: binary search);
    // a band whose longest cluster has more than kClChain steps per level is bushy (a random-join
    // tree's: a wave walks its subtree node after node where the level kernels run a level's
    // nodes side by side) -- the sweeps then start above the last bushy band.
    std::vector<std::pair<int32_t, int32_t>> bands;
    int32_t start = 0;
    for (int32_t l0 = h0; l0 < H;) {
        int32_t lo = l0 + 1, hi = std::min(H, l0 + kClBandHeights);
        if (!band(l0, hi, false)) {
            while (hi - lo > 1) {   // band(l0, lo) fits, band(l0, hi) does not
                const int32_t mid = (lo + hi) / 2;
                if (band(l0, mid, false)) lo = mid;
                else hi = mid;
            }
            hi = lo;
            band(l0, hi, false);   // (its sizes)
        }
        int32_t longest = 0, roots = 0;
        for (int32_t l = l0; l < hi; ++l)
            for (int32_t i = ht.up_level_off_k[l]; i < ht.up_level_off_k[l + 1]; ++i) {
                const int32_t d = up_order_k[i];
                const int32_t p = parent_dense[d];
                if (!(p >= 0 && level_of[p] >= l0 && level_of[p] < hi)) {
                    longest = std::max(longest, size[d]);
                    ++roots;
                }
            }
        if (std::getenv("PM_CL_DEBUG"))
            std::fprintf(stderr, "band [%d, %d) longest %d clusters %d nodes %d\n", l0, hi, longest, roots,
                         ht.up_level_off_k[hi] - ht.up_level_off_k[l0]);
        bands.emplace_back(l0, hi);
        if (chain_check && (longest > kClChain * (hi - l0) || roots > kClMaxClusters)) start = (int32_t)bands.size();
        l0 = hi;
    }
    if (start >= (int32_t)bands.size()) {
        out.h0 = H;
        return 0;
    }
    h0 = out.h0 = bands[start].first;
    for (size_t k = start; k < bands.size(); ++k) {
        band(bands[k].first, bands[k].second, true);
        out.band_level.push_back(bands[k].first);
    }
    out.band_level.push_back(H);
    out.n_items = (int32_t)out.items.size();
    return 0;
}

}  // namespace pm

namespace pm {

// The pre-order over the same clusters (k_down_cluster): per cluster its nodes in depth-first
// pre-order (a node before its children, the child with the most in-cluster nodes last, so a
// chain holds one final at a time), the pre-order descriptor of each (the subtree form's:
// S2 / S3 children left to the tail launch) with pad0 = the LDS slot holding the parent's
// final (-1: the parent is outside the cluster, its final in memory) and pad1 = the slot this
// node's final goes to (-1: no child in the cluster).  A final occupies its slot from its
// node's step to its last in-cluster child's.  False (no pre-order sweeps) when a cluster needs
// more than kClFSlots slots.
bool plan_cluster_down(const HostTree& ht, const std::vector<int32_t>& down_order_k, const std::vector<NodeDesc>& down_desc_k,
                       const std::vector<int32_t>& child_enc_k, ClusterPlan& cl) {
    cl.down_items.clear();
    if (cl.wg_off.size() < 2 || cl.h0 != 0) return false;   // (every level swept: the pre-order runs the clusters only)
    const int32_t I = (int32_t)ht.child_off.size() - 1;
    std::vector<int32_t> pos(I, -1);
    for (size_t k = 0; k < down_order_k.size(); ++k) pos[down_order_k[k]] = (int32_t)k;
    cl.down_items.assign(cl.items.size(), NodeDesc{});
    const int32_t W = (int32_t)cl.wg_off.size() - 1;
    std::atomic<bool> ok{true};
    const int tasks = std::min(W, 4 * host_threads());
    host_parallel_for(tasks, [&](int t) {
        std::vector<int32_t> size, step, seq, stack, kids, slot;
        for (int32_t w = t; w < W && ok; w += tasks) {
            const int32_t lo = cl.wg_off[w], hi = cl.wg_off[w + 1], n = hi - lo;
            auto local = [&](int32_t x) {   // x's position in the cluster's post-order items, or -1
                if (x < 0 || (x & kVirtualBit)) return -1;
                const int32_t it = cl.item_of[x];
                return it >= lo && it < hi ? it - lo : -1;
            };
            size.assign(n, 1);
            for (int32_t j = 0; j < n; ++j) {   // (post-order: children first)
                const int32_t d = cl.items[lo + j].node;
                for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e) {
                    const int32_t c = local(child_enc_k[e]);
                    if (c >= 0) size[j] += size[c];
                }
            }
            seq.clear();
            stack.assign(1, n - 1);   // the root: the last post-order item
            while (!stack.empty()) {
                const int32_t j = stack.back();
                stack.pop_back();
                seq.push_back(j);
                const int32_t d = cl.items[lo + j].node;
                kids.clear();
                for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e) {
                    const int32_t c = local(child_enc_k[e]);
                    if (c >= 0) kids.push_back(c);
                }
                std::sort(kids.begin(), kids.end(), [&](int32_t x, int32_t y) { return size[x] > size[y]; });
                for (const int32_t c : kids) stack.push_back(c);   // (the largest pushed first: popped last)
            }
            step.assign(n, 0);
            for (int32_t s = 0; s < n; ++s) step[seq[s]] = s;
            // final slots: [step(d), the last in-cluster child's step]
            slot.assign(n, -1);
            int32_t busy_until[kClFSlots];
            for (int q = 0; q < kClFSlots; ++q) busy_until[q] = -1;
            for (int32_t s = 0; s < n; ++s) {
                const int32_t j = seq[s];
                const int32_t d = cl.items[lo + j].node;
                int32_t last = -1;
                for (int32_t e = ht.child_off[d]; e < ht.child_off[d + 1]; ++e) {
                    const int32_t c = local(child_enc_k[e]);
                    if (c >= 0) last = std::max(last, step[c]);
                }
                if (last < 0) continue;
                int q = 0;
                while (q < kClFSlots && busy_until[q] > s) ++q;
                if (q == kClFSlots) {
                    ok = false;
                    return;
                }
                busy_until[q] = last;
                slot[j] = q;
            }
            for (int32_t s = 0; s < n; ++s) {
                const int32_t j = seq[s];
                const int32_t d = cl.items[lo + j].node;
                NodeDesc x = down_desc_k[pos[d]];
                const int32_t pj = x.parent >= 0 ? local(x.parent) : -1;
                x.pad0 = pj >= 0 ? slot[pj] : -1;
                x.pad1 = slot[j];
                cl.down_items[lo + s] = x;
            }
        }
    });
    if (!ok) cl.down_items.clear();
    return ok;
}

}  // namespace pm
