// pm_reroot.cpp -- Tree::reroot (src/reroot.cpp:4-262) with the parsimony on the GPU.
//
//   1. every leaf's sequence (getSequenceFromReference, src/panman.cpp:4676-5000, no
//      rotation): the replay kernels build all canonical rows in HBM at once;
//   2. transform / transformHelper (src/panman.cpp:5831-5906): host, on parent arrays;
//   3. block Fitch per block id (src/reroot.cpp:53-125): PM_MODE_BLOCK_FITCH, root forced
//      to the new root's block state, root parent state 1;
//   4. nucleotide Fitch per canonical column (main positions and gap slots,
//      src/reroot.cpp:130-226): the rows are converted to packed codes on the device
//      ('-' and 'x' are state 1) and fed to the Fitch kernels in column chunks with the root
//      forced to the new root's characters; the root's parent state is the block
//      consensus for main columns and a gap for gap slots;
//   5. grouping into NucMut runs (src/reroot.cpp:228-262) on the host.
// The result is an owned tree (pm_panman) in the pre-order of the new topology.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "pm_internal.h"
#include "pm_newick.h"
#include "pm_panman_tree.h"
#include "pm_replay.h"

namespace pm {
namespace {

uint8_t code_of(char ch) {
    switch (ch) {
        case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
        case 'R': return 5;  case 'Y': return 10; case 'S': return 6;  case 'W': return 9;
        case 'K': return 12; case 'M': return 3;  case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7;  case 'N': return 15;
        default: return 0;   // '-', the 'x' sentinel: state 1
    }
}

struct Shape {   // the reference's in-memory tree after transform, indexed by old id (+ new root)
    std::vector<std::string> name;
    std::vector<std::vector<int32_t>> kids;
    std::vector<int32_t> parent;
    std::vector<float> len;
    std::vector<char> alive;
    int32_t root = -1;
};

// transform(leaf) and transformHelper (src/panman.cpp:5831-5906), iteratively.
bool transform(Shape& t, int32_t leaf, int64_t internal_nodes, std::string& err) {
    const int32_t par = t.parent[leaf];
    if (par < 0) return true;                 // already the root
    if (par == t.root) {                      // the root keeps the leaf's sequence
        t.len[leaf] = 0;
        return true;
    }
    auto erase = [&](int32_t from, int32_t child) {
        auto& k = t.kids[from];
        k.erase(std::find(k.begin(), k.end(), child));
    };
    erase(par, leaf);
    t.parent[leaf] = -1;
    const float leaf_len = t.len[leaf];
    const int32_t nr = (int32_t)t.name.size();
    t.name.push_back("node_" + std::to_string(internal_nodes + 1));   // newInternalNodeId()
    t.kids.push_back({leaf});
    t.parent.push_back(-1);
    t.len.push_back(0);
    t.alive.push_back(1);
    t.parent[leaf] = nr;
    t.len[leaf] = 0;
    // transformHelper(par): chain par = v0 -> v1 -> ... -> vk = old root
    std::vector<int32_t> chain{par};
    while (chain.back() != t.root) chain.push_back(t.parent[chain.back()]);
    const size_t k = chain.size() - 1;
    std::vector<float> old_len(k);
    for (size_t j = 0; j < k; ++j) {
        erase(chain[j + 1], chain[j]);
        t.parent[chain[j]] = -1;
        old_len[j] = t.len[chain[j]];
        t.len[chain[j]] = 0;
    }
    int32_t top;   // what helper(old root) returns
    const int32_t old_root = chain[k];
    if (t.kids[old_root].size() > 1) {
        t.len[old_root] = 0;
        top = old_root;
    } else if (t.kids[old_root].size() == 1) {
        top = t.kids[old_root][0];
        t.len[top] = 0;
        t.alive[old_root] = 0;   // deleted and erased from allNodes
        t.kids[old_root].clear();
    } else {
        err = "the old root has no child left after rerooting (unary root)";
        return false;
    }
    for (size_t j = k; j-- > 0;) {
        const int32_t c = j + 1 == k ? top : chain[j + 1];
        t.kids[chain[j]].push_back(c);
        t.parent[c] = chain[j];
        t.len[c] = old_len[j];
    }
    t.kids[nr].push_back(par);
    t.parent[par] = nr;
    t.len[par] = leaf_len;
    t.root = nr;
    return true;
}

struct Tup {
    int32_t block, pos, gap;
    uint8_t type, code;
};

// NucMut runs (src/reroot.cpp:228-262): at most 6, same block, consecutive positions (main)
// or consecutive slots of one position (gap), same type; tuples arrive sorted.
void group(const std::vector<Tup>& v, bool gap, PanmanTree& out) {
    size_t start = 0;
    auto emit = [&](size_t a, size_t b) {
        uint32_t nucs = 0;
        for (size_t i = a; i < b; ++i) nucs |= (uint32_t)v[i].code << (4 * (5 - (i - a)));
        out.nm_primary.push_back(v[a].block);
        out.nm_secondary.push_back(-1);
        out.nm_pos.push_back(v[a].pos);
        out.nm_gap.push_back(gap ? v[a].gap : -1);
        out.nm_info.push_back((uint8_t)(((b - a) << 4) + v[a].type));
        out.nm_nucs.push_back(nucs);
    };
    for (size_t i = 1; i < v.size(); ++i) {
        const Tup& p = v[i - 1];
        const Tup& q = v[i];
        const bool brk = i - start == 6 || q.block != p.block || q.type != p.type ||
                         (gap ? (q.pos != p.pos || q.gap != p.gap + 1) : q.pos != p.pos + 1);
        if (brk) {
            emit(start, i);
            start = i;
        }
    }
    if (!v.empty()) emit(start, v.size());
}

void pack(const std::vector<uint8_t>& codes, std::vector<uint8_t>& out) {
    out.assign((codes.size() + 1) / 2, 0);
    for (size_t s = 0; s < codes.size(); ++s) out[s / 2] |= (uint8_t)(codes[s] << (4 * (s & 1)));
}

int fetch(pm_ctx* c, std::vector<pm_mut>& recs) {
    int64_t n = 0;
    int rc = pm_mutation_count(c, &n);
    if (rc != PM_OK) return rc;
    recs.resize((size_t)n);
    return n ? pm_mutations_fetch(c, recs.data(), n, &n) : PM_OK;
}

int reroot(pm_ctx* c, const pm_panmat* p, const std::string& leaf_name, PanmanTree& out) {
    const int32_t N = p->num_nodes;
    if (N < 2 || !p->names || !p->child_offsets) return fail(c, PM_ERR_ARG, "bad PanMAT topology");
    Shape t;
    t.name.resize(N);
    const char* nm = p->names;
    for (int32_t i = 0; i < N; ++i) {
        t.name[i] = nm;
        nm += t.name[i].size() + 1;
    }
    t.kids.assign(N, {});
    t.parent.assign(N, -1);
    t.alive.assign(N, 1);
    t.len.assign(N, 1.0f);
    if (p->branch_length) t.len.assign(p->branch_length, p->branch_length + N);
    int64_t internal = 0;
    for (int32_t i = 0; i < N; ++i) {
        for (int32_t e = p->child_offsets[i]; e < p->child_offsets[i + 1]; ++e) {
            t.kids[i].push_back(p->child_index[e]);
            t.parent[p->child_index[e]] = i;
        }
        internal += !t.kids[i].empty();
    }
    t.root = p->root;
    int32_t leaf = -1;
    for (int32_t i = 0; i < N && leaf < 0; ++i)
        if (t.name[i] == leaf_name) leaf = i;
    if (leaf < 0) return fail(c, PM_ERR_ARG, "Sequence with name " + leaf_name + " not found!");
    if (!t.kids[leaf].empty()) return fail(c, PM_ERR_ARG, "Node with id " + leaf_name + " is not a tip!");
    if (p->nuc_mut_secondary)
        for (int64_t k = 0; k < p->nuc_mut_offsets[N]; ++k)
            if (p->nuc_mut_secondary[k] != -1) return fail(c, PM_ERR_UNSUPPORTED, "secondary blocks");

    // 1. all leaf sequences (R4) on the device
    free_replay(c);
    c->replay = new ReplayState();
    ReplayState& r = *c->replay;
    int rc = replay_prepare(c, p, r);
    if (rc != PM_OK) return rc;
    for (int32_t id = 0; id <= r.max_id; ++id)
        if (!r.is_block[id])
            return fail(c, PM_ERR_ARG, "Block with id " + std::to_string(id) + " -1 not found!");
    hipError_t e = launch_replay(c, r.dev);
    if (e != hipSuccess) return hip_fail(c, e, "replay launch");
    r.ran = true;
    std::vector<int32_t> li_of(N, -1);
    for (size_t li = 0; li < r.leaves.size(); ++li) li_of[r.leaves[li]] = (int32_t)li;
    const int32_t L = (int32_t)r.leaves.size();
    const int32_t root_li = li_of[leaf];

    // 2. topology
    std::string err;
    if (!transform(t, leaf, internal, err)) return fail(c, PM_ERR_UNSUPPORTED, err);
    std::vector<int32_t> order;   // new id -> old id (pre-order)
    std::vector<int32_t> st{t.root};
    while (!st.empty()) {
        const int32_t v = st.back();
        st.pop_back();
        order.push_back(v);
        for (size_t j = t.kids[v].size(); j-- > 0;) st.push_back(t.kids[v][j]);
    }
    const int32_t M = (int32_t)order.size();
    std::vector<int32_t> new_of((size_t)t.name.size(), -1);
    for (int32_t v = 0; v < M; ++v) new_of[order[v]] = v;
    Topology topo;
    topo.root = 0;
    out.num_nodes = M;
    out.root = 0;
    out.child_off.assign(M + 1, 0);
    for (int32_t v = 0; v < M; ++v) {
        const int32_t o = order[v];
        topo.name.push_back(t.name[o]);
        topo.length.push_back(t.len[o]);
        topo.kids.emplace_back();
        for (int32_t ch : t.kids[o]) {
            topo.kids[v].push_back(new_of[ch]);
            out.child_idx.push_back(new_of[ch]);
        }
        out.child_off[v + 1] = (int32_t)out.child_idx.size();
        out.names_blob += t.name[o];
        out.names_blob.push_back('\0');
    }
    out.length = topo.length;
    out.newick = newick_of(topo);
    std::vector<int32_t> node_row(M, -1);
    for (int32_t v = 0; v < M; ++v)
        if (topo.kids[v].empty()) node_row[v] = order[v] < N ? li_of[order[v]] : -1;
    pm_tree tree{M, 0, out.child_off.data(), out.child_idx.data()};
    if ((rc = pm_tree_upload(c, &tree)) != PM_OK) return rc;

    // 3. block mutations
    const int32_t B = r.max_id + 1;
    const int64_t bstride = (B + 1) / 2;
    std::vector<uint8_t> bcodes((size_t)L * bstride, 0), col(B), packed_cons, packed_forced;
    auto block_code = [&](int32_t li, int32_t id) -> uint8_t {
        return r.exists[li][id] ? (r.strand[li][id] ? 1 : 2) : 0;   // states 1 / 2 / 4
    };
    for (int32_t li = 0; li < L; ++li)
        for (int32_t id = 0; id < B; ++id) bcodes[(size_t)li * bstride + id / 2] |= block_code(li, id) << (4 * (id & 1));
    pack(std::vector<uint8_t>(B, 0), packed_cons);
    for (int32_t id = 0; id < B; ++id) col[id] = block_code(root_li, id);
    pack(col, packed_forced);
    std::vector<pm_mut> recs;
    if ((rc = pm_leaves_upload(c, B, bcodes.data(), bstride, node_row.data(), nullptr, 0)) != PM_OK ||
        (rc = pm_sites_upload(c, packed_cons.data(), packed_forced.data())) != PM_OK ||
        (rc = pm_run(c, PM_MODE_BLOCK_FITCH)) != PM_OK || (rc = fetch(c, recs)) != PM_OK)
        return rc;
    std::vector<std::vector<std::pair<int32_t, uint8_t>>> bmuts(M);   // (block, type<<4|code)
    for (const pm_mut& m : recs) bmuts[m.node].emplace_back((int32_t)(m.site_info >> 8), (uint8_t)(m.site_info & 0xFF));

    // 4. nucleotide mutations over the canonical columns, in chunks
    const int64_t C = r.columns;
    std::vector<int32_t> col_block(C), col_pos(C), col_gap(C);
    for (int32_t id = 0; id < B; ++id)
        for (size_t j = 0; j < r.main_col[id].size(); ++j) {
            const int64_t g0 = r.gap_col[id][j];
            for (int32_t w = 0; w < r.slots[id][j]; ++w) {
                col_block[g0 + w] = id;
                col_pos[g0 + w] = (int32_t)j;
                col_gap[g0 + w] = w;
            }
            col_block[r.main_col[id][j]] = id;
            col_pos[r.main_col[id][j]] = (int32_t)j;
            col_gap[r.main_col[id][j]] = -1;
        }
    std::vector<char> root_row(C);
    e = hipMemcpyAsync(root_row.data(), r.d_rows + (size_t)root_li * r.dev.row_stride, C, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "root row download");
    const int64_t budget = (int64_t)24 << 30;   // device bytes for sets / finals / codes per chunk
    const int64_t per_col = 3 * (int64_t)M + L + 64;
    const int64_t chunk = std::max<int64_t>(1 << 16, std::min<int64_t>(((int64_t)1 << 24) - 4096, budget / per_col));
    const int64_t cstride = (std::min(chunk, C) + 1) / 2 + 15 & ~(int64_t)15;
    uint8_t* d_codes = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&d_codes), (size_t)std::max(L, 1) * cstride)) != hipSuccess)
        return fail(c, PM_ERR_OOM, "reroot code staging");
    std::vector<std::vector<Tup>> main_t(M), gap_t(M);
    std::vector<uint8_t> cons_codes, forced_codes;
    for (int64_t c0 = 0; c0 < C && rc == PM_OK; c0 += chunk) {
        const int64_t n = std::min(chunk, C - c0);
        e = launch_rows_to_codes(c, r.d_rows, r.dev.row_stride, L, c0, n, d_codes, cstride);
        if (e != hipSuccess) {
            rc = hip_fail(c, e, "rows to codes");
            break;
        }
        if ((rc = leaves_install(c, n, d_codes, cstride, node_row.data())) != PM_OK) break;
        cons_codes.resize(n);
        forced_codes.resize(n);
        for (int64_t s = 0; s < n; ++s) {
            cons_codes[s] = code_of(r.cons[c0 + s]);      // main: consensus (sentinel: '-'); gap: 1
            forced_codes[s] = code_of(root_row[c0 + s]);
        }
        pack(cons_codes, packed_cons);
        pack(forced_codes, packed_forced);
        if ((rc = pm_sites_upload(c, packed_cons.data(), packed_forced.data())) != PM_OK ||
            (rc = pm_run(c, PM_MODE_FITCH)) != PM_OK || (rc = fetch(c, recs)) != PM_OK)
            break;
        for (const pm_mut& m : recs) {
            const int64_t cc = c0 + (m.site_info >> 8);
            const Tup tu{col_block[cc], col_pos[cc], col_gap[cc], (uint8_t)((m.site_info >> 4) & 15),
                         (uint8_t)(m.site_info & 15)};
            (tu.gap < 0 ? main_t : gap_t)[m.node].push_back(tu);
        }
    }
    (void)hipFree(d_codes);
    if (rc != PM_OK) return rc;

    // 5. the new tree's arrays
    out.block_primary.assign(p->block_primary, p->block_primary + p->num_blocks);
    out.block_seq_off.assign(p->block_seq_offsets, p->block_seq_offsets + p->num_blocks + 1);
    out.block_seq.assign(p->block_seq, p->block_seq + p->block_seq_offsets[p->num_blocks]);
    out.gap_primary.assign(p->gap_primary, p->gap_primary + p->num_gaps);
    out.gap_off.assign(p->gap_offsets, p->gap_offsets + p->num_gaps + 1);
    out.gap_pos.assign(p->gap_position, p->gap_position + p->gap_offsets[p->num_gaps]);
    out.gap_len.assign(p->gap_length, p->gap_length + p->gap_offsets[p->num_gaps]);
    out.bm_off.assign(M + 1, 0);
    out.nm_off.assign(M + 1, 0);
    for (int32_t v = 0; v < M; ++v) {
        for (auto& bm : bmuts[v]) {   // sorted by block id (the reference's order is TBB-scheduled)
            const int type = bm.second >> 4, code = bm.second & 15;
            out.bm_primary.push_back(bm.first);
            out.bm_info.push_back(type == PM_MUT_NI ? 1 : 0);
            out.bm_inv.push_back(type == PM_MUT_NI ? code == 2 : type == PM_MUT_NS);
        }
        out.bm_off[v + 1] = (int64_t)out.bm_primary.size();
        group(main_t[v], false, out);   // nonGapMutations first, then gapMutations
        group(gap_t[v], true, out);
        out.nm_off[v + 1] = (int64_t)out.nm_primary.size();
    }
    out.circular.assign(M, -1);
    out.rotation.assign(M, 0);
    out.inverted.assign(M, 0);
    for (int32_t v = 0; v < M; ++v) {
        const int32_t o = order[v];
        if (o >= N) continue;
        if (p->circular_offset) out.circular[v] = p->circular_offset[o];
        if (p->rotation_index) out.rotation[v] = p->rotation_index[o];
        if (p->sequence_inverted) out.inverted[v] = p->sequence_inverted[o];
    }
    return PM_OK;
}

}  // namespace
}  // namespace pm

extern "C" int pm_reroot(pm_ctx* c, const pm_panmat* p, const char* leaf, pm_panman** out) {
    if (!c || !p || !leaf || !out) return PM_ERR_ARG;
    *out = nullptr;
    (void)hipSetDevice(c->device);
    auto* res = new pm_panman();
    res->trees.resize(1);
    const int rc = pm::reroot(c, p, leaf, res->trees[0]);
    if (rc != PM_OK) {
        delete res;
        return rc;
    }
    *out = res;
    return PM_OK;
}
