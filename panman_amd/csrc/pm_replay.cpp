// pm_replay.cpp -- host side of FASTA replay: flatten a PanMAT for the GPU and format
// the replayed rows as the reference prints them.
//
// Reference: Tree::printFASTAUltraFast (src/fasta.cpp:1981-2099), getBlockSequence
// (:1766-1787), printFASTAUltraFastHelper (:1789-1979), printSequenceLinesNew (:155-254),
// getComplementCharacter (src/panman.cpp:171-204).
//
// Canonical row of a leaf: blocks in primary-id order; inside a block, for each position
// j = 0..len (len = the sentinel 'x'): its gap slots, then its main character.  The GPU
// fills every leaf's row from the consensus and applies path mutations; the formatter
// walks blocks in print order (rotation, inversion), forward or reverse-complemented,
// drops '-' (unaligned) and the 'x' sentinels, rotates by the circular offset and wraps
// at 70 columns.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "pm_replay.h"

namespace pm {

namespace {

char nuc_char(int code) {
    static const char tab[16] = {'-', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
    return tab[code & 15];
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

template <class T>
hipError_t dput(T** dst, const std::vector<T>& v, hipStream_t s) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), sizeof(T) * std::max<size_t>(v.size(), 1));
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s);
}

}  // namespace


namespace {

struct FlatErr {
    int code = PM_OK;
    std::string msg;
    int set(int c, const char* m) {
        code = c;
        msg = m;
        return c;
    }
};

}  // namespace

// The host half of replay_prepare: canonical columns, per-node edits, per-leaf block state.
// Per-node edit lists are independent and built by host threads (a C5 PanMAT carries ~18 M
// edits); everything else is linear in blocks, nodes or leaves.
int replay_flatten(const pm_panmat* p, ReplayState& r, ReplayHost& h, int64_t leaf_begin, int64_t leaf_end,
                   std::string& err_msg) {
    FlatErr ferr;
    PhaseClock clock;
    auto fail_ = [&](int code, const char* msg) {
        err_msg = msg;
        return code;
    };
    const int32_t N = p->num_nodes;
    if (N < 1 || p->root < 0 || p->root >= N || !p->child_offsets || !p->names)
        return fail_(PM_ERR_ARG, "bad PanMAT topology");
    r.num_nodes = N;
    r.names.resize(N);
    const char* nm = p->names;
    for (int32_t i = 0; i < N; ++i) {
        r.names[i] = nm;
        nm += r.names[i].size() + 1;
    }
    r.parent.assign(N, -2);
    r.parent[p->root] = -1;
    for (int32_t i = 0; i < N; ++i)
        for (int32_t e = p->child_offsets[i]; e < p->child_offsets[i + 1]; ++e) {
            const int32_t ch = p->child_index[e];
            if (ch < 0 || ch >= N || r.parent[ch] != -2) return fail_(PM_ERR_ARG, "bad child index");
            r.parent[ch] = i;
        }
    for (int32_t i = 0; i < N; ++i) {
        if (r.parent[i] == -2) return fail_(PM_ERR_ARG, "node unreachable from the root");
        if (p->child_offsets[i] == p->child_offsets[i + 1]) r.leaves.push_back(i);
    }
    if (leaf_begin >= 0 || leaf_end >= 0) {   // a shard of the leaves
        if (leaf_begin < 0 || leaf_end < leaf_begin || leaf_end > (int64_t)r.leaves.size())
            return fail_(PM_ERR_ARG, "leaf range outside [0, leaves]");
        r.leaves = std::vector<int32_t>(r.leaves.begin() + leaf_begin, r.leaves.begin() + leaf_end);
    }

    // ---- blocks (vector order defines blockLengths resets; ids must be unique)
    const int32_t B = p->num_blocks;
    for (int32_t b = 0; b < B; ++b) r.max_id = std::max(r.max_id, p->block_primary[b]);
    if (B == 0) return fail_(PM_ERR_ARG, "PanMAT has no blocks");
    const int32_t M = r.max_id + 1;
    r.is_block.assign(M, 0);
    std::vector<int32_t> len(M, 0);
    std::vector<int32_t> blk_of(M, -1);
    for (int32_t b = 0; b < B; ++b) {
        const int32_t id = p->block_primary[b];
        if (id < 0 || r.is_block[id]) return fail_(PM_ERR_UNSUPPORTED, "duplicate or negative primary block id");
        r.is_block[id] = 1;
        blk_of[id] = b;
        int32_t n = 0;
        bool end = false;
        for (int64_t w = p->block_seq_offsets[b]; w < p->block_seq_offsets[b + 1] && !end; ++w)
            for (int k = 0; k < 8; ++k) {
                if (((p->block_seq[w] >> (4 * (7 - k))) & 15) == 0) { end = true; break; }
                ++n;
            }
        len[id] = n;
    }
    // gap slots: resize semantics (last entry wins) for present blocks; absent blocks
    // accumulate every listed length (src/fasta.cpp:2067-2088)
    std::vector<std::vector<int32_t>> slots(M);
    std::vector<int64_t> gap_sum(M, 0);
    for (int32_t id = 0; id < M; ++id)
        if (r.is_block[id]) slots[id].assign(len[id] + 1, 0);
    for (int32_t g = 0; g < p->num_gaps; ++g) {
        const int32_t id = p->gap_primary[g];
        if (id < 0 || id >= M || !r.is_block[id]) return fail_(PM_ERR_UNSUPPORTED, "gap list for a missing block");
        for (int64_t k = p->gap_offsets[g]; k < p->gap_offsets[g + 1]; ++k) {
            const uint32_t pos = p->gap_position[k];
            if (pos > (uint32_t)len[id]) return fail_(PM_ERR_ARG, "gap position beyond the block");
            slots[id][pos] = (int32_t)p->gap_length[k];
            gap_sum[id] += p->gap_length[k];
        }
    }
    r.col_start.assign(M, 0);
    r.width.assign(M, 0);
    r.absent_len.assign(M, 0);
    std::vector<std::vector<int64_t>> main_col(M), gap_col(M);   // column of main j / first slot of j
    int64_t cols = 0;
    for (int32_t id = 0; id < M; ++id) {
        r.col_start[id] = cols;
        if (!r.is_block[id]) continue;
        for (int32_t j = 0; j <= len[id]; ++j) cols += slots[id][j] + 1;
        r.width[id] = cols - r.col_start[id];
        r.absent_len[id] = len[id] + gap_sum[id];
    }
    r.columns = cols;
    if (r.columns >= ((int64_t)1 << 32)) return fail_(PM_ERR_UNSUPPORTED, "more than 2^32 aligned columns");
    std::string cons((size_t)cols, '-');
    host_parallel_for(M, [&](int id) {   // blocks fill disjoint column ranges
        if (!r.is_block[id]) return;
        main_col[id].resize(len[id] + 1);
        gap_col[id].resize(len[id] + 1);
        const int32_t b = blk_of[id];
        int64_t at = r.col_start[id];
        int32_t j = 0;
        for (int64_t w = p->block_seq_offsets[b]; w < p->block_seq_offsets[b + 1] && j < len[id]; ++w)
            for (int k = 0; k < 8 && j < len[id]; ++k, ++j) {
                gap_col[id][j] = at;
                at += slots[id][j];
                main_col[id][j] = at;
                cons[(size_t)at++] = nuc_char((int)((p->block_seq[w] >> (4 * (7 - k))) & 15));
            }
        gap_col[id][len[id]] = at;
        at += slots[id][len[id]];
        main_col[id][len[id]] = at;
        cons[(size_t)at] = 'x';
    });

    clock.lap("replay.flat_blocks");
    // ---- per-node edits (column, char), last write per column within a node wins.  Each
    // node's list is written into its own slice of one array (sized from the mutations'
    // lengths), sorted by column and deduplicated in place by host threads, then the slices
    // are compacted in node order.
    std::vector<int64_t> cap_off(N + 1, 0);
    host_parallel_for((N + 15) / 16, [&](int task) {
        for (int32_t v = task * 16; v < std::min(N, task * 16 + 16); ++v) {
            int64_t n = 0;
            for (int64_t k = p->nuc_mut_offsets[v]; k < p->nuc_mut_offsets[v + 1]; ++k) {
                const uint32_t info = p->nuc_mut_info[k], type = info & 7u;
                n += type > 5 ? 0 : type >= 3 ? 1 : std::min<int64_t>(info >> 4, 7);
            }
            cap_off[v + 1] = n;
        }
    });
    for (int32_t v = 0; v < N; ++v) cap_off[v + 1] += cap_off[v];
    // (column << 32) | (list index << 8) | char; uninitialised: the threads fault its pages in
    std::unique_ptr<uint64_t[]> all(new uint64_t[(size_t)std::max<int64_t>(cap_off[N], 1)]);
    std::vector<int64_t> kept(N, 0);
    std::vector<int> node_err(N, PM_OK);
    std::vector<const char*> node_msg(N, nullptr);
    host_parallel_for((N + 15) / 16, [&](int task) {
        for (int32_t v = task * 16; v < std::min(N, task * 16 + 16); ++v) {
            uint64_t* out = all.get() + cap_off[v];
            int64_t cnt = 0;
            auto bad = [&](int code, const char* msg) {
                node_err[v] = code;
                node_msg[v] = msg;
            };
            const int64_t k_end = p->nuc_mut_offsets[v + 1];
            for (int64_t k = p->nuc_mut_offsets[v]; k < k_end && node_err[v] == PM_OK; ++k) {
                if (k + 16 < k_end) {   // the column lookups are random accesses: prefetch ahead
                    const int32_t pid = p->nuc_mut_primary[k + 16], ppos = p->nuc_mut_position[k + 16];
                    if (pid >= 0 && pid < M && r.is_block[pid] && ppos >= 0 && ppos <= len[pid])
                        __builtin_prefetch(p->nuc_mut_gap_position[k + 16] != -1 ? &gap_col[pid][ppos] : &main_col[pid][ppos]);
                }
                const int32_t id = p->nuc_mut_primary[k];
                // the secondary block id is read and never used (src/fasta.cpp:1838-1842): a
                // mutation on a secondary block lands on its primary block, as there
                const uint32_t info = p->nuc_mut_info[k], type = info & 7u;
                int32_t n = (int32_t)(info >> 4);
                if (type > 5) continue;           // no-op types
                if (type >= 3) n = 1;             // NSNPS / NSNPI / NSNPD: one code
                if (id < 0 || id >= M || !r.is_block[id]) { bad(PM_ERR_UNSUPPORTED, "mutation on a missing block"); break; }
                if (n > 6) { bad(PM_ERR_UNSUPPORTED, "nucleotide run longer than 6"); break; }
                const int32_t pos = p->nuc_mut_position[k], gap = p->nuc_mut_gap_position[k];
                const bool del = type == 1 || type == 5;
                for (int32_t j = 0; j < n; ++j) {
                    const int code = (p->nuc_mut_nucs[k] >> (4 * (5 - j))) & 15;
                    int64_t col;
                    if (gap != -1) {
                        if (pos < 0 || pos > len[id] || gap + j >= slots[id][pos] || gap < 0) {
                            bad(PM_ERR_ARG, "gap-slot mutation outside the slot range");
                            break;
                        }
                        col = gap_col[id][pos] + gap + j;
                    } else {
                        if (pos < 0 || pos + j > len[id]) { bad(PM_ERR_ARG, "mutation beyond the block"); break; }
                        col = main_col[id][pos + j];   // pos + j == len rewrites the sentinel, as the reference does
                    }
                    const uint64_t chr = (uint8_t)(del ? '-' : nuc_char(code));
                    out[cnt] = ((uint64_t)col << 32) | ((uint64_t)cnt << 8) | chr;
                    ++cnt;
                }
            }
            if (node_err[v] != PM_OK) continue;
            if (cnt >= ((int64_t)1 << 24)) {
                bad(PM_ERR_UNSUPPORTED, "more than 2^24 column edits on one node");
                continue;
            }
            // (column, list index) order; keep the last edit of each column
            if (!std::is_sorted(out, out + cnt)) std::sort(out, out + cnt);
            int64_t w = 0;
            for (int64_t i = 0; i < cnt; ++i)
                if (i + 1 == cnt || (out[i + 1] >> 32) != (out[i] >> 32)) out[w++] = out[i];
            kept[v] = w;
        }
    });
    for (int32_t v = 0; v < N; ++v)
        if (node_err[v] != PM_OK) return fail_(node_err[v], node_msg[v]);
    std::vector<int64_t>& eoff = h.eoff;
    eoff.assign(N + 1, 0);
    for (int32_t v = 0; v < N; ++v) eoff[v + 1] = eoff[v] + kept[v];
    r.edits = eoff[N];
    std::vector<uint32_t>& ecol = h.ecol;
    std::vector<uint8_t>& echr = h.echr;
    ecol.resize((size_t)r.edits);
    echr.resize((size_t)r.edits);
    host_parallel_for((N + 15) / 16, [&](int task) {
        for (int32_t v = task * 16; v < std::min(N, task * 16 + 16); ++v) {
            const uint64_t* in = all.get() + cap_off[v];
            for (int64_t i = 0, e = eoff[v]; i < kept[v]; ++i, ++e) {
                ecol[e] = (uint32_t)(in[i] >> 32);
                echr[e] = (uint8_t)(in[i] & 0xff);
            }
        }
    });
    all.reset();

    clock.lap("replay.flat_edits");

    // ---- root-to-leaf paths (root first) of this shard's leaves
    const int32_t L = (int32_t)r.leaves.size();
    std::vector<int64_t>& path_off = h.path_off;
    std::vector<int32_t>& path_all = h.path_all;
    path_off.assign(L + 1, 0);
    for (int32_t li = 0; li < L; ++li) {
        int32_t depth = 0;
        for (int32_t n = r.leaves[li]; n >= 0; n = r.parent[n]) ++depth;
        path_off[li + 1] = path_off[li] + depth;
        h.max_depth = std::max(h.max_depth, depth);
    }
    path_all.resize((size_t)path_off[L]);
    host_parallel_for((L + 255) / 256, [&](int task) {
        for (int32_t li = task * 256; li < std::min(L, task * 256 + 256); ++li) {
            int32_t at = (int32_t)(path_off[li + 1] - path_off[li]);
            for (int32_t n = r.leaves[li]; n >= 0; n = r.parent[n]) path_all[(size_t)path_off[li] + --at] = n;
        }
    });
    // ---- leaf groups for k_replay_dfs: the leaves in depth-first order, cut into runs of at
    // most kDfsLeaves whose paths together hold at most kDfsUnionCap nodes; per leaf its path
    // length and the prefix it shares with the previous leaf of its group.  Only when every
    // path fits (else k_replay, tiles of kReplayTile).
    h.dfs = h.max_depth <= kDfsUnionCap && L > 0;
    if (h.dfs) {
        std::vector<int32_t> row_of(N, -1);
        for (int32_t li = 0; li < L; ++li) row_of[r.leaves[li]] = li;
        std::vector<int32_t> order;
        order.reserve(L);
        std::vector<int32_t> st{p->root};
        while (!st.empty()) {   // pre-order, children in list order
            const int32_t v = st.back();
            st.pop_back();
            if (row_of[v] >= 0) order.push_back(row_of[v]);
            for (int32_t e = p->child_offsets[v + 1] - 1; e >= p->child_offsets[v]; --e) st.push_back(p->child_index[e]);
        }
        h.dfs_row = order;
        h.dfs_len.resize(L);
        h.dfs_lpfx.resize(L);
        h.g_leaf_off.assign(1, 0);
        h.g_union_off.assign(1, 0);
        h.g_union.clear();
        int32_t cnt = 0, uni = 0;
        for (int32_t i = 0; i < L; ++i) {
            const int32_t* pa = path_all.data() + path_off[order[i]];
            const int32_t la = (int32_t)(path_off[order[i] + 1] - path_off[order[i]]);
            int32_t lp = 0;
            if (i > 0) {
                const int32_t* pb = path_all.data() + path_off[order[i - 1]];
                const int32_t lb = (int32_t)(path_off[order[i - 1] + 1] - path_off[order[i - 1]]);
                while (lp < la && lp < lb && pa[lp] == pb[lp]) ++lp;
            }
            if (i == 0 || cnt == kDfsLeaves || uni + (la - lp) > kDfsUnionCap) {   // a new group
                if (i > 0) {
                    h.g_leaf_off.push_back(i);
                    h.g_union_off.push_back((int32_t)h.g_union.size());
                }
                cnt = 0;
                uni = 0;
                lp = 0;
            }
            for (int32_t k = lp; k < la; ++k) h.g_union.push_back(pa[k]);
            uni += la - lp;
            ++cnt;
            h.dfs_len[i] = (uint16_t)la;
            h.dfs_lpfx[i] = (uint16_t)lp;
        }
        h.g_leaf_off.push_back(L);
        h.g_union_off.push_back((int32_t)h.g_union.size());
    }
    const int64_t tb = h.dfs ? kDfsTile : kReplayTile;   // bytes per column tile

    // ---- column tiles: per node, the first (column-sorted) edit of every tile
    const int64_t stride = (r.columns + 15) / 16 * 16;
    const int32_t tiles = (int32_t)((stride + tb - 1) / tb);
    std::vector<int64_t>& tile_edit = h.tile_edit;
    tile_edit.resize((size_t)N * (tiles + 1));
    host_parallel_for((N + 15) / 16, [&](int task) {
        for (int32_t v = task * 16; v < std::min(N, task * 16 + 16); ++v) {
            int64_t e = eoff[v];
            for (int32_t t = 0; t <= tiles; ++t) {
                const int64_t c0 = std::min<int64_t>((int64_t)t * tb, stride);
                while (e < eoff[v + 1] && (int64_t)ecol[e] < c0) ++e;
                tile_edit[(size_t)v * (tiles + 1) + t] = e;
            }
        }
    });

    // ---- edits that overwrite an ancestor's edit of the same column get kEditOverrides in
    // their character byte: the replay kernel writes the others in any order and only these
    // in path order (k_replay_piped).  A depth-first walk with a count of the ancestors' edits
    // per column; the columns are split into ranges of tiles walked by host threads (each
    // node's edits of a range are one slice of its column-sorted list, tile_edit).
    {
        std::vector<std::pair<int32_t, bool>> walk;   // (node, leaving) in depth-first order
        walk.reserve(2 * (size_t)N);
        std::vector<std::pair<int32_t, bool>> stack{{p->root, false}};
        while (!stack.empty()) {
            const auto ev = stack.back();
            stack.pop_back();
            walk.push_back(ev);
            if (ev.second) continue;
            stack.push_back({ev.first, true});
            for (int32_t e = p->child_offsets[ev.first]; e < p->child_offsets[ev.first + 1]; ++e)
                stack.push_back({p->child_index[e], false});
        }
        const int T = std::max(1, std::min(host_threads() * 2, tiles));
        host_parallel_for(T, [&](int task) {
            const int32_t t0 = (int32_t)((int64_t)tiles * task / T), t1 = (int32_t)((int64_t)tiles * (task + 1) / T);
            if (t1 <= t0) return;
            const int64_t c0 = (int64_t)t0 * tb;
            std::vector<int32_t> active((size_t)(t1 - t0) * tb, 0);
            for (const auto& [v, leaving] : walk) {
                const int64_t e0 = tile_edit[(size_t)v * (tiles + 1) + t0], e1 = tile_edit[(size_t)v * (tiles + 1) + t1];
                if (leaving) {
                    for (int64_t e = e0; e < e1; ++e) --active[ecol[e] - c0];
                    continue;
                }
                for (int64_t e = e0; e < e1; ++e)
                    if (active[ecol[e] - c0]++ > 0) echr[e] |= kEditOverrides;
            }
        });
    }
    // ---- each node's slice as [plain edits | overriding edits], both column-sorted, and per
    // (node, tile) the first edit of each part (int2 {plain, overriding}): the kernel writes a
    // tile's plain edits in any order and resolves the overriding ones afterwards
    // (k_replay: deepest on the path wins)
    if (r.edits >= ((int64_t)1 << 31)) return fail_(PM_ERR_UNSUPPORTED, "more than 2^31 column edits");
    std::vector<int2>& tile2 = h.tile2;
    tile2.resize((size_t)N * (tiles + 1));
    host_parallel_for((N + 15) / 16, [&](int task) {
        std::vector<uint32_t> oc;
        std::vector<uint8_t> oh;
        for (int32_t v = task * 16; v < std::min(N, task * 16 + 16); ++v) {
            const int64_t b = eoff[v], e = eoff[v + 1];
            oc.clear();
            oh.clear();
            int64_t w = b;
            for (int64_t k = b; k < e; ++k) {
                if (echr[k] & kEditOverrides) {
                    oc.push_back(ecol[k]);
                    oh.push_back(echr[k]);
                } else {
                    ecol[w] = ecol[k];
                    echr[w] = echr[k];
                    ++w;
                }
            }
            const int64_t mid = w;
            for (size_t k = 0; k < oc.size(); ++k, ++w) {
                ecol[w] = oc[k];
                echr[w] = oh[k];
            }
            int64_t ep = b, eo = mid;
            for (int32_t t = 0; t <= tiles; ++t) {
                const int64_t c0 = std::min<int64_t>((int64_t)t * tb, stride);
                while (ep < mid && (int64_t)ecol[ep] < c0) ++ep;
                while (eo < e && (int64_t)ecol[eo] < c0) ++eo;
                tile2[(size_t)v * (tiles + 1) + t] = make_int2((int)ep, (int)eo);
            }
        }
    });
    std::vector<int64_t>().swap(tile_edit);
    clock.lap("replay.flat_overrides");
    // ---- per-leaf block state (getBlockSequence + the block-mutation pass of the helper)
    const int32_t words = (M + 31) / 32;
    std::vector<uint32_t>& presence = h.presence;
    presence.assign((size_t)L * words, 0);
    r.present.assign(L, {});
    r.exists.assign(L, {});
    r.strand.assign(L, {});
    const int64_t nb_slots = (int64_t)B + 1;   // blockSequence has blocks.size()+1 entries
    std::vector<int> leaf_err(L, PM_OK);
    host_parallel_for((L + 15) / 16, [&](int task) {
        for (int32_t li = task * 16; li < std::min(L, task * 16 + 16); ++li) {
            const int32_t* path = path_all.data() + path_off[li];   // root first
            const int32_t depth = (int32_t)(path_off[li + 1] - path_off[li]);
            std::vector<uint8_t> pres(std::max<int64_t>(M, nb_slots), 0), ex(M, 0), st(M, 1);
            for (int32_t i = 0; i < depth; ++i) {
                const int32_t n = path[i];
                for (int64_t k = p->block_mut_offsets[n]; k < p->block_mut_offsets[n + 1]; ++k) {
                    const int32_t id = p->block_mut_primary[k];
                    if (id < 0 || id >= (int32_t)pres.size()) {
                        leaf_err[li] = PM_ERR_ARG;
                        break;
                    }
                    if (p->block_mut_info[k]) pres[id] = 1;
                    else if (!p->block_mut_inversion[k]) pres[id] = 0;
                }
            }
            if (leaf_err[li] != PM_OK) continue;
            for (int32_t i = 0; i < depth; ++i) {
                const int32_t n = path[i];
                for (int64_t k = p->block_mut_offsets[n]; k < p->block_mut_offsets[n + 1]; ++k) {
                    const int32_t id = p->block_mut_primary[k];
                    if (id >= M || !pres[id]) continue;
                    if (p->block_mut_info[k]) { ex[id] = 1; st[id] = !p->block_mut_inversion[k]; }
                    else if (p->block_mut_inversion[k]) st[id] = !st[id];
                    else { ex[id] = 0; st[id] = 1; }
                }
            }
            pres.resize(M);
            for (int32_t id = 0; id < M; ++id)
                if (pres[id]) presence[(size_t)li * words + id / 32] |= 1u << (id % 32);
            r.present[li] = std::move(pres);
            r.exists[li] = std::move(ex);
            r.strand[li] = std::move(st);
        }
    });
    for (int32_t li = 0; li < L; ++li)
        if (leaf_err[li] != PM_OK) return fail_(PM_ERR_ARG, "block mutation id out of range");
    r.circular.assign(L, -1);
    r.rotation.assign(L, 0);
    r.inverted.assign(L, 0);
    for (int32_t li = 0; li < L; ++li) {
        const int32_t v = r.leaves[li];
        if (p->circular_offset) r.circular[li] = p->circular_offset[v];
        if (p->rotation_index) r.rotation[li] = p->rotation_index[v];
        if (p->sequence_inverted) r.inverted[li] = p->sequence_inverted[v];
    }

    clock.lap("replay.flat_leaves");
    h.blk_lo.resize(M);
    h.blk_hi.resize(M);
    for (int32_t id = 0; id < M; ++id) {
        h.blk_lo[id] = r.col_start[id];
        h.blk_hi[id] = r.col_start[id] + r.width[id];
    }
    h.tile_blk.resize(tiles + 1);
    for (int32_t t = 0, id = 0; t <= tiles; ++t) {
        const int64_t c0 = (int64_t)t * tb;
        while (id < M && h.blk_hi[id] <= c0) ++id;
        h.tile_blk[t] = id;
    }
    h.cons_row.assign((size_t)stride, '-');
    std::memcpy(h.cons_row.data(), cons.data(), cons.size());
    h.words = words;
    h.stride = stride;
    h.tiles = tiles;
    h.tile_bytes = (int32_t)tb;
    r.cons = std::move(cons);
    r.main_col = std::move(main_col);
    r.gap_col = std::move(gap_col);
    r.slots = std::move(slots);
    clock.lap("replay.flat_tiles");
    (void)ferr;
    return PM_OK;
}

int replay_prepare(pm_ctx* c, const pm_panmat* p, ReplayState& r, int64_t leaf_begin, int64_t leaf_end) {
    PhaseClock clock;
    ReplayHost h;
    std::string msg;
    const int rc = replay_flatten(p, r, h, leaf_begin, leaf_end, msg);
    if (rc != PM_OK) return fail(c, rc, msg);
    clock.lap("replay.prepare_host");
    const int32_t L = (int32_t)r.leaves.size();
    const int32_t M = r.max_id + 1;
    hipError_t e;
    // (the rows live in the context's grow-only buffer: a 5 GB hipMalloc + hipFree per call
    // is not free, and pm_fasta prepares again on every call)
    if ((e = grow_device(&c->rows_buf, &c->rows_cap, (size_t)std::max<int64_t>(L, 1) * h.stride)) != hipSuccess)
        return fail(c, PM_ERR_OOM, "replay rows");
    r.d_rows = static_cast<char*>(c->rows_buf);
    if ((e = dput(&r.d_cons, h.cons_row, c->stream)) != hipSuccess || (e = dput(&r.d_parent, r.parent, c->stream)) != hipSuccess ||
        (e = dput(&r.d_leaf, r.leaves, c->stream)) != hipSuccess || (e = dput(&r.d_presence, h.presence, c->stream)) != hipSuccess ||
        (e = dput(&r.d_eoff, h.eoff, c->stream)) != hipSuccess || (e = dput(&r.d_ecol, h.ecol, c->stream)) != hipSuccess ||
        (e = dput(&r.d_echr, h.echr, c->stream)) != hipSuccess || (e = dput(&r.d_blk_lo, h.blk_lo, c->stream)) != hipSuccess ||
        (e = dput(&r.d_blk_hi, h.blk_hi, c->stream)) != hipSuccess || (e = dput(&r.d_tile_blk, h.tile_blk, c->stream)) != hipSuccess ||
        (e = dput(&r.d_tile2, h.tile2, c->stream)) != hipSuccess ||
        (e = dput(&r.d_path_off, h.path_off, c->stream)) != hipSuccess || (e = dput(&r.d_path, h.path_all, c->stream)) != hipSuccess ||
        (e = dput(&r.d_dfs_row, h.dfs_row, c->stream)) != hipSuccess || (e = dput(&r.d_dfs_len, h.dfs_len, c->stream)) != hipSuccess ||
        (e = dput(&r.d_dfs_lpfx, h.dfs_lpfx, c->stream)) != hipSuccess ||
        (e = dput(&r.d_g_leaf_off, h.g_leaf_off, c->stream)) != hipSuccess ||
        (e = dput(&r.d_g_union_off, h.g_union_off, c->stream)) != hipSuccess ||
        (e = dput(&r.d_g_union, h.g_union, c->stream)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&r.d_rebuilds), sizeof(int32_t))) != hipSuccess ||
        (e = hipMemsetAsync(r.d_rebuilds, 0, sizeof(int32_t), c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, e, "replay upload");
    clock.lap("replay.upload");
    // (counts, not seconds: the deepest root->leaf path and its 64-node edit chunks per tile)
    phase_add("replay.max_depth", (double)h.max_depth);
    phase_add("replay.path_chunks", (double)((h.max_depth + kWave - 1) / kWave));
    phase_add("replay.dfs_groups", h.dfs ? (double)(h.g_leaf_off.size() - 1) : 0.0);   // 0: k_replay
    if (h.dfs) {   // edits k_replay_dfs reads: every edit of each group's path-node union, once per group
        double ge = 0.0;
        for (int32_t v : h.g_union) ge += (double)(h.eoff[(size_t)v + 1] - h.eoff[(size_t)v]);
        phase_add("replay.group_edits", ge);
    }
    ReplayDev& d = r.dev;
    d.leaves = L;
    d.row_stride = h.stride;
    d.columns = r.columns;
    d.max_depth = h.max_depth;
    d.presence_words = h.words;
    d.rows = r.d_rows;
    d.cons_row = r.d_cons;
    d.parent = r.d_parent;
    d.leaf_node = r.d_leaf;
    d.presence = r.d_presence;
    d.edit_off = r.d_eoff;
    d.edit_col = r.d_ecol;
    d.edit_chr = r.d_echr;
    d.blocks = M;
    d.blk_lo = r.d_blk_lo;
    d.blk_hi = r.d_blk_hi;
    d.tile_blk = r.d_tile_blk;
    d.tiles = h.tiles;
    d.tile2 = r.d_tile2;
    d.ring = std::min(std::max(kWave, (h.max_depth + kWave - 1) / kWave * kWave), kReplayRingMax);
    d.path_off = r.d_path_off;
    d.path = r.d_path;
    d.tile_bytes = h.tile_bytes;
    d.dfs = h.dfs;
    d.groups = h.dfs ? (int32_t)h.g_leaf_off.size() - 1 : 0;
    d.dfs_row = r.d_dfs_row;
    d.dfs_len = r.d_dfs_len;
    d.dfs_lpfx = r.d_dfs_lpfx;
    d.g_leaf_off = r.d_g_leaf_off;
    d.g_union_off = r.d_g_union_off;
    d.g_union = r.d_g_union;
    d.dfs_rebuilds = r.d_rebuilds;
    return PM_OK;
}

void free_replay(pm_ctx* c) {
    if (!c->replay) return;
    ReplayState* r = c->replay;
    r->d_rows = nullptr;   // (c->rows_buf, kept)
    dfree(r->d_cons);
    dfree(r->d_parent);
    dfree(r->d_leaf);
    dfree(r->d_presence);
    dfree(r->d_eoff);
    dfree(r->d_ecol);
    dfree(r->d_echr);
    dfree(r->d_blk_lo);
    dfree(r->d_blk_hi);
    dfree(r->d_tile_blk);
    dfree(r->d_tile2);
    dfree(r->d_path_off);
    dfree(r->d_path);
    dfree(r->d_dfs_row);
    dfree(r->d_dfs_len);
    dfree(r->d_dfs_lpfx);
    dfree(r->d_g_leaf_off);
    dfree(r->d_g_union_off);
    dfree(r->d_g_union);
    dfree(r->d_rebuilds);
    delete r;
    c->replay = nullptr;
}

}  // namespace pm

namespace pm {
// The FASTA text of the replayed rows in the context's device text buffer (c->text_buf),
// `total` bytes; `clock` carries on into the caller's download phase.
int format_device(pm_ctx* c, int aligned, int64_t& total, PhaseClock& clock) {
    if (!c) return PM_ERR_ARG;
    if (!c->replay || !c->replay->ran) return fail(c, PM_ERR_STATE, "run the replay first");
    (void)hipSetDevice(c->device);
    const ReplayState& r = *c->replay;
    const int32_t L = (int32_t)r.leaves.size();
    const int32_t M = r.max_id + 1;
    std::vector<FmtSeg> seg((size_t)L * M);
    const int32_t LB = 64;   // leaves per host task
    host_parallel_for((L + LB - 1) / LB, [&](int task) {
    std::vector<int32_t> order(M);
    for (int32_t li = task * LB; li < std::min(L, (task + 1) * LB); ++li) {
        for (int32_t i = 0; i < M; ++i) order[i] = i;
        const auto& ex = r.exists[li];
        if (r.rotation[li] != 0) {   // rotate to the rotationIndexes-th existing block (:1950-1964)
            int32_t ctr = -1, at = 0;
            for (int32_t i = 0; i < M; ++i) {
                if (ex[i]) ++ctr;
                if (ctr == r.rotation[li]) { at = i; break; }
            }
            std::rotate(order.begin(), order.begin() + at, order.end());
        }
        if (r.inverted[li]) std::reverse(order.begin(), order.end());
        for (int32_t i = 0; i < M; ++i) {
            const int32_t id = order[i];
            FmtSeg& sg = seg[(size_t)li * M + i];
            if (ex[id]) {
                sg = FmtSeg{r.col_start[id], r.width[id], r.strand[li][id] ? 0 : 1, 0};
            } else {   // blockLengths is indexed by print position i, not by the block printed there
                sg = FmtSeg{-1, (r.is_block[i] && !r.present[li][i]) ? r.absent_len[i] : 0, 0, 0};
            }
        }
    }
    });
    std::vector<int64_t> name_off(L + 1, 0);
    std::string names;
    for (int32_t li = 0; li < L; ++li) {
        names += r.names[r.leaves[li]];
        name_off[li + 1] = (int64_t)names.size();
    }
    const size_t NS = (size_t)L * M;
    FmtSeg* d_seg = nullptr;
    int64_t *d_len = nullptr, *d_off = nullptr, *d_line = nullptr, *d_start = nullptr, *d_text_off = nullptr,
            *d_name_off = nullptr;
    char *d_names = nullptr, *d_text = nullptr;   // (d_text: the context's grow-only text buffer)
    auto cleanup = [&]() {
        dfree(d_seg); dfree(d_len); dfree(d_off); dfree(d_line); dfree(d_start); dfree(d_text_off);
        dfree(d_name_off); dfree(d_names);
    };
    clock.lap("fasta.segments_host");
    hipError_t e = dput(&d_seg, seg, c->stream);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_len), sizeof(int64_t) * std::max<size_t>(NS, 1));
    if (e != hipSuccess) {
        cleanup();
        return fail(c, PM_ERR_OOM, "FASTA segments");
    }
    FmtArgs f{};
    f.rows = r.d_rows;
    f.row_stride = r.dev.row_stride;
    f.positions = M;
    f.aligned = aligned != 0;
    f.seg = d_seg;
    f.seg_len = d_len;
    std::vector<int64_t> len(NS);
    e = launch_fmt_count(c, f, L);
    if (e == hipSuccess && NS) e = hipMemcpyAsync(len.data(), d_len, sizeof(int64_t) * NS, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        cleanup();
        return hip_fail(c, e, "FASTA segment count");
    }
    std::vector<int64_t> off(NS), line(L), start(L), text_off(L + 1, 0);
    for (int32_t li = 0; li < L; ++li) {
        int64_t p = 0;
        for (int32_t i = 0; i < M; ++i) {
            off[(size_t)li * M + i] = p;
            p += len[(size_t)li * M + i];
        }
        line[li] = p;
        // circular offset, unaligned only: the line holds no '-' then, so the offset-th
        // character starts the record (or the line is printed as is when it is shorter)
        const int64_t o = aligned ? 0 : std::max(0, r.circular[li]);
        start[li] = o < p ? o : 0;
        const int64_t hdr = name_off[li + 1] - name_off[li] + 2;
        text_off[li + 1] = text_off[li] + hdr + p + p / 70 + 1;
    }
    total = text_off[L];
    clock.lap("fasta.count");
    if ((e = dput(&d_off, off, c->stream)) != hipSuccess || (e = dput(&d_line, line, c->stream)) != hipSuccess ||
        (e = dput(&d_start, start, c->stream)) != hipSuccess || (e = dput(&d_text_off, text_off, c->stream)) != hipSuccess ||
        (e = dput(&d_name_off, name_off, c->stream)) != hipSuccess ||
        (e = dput(&d_names, std::vector<char>(names.begin(), names.end()), c->stream)) != hipSuccess ||
        (e = grow_device(&c->text_buf, &c->text_cap, (size_t)std::max<int64_t>(total, 1))) != hipSuccess) {
        cleanup();
        return fail(c, PM_ERR_OOM, "FASTA buffers");
    }
    d_text = static_cast<char*>(c->text_buf);
    f.seg_off = d_off;
    f.line_len = d_line;
    f.start = d_start;
    f.text_off = d_text_off;
    f.name_off = d_name_off;
    f.names = d_names;
    f.text = d_text;
    e = launch_fmt_write(c, f, L);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    clock.lap("fasta.text_kernel");
    cleanup();
    if (e != hipSuccess) return hip_fail(c, e, "FASTA text kernel");
    return PM_OK;
}
}  // namespace pm

using namespace pm;

extern "C" {

int pm_replay_prepare_range(pm_ctx* c, const pm_panmat* p, int64_t leaf_begin, int64_t leaf_end) {
    if (!c || !p) return PM_ERR_ARG;
    (void)hipSetDevice(c->device);
    free_replay(c);
    c->replay = new ReplayState();
    int rc = replay_prepare(c, p, *c->replay, leaf_begin, leaf_end);
    if (rc != PM_OK) free_replay(c);
    return rc;
}

int pm_replay_prepare(pm_ctx* c, const pm_panmat* p) { return pm_replay_prepare_range(c, p, -1, -1); }

int pm_replay_run(pm_ctx* c) {
    if (!c) return PM_ERR_ARG;
    if (!c->replay) return fail(c, PM_ERR_STATE, "prepare a PanMAT first");
    (void)hipSetDevice(c->device);
    hipError_t e = launch_replay(c, c->replay->dev);
    if (e != hipSuccess) return hip_fail(c, e, "replay launch");
    c->replay->ran = true;
    return PM_OK;
}

int pm_replay_shape(pm_ctx* c, int64_t* leaves, int64_t* columns, int64_t* edits) {
    if (!c || !c->replay) return PM_ERR_ARG;
    if (leaves) *leaves = (int64_t)c->replay->leaves.size();
    if (columns) *columns = c->replay->columns;
    if (edits) *edits = c->replay->edits;
    return PM_OK;
}

// printFASTAUltraFast's output stage (src/fasta.cpp:1944-1975, 2089-2094) and
// printSequenceLinesNew (:155-254) on the device: per leaf the blocks in print order
// (rotation to the rotationIndexes-th existing block, reversal when inverted), forward or
// reverse-complemented, '-' dropped when unaligned, absent blocks as blockLengths dashes
// (indexed by print position, as the reference does), the line rotated by the circular
// offset (unaligned only) and wrapped at 70 columns.  Host work: segment table, scans.

int pm_replay_format(pm_ctx* c, int aligned, char** text, int64_t* length) {
    if (!c || !text || !length) return PM_ERR_ARG;
    PhaseClock clock;
    int64_t total = 0;
    int rc = format_device(c, aligned, total, clock);
    if (rc != PM_OK) return rc;
    char* out = static_cast<char*>(host_alloc_large((size_t)total + 1));
    if (!out) return fail(c, PM_ERR_OOM, "FASTA text");
    // the text through pinned slots drained by host threads (pm_hostio.cpp), not one pageable copy
    const hipError_t e = d2h_large(c, out, c->text_buf, (size_t)total);
    if (e != hipSuccess) {
        std::free(out);
        return hip_fail(c, e, "FASTA write");
    }
    out[total] = 0;
    clock.lap("fasta.download");
    *text = out;
    *length = total;
    return PM_OK;
}

int pm_replay_format_fd(pm_ctx* c, int aligned, int fd, int64_t* length) {
    if (!c || fd < 0) return PM_ERR_ARG;
    PhaseClock clock;
    int64_t total = 0;
    int rc = format_device(c, aligned, total, clock);
    if (rc != PM_OK) return rc;
    bool wrote = true;
    const hipError_t e = d2h_stream(c, c->text_buf, (size_t)total,
                                    [fd](const char* p, size_t n) { return write_all(fd, p, n); }, wrote);
    if (e != hipSuccess) return hip_fail(c, e, "FASTA download");
    if (!wrote) return fail(c, PM_ERR_ARG, "FASTA write: " + std::string(std::strerror(errno)));
    clock.lap("fasta.download_write");
    if (length) *length = total;
    return PM_OK;
}

namespace {
// prepare + replay (+ the depth-first kernel's rebuild count in the phase log)
int fasta_replay(pm_ctx* c, const pm_panmat* p) {
    int rc = pm_replay_prepare(c, p);
    if (rc == PM_OK) {
        PhaseClock clock;
        rc = pm_replay_run(c);
        if (rc == PM_OK && c && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(c, PM_ERR_HIP, "replay");
        clock.lap("replay.kernel");
        int32_t rebuilds = 0;   // (a count: k_replay_dfs's (leaf, tile) rows rebuilt after a stack overflow)
        if (rc == PM_OK && c->replay->dev.dfs) {
            if (hipMemcpy(&rebuilds, c->replay->d_rebuilds, sizeof(rebuilds), hipMemcpyDeviceToHost) != hipSuccess)
                rc = fail(c, PM_ERR_HIP, "replay rebuild count");
            phase_add("replay.dfs_rebuilds", (double)rebuilds);
        }
    }
    return rc;
}
}  // namespace

int pm_fasta_fd(pm_ctx* c, const pm_panmat* p, int aligned, int fd, int64_t* length) {
    int rc = fasta_replay(c, p);
    if (rc == PM_OK) rc = pm_replay_format_fd(c, aligned, fd, length);
    return rc;
}

int pm_fasta(pm_ctx* c, const pm_panmat* p, int aligned, char** text, int64_t* length) {
    int rc = fasta_replay(c, p);
    if (rc == PM_OK) rc = pm_replay_format(c, aligned, text, length);
    return rc;
}

int pm_fasta_multi(const pm_panmat* p, int aligned, const int* devices, int num_devices, char** text,
                   int64_t* length, char* err, int64_t err_len) {
    auto set_err = [&](const std::string& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
    };
    if (!p || !devices || num_devices < 1 || !text || !length || p->num_nodes < 1 || !p->child_offsets) {
        set_err("bad arguments");
        return PM_ERR_ARG;
    }
    int64_t L = 0;
    for (int32_t i = 0; i < p->num_nodes; ++i) L += p->child_offsets[i] == p->child_offsets[i + 1];
    // leaves split into contiguous ranges, one host thread + context per device; the
    // ranges' texts concatenate to the single-device text
    const int G = num_devices;
    std::vector<char*> part(G, nullptr);
    std::vector<int64_t> plen(G, 0);
    std::vector<int> rc(G, PM_OK);
    std::vector<std::string> msg(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g]() {
            const int64_t lo = L * g / G, hi = L * (g + 1) / G;
            if (hi == lo) return;   // more devices than leaves
            pm_ctx* c = nullptr;
            if ((rc[g] = pm_create(devices[g], &c)) != PM_OK) {
                msg[g] = "no HIP device " + std::to_string(devices[g]);
                return;
            }
            rc[g] = pm_replay_prepare_range(c, p, lo, hi);
            if (rc[g] == PM_OK) rc[g] = pm_replay_run(c);
            if (rc[g] == PM_OK) rc[g] = pm_replay_format(c, aligned, &part[g], &plen[g]);
            if (rc[g] != PM_OK) msg[g] = pm_last_error(c);
            pm_destroy(c);
        });
    for (auto& t : th) t.join();
    int64_t total = 0;
    for (int g = 0; g < G; ++g) {
        if (rc[g] != PM_OK) {
            for (char* x : part) std::free(x);
            set_err(msg[g]);
            return rc[g];
        }
        total += plen[g];
    }
    int nonempty = 0, only = -1;
    for (int g = 0; g < G; ++g)
        if (part[g]) {
            ++nonempty;
            only = g;
        }
    if (nonempty == 1) {   // one shard holds every leaf: its text is the result
        for (int g = 0; g < G; ++g)
            if (g != only) std::free(part[g]);
        *text = part[only];
        *length = plen[only];
        return PM_OK;
    }
    char* out = static_cast<char*>(host_alloc_large((size_t)total + 1));
    if (!out) {
        for (char* x : part) std::free(x);
        set_err("FASTA text");
        return PM_ERR_OOM;
    }
    std::vector<int64_t> at(G + 1, 0);
    for (int g = 0; g < G; ++g) at[g + 1] = at[g] + plen[g];
    constexpr int64_t kPiece = (int64_t)8 << 20;   // concatenation by host threads, 8 MiB pieces
    std::vector<std::pair<int, int64_t>> pieces;
    for (int g = 0; g < G; ++g)
        for (int64_t a = 0; a < plen[g]; a += kPiece) pieces.emplace_back(g, a);
    host_parallel_for((int)pieces.size(), [&](int i) {
        const auto [g, a] = pieces[i];
        std::memcpy(out + at[g] + a, part[g] + a, (size_t)std::min(kPiece, plen[g] - a));
    });
    for (char* x : part) std::free(x);
    out[total] = 0;
    *text = out;
    *length = total;
    return PM_OK;
}


// pm_fasta_multi straight to a file descriptor: the shards are replayed and formatted on their
// devices side by side, then each shard's text streams from its device to `fd` in leaf order
// (the single-device text, byte for byte).
int pm_fasta_multi_fd(const pm_panmat* p, int aligned, const int* devices, int num_devices, int fd, int64_t* length,
                      char* err, int64_t err_len) {
    auto set_err = [&](const std::string& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
    };
    if (!p || !devices || num_devices < 1 || fd < 0 || p->num_nodes < 1 || !p->child_offsets) {
        set_err("bad arguments");
        return PM_ERR_ARG;
    }
    int64_t L = 0;
    for (int32_t i = 0; i < p->num_nodes; ++i) L += p->child_offsets[i] == p->child_offsets[i + 1];
    const int G = num_devices;
    std::vector<pm_ctx*> ctx(G, nullptr);
    std::vector<int64_t> plen(G, 0);
    std::vector<int> rc(G, PM_OK);
    std::vector<std::string> msg(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g]() {
            const int64_t lo = L * g / G, hi = L * (g + 1) / G;
            if (hi == lo) return;   // more devices than leaves
            if ((rc[g] = pm_create(devices[g], &ctx[g])) != PM_OK) {
                msg[g] = "no HIP device " + std::to_string(devices[g]);
                ctx[g] = nullptr;
                return;
            }
            pm_ctx* c = ctx[g];
            rc[g] = G == 1 ? fasta_replay(c, p) : pm_replay_prepare_range(c, p, lo, hi);
            if (rc[g] == PM_OK && G > 1) rc[g] = pm_replay_run(c);
            if (rc[g] == PM_OK) {
                PhaseClock clock;
                rc[g] = format_device(c, aligned, plen[g], clock);
            }
            if (rc[g] != PM_OK) msg[g] = pm_last_error(c);
        });
    for (auto& t : th) t.join();
    int status = PM_OK;
    for (int g = 0; g < G && status == PM_OK; ++g)
        if (rc[g] != PM_OK) {
            set_err(msg[g]);
            status = rc[g];
        }
    int64_t total = 0;
    PhaseClock clock;
    for (int g = 0; g < G && status == PM_OK; ++g) {
        if (!ctx[g] || plen[g] == 0) continue;
        bool wrote = true;
        const hipError_t e = d2h_stream(ctx[g], ctx[g]->text_buf, (size_t)plen[g],
                                        [fd](const char* q, size_t n) { return write_all(fd, q, n); }, wrote);
        if (e != hipSuccess) {
            set_err(std::string("FASTA download: ") + hipGetErrorString(e));
            status = PM_ERR_HIP;
        } else if (!wrote) {
            set_err(std::string("FASTA write: ") + std::strerror(errno));
            status = PM_ERR_ARG;
        }
        total += plen[g];
    }
    clock.lap("fasta.download_write");
    for (pm_ctx* c : ctx)
        if (c) pm_destroy(c);
    if (length) *length = total;
    return status;
}

}  // extern "C"
