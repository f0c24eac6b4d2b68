// pm_pangraph.cpp -- PanMAN construction from a PanGraph JSON + Newick (reference:
// Tree(ifstream&, ifstream&, FILE_TYPE::PANGRAPH, reference), src/panman.cpp:820-1273;
// Pangraph, :6200-6476; chain_align, src/chaining.cpp; rotate_sample, src/rotation.cpp).
//
// Host: the PanGraph model (paths, blocks, per-sequence edits), block ordering by chained
// alignment of the paths, per-sequence block expansion.  Device: every block column
// (block parsimony) and every nucleotide column (main positions + gap slots) of every
// block at once through the batch kernels, leaves lacking a block absent from its columns.
//
// Order-dependent steps follow the reference's containers: std::unordered_map where it
// uses one (paths, alignedSequences, the chaining score map -- libstdc++ iteration order
// reproduced by the same container fed the same insertions), and for the root forcing of
// main columns the oneTBB concurrent_unordered_map order of individualSequences, restated
// as ascending bit-reversed tbb_hasher(name).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#include "pm_internal.h"
#include "pm_json.h"
#include "pm_newick.h"
#include "pm_panman_tree.h"

namespace pm {
namespace {

uint8_t code_of(char ch) {
    switch (ch) {
        case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
        case 'R': return 5;  case 'Y': return 10; case 'S': return 6;  case 'W': return 9;
        case 'K': return 12; case 'M': return 3;  case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7;  case 'N': return 15;
        default: return 0;
    }
}

std::string upper(std::string s) {
    for (char& c : s) c = (char)std::toupper((unsigned char)c);
    return s;
}

// ---- src/chaining.cpp -----------------------------------------------------------------
using Pt = std::pair<int, int>;
const Pt kOrigin(-1, -1);

struct HashPair {   // src/chaining.cpp:24-37
    size_t operator()(const Pt& p) const {
        const size_t h1 = std::hash<int>{}(p.first), h2 = std::hash<int>{}(p.second);
        return h1 != h2 ? h1 ^ h2 : h1;
    }
};

struct RangeNode {
    Pt point;
    int left = -1, right = -1;
};

int build_range_tree(std::vector<Pt>& pts, int start, int end, std::vector<RangeNode>& nodes) {   // :69-82
    if (start > end) return -1;
    std::sort(pts.begin() + start, pts.begin() + end + 1, [](const Pt& a, const Pt& b) { return a.first < b.first; });
    const int mid = (start + end) / 2;
    const int me = (int)nodes.size();
    nodes.push_back(RangeNode{pts[mid]});
    const int l = build_range_tree(pts, start, mid - 1, nodes);
    const int r = build_range_tree(pts, mid + 1, end, nodes);
    nodes[me].left = l;
    nodes[me].right = r;
    return me;
}

void query_range(const std::vector<RangeNode>& nodes, int root, Pt lo, Pt hi, std::vector<Pt>& out) {   // :87-100
    if (root < 0) return;
    const RangeNode& n = nodes[root];
    if (n.point.first >= lo.first && n.point.first <= hi.first && n.point.second >= lo.second &&
        n.point.second <= hi.second)
        out.push_back(n.point);
    if (n.left >= 0 && lo.first <= n.point.first) query_range(nodes, n.left, lo, hi, out);
    if (n.right >= 0 && hi.first >= n.point.first) query_range(nodes, n.right, lo, hi, out);
}

using ScoreMap = std::unordered_map<Pt, std::pair<int, Pt>, HashPair>;

void find_chain(const std::vector<RangeNode>& nodes, int root, Pt point, ScoreMap& map, int K) {   // :102-143
    const int match = 50;
    if (point.first == 0 && point.second == 0) {
        map[point] = {match, Pt(-1, -1)};
        return;
    }
    std::vector<Pt> result;
    query_range(nodes, root, Pt(point.first - K > 0 ? point.first - K : 0, point.second - K > 0 ? point.second - K : 0),
                Pt(point.first - 1, point.second - 1), result);
    int best = 10;
    Pt best_node = kOrigin;
    int xb = -1, yb = -1;
    for (auto it = result.rbegin(); it != result.rend(); ++it) {
        const Pt p = *it;
        if (p.first <= xb && p.second <= yb) continue;
        const int cost = -(point.first - p.first + point.second - p.second);
        if (cost + map[p].first + match > best) {
            best = cost + map[p].first + match;
            best_node = p;
        }
        if (xb < p.first) xb = p.first - 1;
        if (yb < p.second) yb = p.second - 1;
    }
    map[point] = {best, best_node};
}

std::vector<Pt> chaining(const std::vector<std::string>& cons, const std::vector<std::string>& sample) {   // :146-230
    std::vector<Pt> chain;
    const int K = 4000;
    std::vector<Pt> pts;
    for (size_t i = 0; i < cons.size(); ++i)
        for (size_t j = 0; j < sample.size(); ++j)
            if (cons[i] == sample[j]) pts.emplace_back((int)i, (int)j);
    std::sort(pts.begin(), pts.end());   // comparePoint: (x, y), points are distinct
    std::vector<RangeNode> nodes;
    nodes.reserve(pts.size());
    const int root = build_range_tree(pts, 0, (int)pts.size() - 1, nodes);
    if (pts.empty()) return chain;
    ScoreMap map;
    for (const Pt& p : pts) map[p] = {-1, kOrigin};
    for (const Pt& p : pts) find_chain(nodes, root, p, map, K);
    int best = -1;
    Pt seed{};
    for (const auto& m : map)
        if (m.second.first > best) {
            best = m.second.first;
            seed = m.first;
        }
    while (true) {
        chain.push_back(seed);
        seed = map[seed].second;
        if (seed == kOrigin) break;
    }
    return chain;
}

void build_consensus(const std::vector<Pt>& chain, const std::vector<std::string>& cons,
                     const std::vector<std::string>& sample, const std::vector<size_t>& int_cons,
                     std::vector<size_t>& int_sample, size_t& num_blocks, std::vector<std::string>& cons_new,
                     std::vector<size_t>& int_cons_new, std::unordered_map<int, std::string>& int_to_string) {   // :233-277
    int pc = -1, ps = -1;
    for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
        const int cc = it->first, sc = it->second;
        for (int j = pc + 1; j < cc; ++j) {
            cons_new.push_back(cons[j]);
            int_cons_new.push_back(int_cons[j]);
        }
        for (int j = ps + 1; j < sc; ++j) {
            cons_new.push_back(sample[j]);
            int_sample.push_back(num_blocks);
            int_to_string[(int)num_blocks] = sample[j];
            int_cons_new.push_back(num_blocks);
            ++num_blocks;
        }
        cons_new.push_back(cons[cc]);
        int_sample.push_back(int_cons[cc]);
        int_cons_new.push_back(int_cons[cc]);
        pc = cc;
        ps = sc;
    }
    for (int j = pc + 1; j < (int)cons.size(); ++j) {
        cons_new.push_back(cons[j]);
        int_cons_new.push_back(int_cons[j]);
    }
    for (int j = ps + 1; j < (int)sample.size(); ++j) {
        cons_new.push_back(sample[j]);
        int_sample.push_back(num_blocks);
        int_to_string[(int)num_blocks] = sample[j];
        int_cons_new.push_back(num_blocks);
        ++num_blocks;
    }
}

// ---- src/rotation.cpp (ALLOW_INVERSIONS undefined: never inverted) -------------------
std::pair<int, int> rotate_alignment(const std::vector<std::string>& cons, const std::vector<std::string>& sample) {
    std::vector<std::pair<int, int>> score(sample.size(), {-1, -1}), next(sample.size(), {-1, -1});
    std::pair<int, int> best(0, 0);
    const int match = 5, gap = 1, mismatch = 2;
    for (size_t i = 0; i < cons.size(); ++i) {
        for (size_t j = 0; j < sample.size(); ++j) {
            const size_t up = j == 0 ? sample.size() - 1 : j - 1, diag = up, left = j;
            int lv = score[left].first - gap;
            int dv = score[diag].first;
            int uv = j == 0 ? -1 : next[up].first - gap;
            dv = cons[i] == sample[j] ? dv + match : dv - mismatch;
            if (dv >= lv) {
                if (dv >= uv) next[j] = {dv, score[diag].second == -1 ? (int)j : score[diag].second};
                else next[j] = {uv, j == 0 ? -1 : next[up].second};
            } else {
                if (lv >= uv) next[j] = {lv, score[left].second};
                else next[j] = {uv, j == 0 ? -1 : next[up].second};
            }
            if (next[j].first > best.first) best = next[j];
        }
        score = next;
    }
    return best;
}

std::vector<std::string> rotate_sample(const std::vector<std::string>& cons, std::vector<std::string>& sample,
                                       std::vector<int>& strand, std::vector<size_t>& numbers, int& rotation_index) {
    const int rotate = rotate_alignment(cons, sample).second;
    rotation_index = (int)((sample.size() - rotate) % sample.size());
    std::vector<std::string> out;
    std::vector<int> ns;
    std::vector<size_t> nn;
    for (size_t i = 0; i < sample.size(); ++i) {
        const size_t k = (i + rotate) % sample.size();
        out.push_back(sample[k]);
        ns.push_back(strand[k]);
        nn.push_back(numbers[k]);
    }
    strand = ns;
    numbers = nn;
    return out;
}

// ---- the PanGraph model (src/panman.cpp:6200-6476) -----------------------------------
template <class V>
using ByNumber = std::unordered_map<size_t, std::vector<V>>;
template <class V>
using BySeq = std::unordered_map<std::string, ByNumber<V>>;

struct Pangraph {
    std::unordered_map<std::string, std::vector<std::string>> paths;
    std::unordered_map<std::string, std::vector<int>> strand_paths;
    std::unordered_map<std::string, std::vector<size_t>> block_numbers;
    std::unordered_map<std::string, int> circular, rotation;
    std::unordered_map<std::string, bool> inverted;
    std::unordered_map<std::string, std::string> consensus;
    std::unordered_map<std::string, std::vector<std::pair<size_t, size_t>>> gaps;
    std::unordered_map<std::string, BySeq<std::pair<size_t, std::string>>> subs;
    std::unordered_map<std::string, BySeq<std::tuple<size_t, size_t, std::string>>> ins;
    std::unordered_map<std::string, BySeq<std::pair<size_t, size_t>>> dels;
    std::unordered_map<std::string, std::vector<size_t>> int_sequences;
    std::vector<size_t> topo;
    std::unordered_map<size_t, std::string> int_to_string_id;
};

bool load_pangraph(const Json& d, Pangraph& pg, std::string& err) {
    bool circ = false;
    const Json& paths = d["paths"];
    for (size_t i = 0; i < paths.size(); ++i) {
        const Json& p = paths[i];
        const std::string& name = p["name"].as_string();
        const Json& bl = p["blocks"];
        auto& path = pg.paths[name];
        auto& strands = pg.strand_paths[name];
        for (size_t j = 0; j < bl.size(); ++j) {
            path.push_back(bl[j]["id"].as_string());
            strands.push_back(bl[j]["strand"].as_bool());
        }
        if (p["circular"].as_bool()) {
            circ = true;
            pg.circular[name] = -(int)p["offset"].as_int();
        }
    }
    std::unordered_map<std::string, int> block_size;
    const Json& blocks = d["blocks"];
    for (size_t i = 0; i < blocks.size(); ++i) {
        const Json& b = blocks[i];
        const std::string& id = b["id"].as_string();
        const std::string seq = upper(b["sequence"].as_string());
        pg.consensus[id] = seq;
        block_size[id] = (int)seq.size();
        for (const auto& kv : b["gaps"].obj) {   // getMemberNames: sorted keys
            char* end = nullptr;
            const long pos = std::strtol(kv.first.c_str(), &end, 10);
            if (end == kv.first.c_str()) {
                err = "block " + id + ": gap key '" + kv.first + "' is not a position";
                return false;
            }
            pg.gaps[id].emplace_back((size_t)pos, (size_t)kv.second.as_int());
        }
        const Json& mut = b["mutate"];
        for (size_t j = 0; j < mut.size(); ++j) {
            const std::string& sn = mut[j][0]["name"].as_string();
            const size_t num = (size_t)mut[j][0]["number"].as_int();
            auto& lst = pg.subs[id][sn][num];
            for (size_t k = 0; k < mut[j][1].size(); ++k)
                lst.emplace_back((size_t)mut[j][1][k][0].as_int(), upper(mut[j][1][k][1].as_string()));
        }
        const Json& ins = b["insert"];
        for (size_t j = 0; j < ins.size(); ++j) {
            const std::string& sn = ins[j][0]["name"].as_string();
            const size_t num = (size_t)ins[j][0]["number"].as_int();
            auto& lst = pg.ins[id][sn][num];
            for (size_t k = 0; k < ins[j][1].size(); ++k)
                lst.emplace_back((size_t)ins[j][1][k][0][0].as_int(), (size_t)ins[j][1][k][0][1].as_int(),
                                 upper(ins[j][1][k][1].as_string()));
        }
        const Json& del = b["delete"];
        for (size_t j = 0; j < del.size(); ++j) {
            const std::string& sn = del[j][0]["name"].as_string();
            const size_t num = (size_t)del[j][0]["number"].as_int();
            auto& lst = pg.dels[id][sn][num];
            for (size_t k = 0; k < del[j][1].size(); ++k)
                lst.emplace_back((size_t)del[j][1][k][0].as_int(), (size_t)del[j][1][k][1].as_int());
        }
    }
    // block numbers (and rotation of circular paths against the first one)
    if (circ) {
        std::vector<std::string> base;
        int seq_count = 0;
        for (auto& p : pg.paths) {
            std::unordered_map<std::string, size_t> count;
            auto& numbers = pg.block_numbers[p.first];
            for (const auto& blk : p.second) {
                numbers.push_back(count[blk] + 1);
                ++count[blk];
            }
            if (seq_count == 0) {
                pg.inverted[p.first] = false;
                pg.rotation[p.first] = 0;
                base = p.second;
            } else {
                std::vector<std::string> sample = p.second;
                int rot = 0;
                if (sample.empty()) {
                    err = "empty circular path " + p.first;
                    return false;
                }
                auto rotated = rotate_sample(base, sample, pg.strand_paths[p.first], numbers, rot);
                pg.inverted[p.first] = false;
                pg.rotation[p.first] = rot;
                p.second = rotated;
            }
            ++seq_count;
        }
    } else {
        for (auto& p : pg.paths) {
            std::unordered_map<std::string, size_t> count;
            pg.inverted[p.first] = false;
            pg.rotation[p.first] = 0;
            for (const auto& blk : p.second) {
                pg.block_numbers[p.first].push_back(count[blk] + 1);
                ++count[blk];
            }
        }
    }
    (void)block_size;
    // chain the paths into one block order ("Resolving rearrangements and duplications")
    size_t num_nodes = 0;
    std::unordered_map<int, std::string> int_to_string;
    std::vector<std::string> cons;
    std::vector<size_t> int_cons;
    int seq_count = 0;
    for (const auto& p : pg.paths) {
        if (seq_count == 0) {
            for (const auto& blk : p.second) {
                cons.push_back(blk);
                int_to_string[(int)num_nodes] = blk;
                pg.int_sequences[p.first].push_back(num_nodes);
                int_cons.push_back(num_nodes);
                ++num_nodes;
            }
        } else {
            std::vector<size_t> int_sample, int_cons_new;
            std::vector<std::string> cons_new;
            const std::vector<Pt> chain = chaining(cons, p.second);
            build_consensus(chain, cons, p.second, int_cons, int_sample, num_nodes, cons_new, int_cons_new, int_to_string);
            auto& dst = pg.int_sequences[p.first];
            dst.insert(dst.end(), int_sample.begin(), int_sample.end());
            cons = cons_new;
            int_cons = int_cons_new;
        }
        ++seq_count;
    }
    std::unordered_map<int, int> order;
    int reorder = 0;
    for (size_t i : int_cons) {
        order[(int)i] = reorder;
        pg.int_to_string_id[(size_t)reorder] = int_to_string[(int)i];
        pg.topo.push_back((size_t)reorder);
        ++reorder;
    }
    for (auto& m : pg.int_sequences)
        for (auto& s : m.second) s = (size_t)order[(int)s];
    return true;
}

// oneTBB tbb_hasher(std::string) and the split-ordered list's iteration key
uint64_t tbb_order_key(const std::string& s) {
    uint64_t h = 0;
    for (char c : s) h = (uint64_t)(int64_t)c ^ (h * 0x9E3779B97F4A7C15ull);
    uint64_t r = 0;
    for (int b = 0; b < 64; ++b) r |= ((h >> b) & 1ull) << (63 - b);
    return r | 1ull;
}

struct Column {   // one nucleotide column of the PanMAT
    int32_t block, pos, gap;   // gap = -1: main position
};

using Seq = std::vector<std::pair<char, std::vector<char>>>;

int fetch_records(pm_ctx* c, std::vector<pm_mut>& recs) {
    int64_t n = 0;
    int rc = pm_mutation_count(c, &n);
    if (rc != PM_OK) return rc;
    recs.resize((size_t)n);
    return n ? pm_mutations_fetch(c, recs.data(), n, &n) : PM_OK;
}

std::vector<uint8_t> pack4(const std::vector<uint8_t>& codes) {
    std::vector<uint8_t> out((codes.size() + 1) / 2, 0);
    for (size_t s = 0; s < codes.size(); ++s) out[s / 2] |= (uint8_t)(codes[s] << (4 * (s & 1)));
    return out;
}

struct Tup {
    int32_t block, pos, gap;
    uint8_t type, code;
};

// NucMut runs (src/panman.cpp:1236-1272): same rules as the reroot driver.
void group(std::vector<Tup>& v, bool gap, PanmanTree& out) {
    std::sort(v.begin(), v.end(), [](const Tup& a, const Tup& b) {
        return std::tie(a.block, a.pos, a.gap) < std::tie(b.block, b.pos, b.gap);
    });
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

std::vector<uint32_t> encode_block(const std::string& seq) {   // Block(i, seq), src/panman.cpp:246-257
    std::vector<uint32_t> w;
    for (size_t i = 0; i < seq.size(); i += 8) {
        uint32_t x = 0;
        for (size_t j = i; j < std::min(i + 8, seq.size()); ++j) x ^= (uint32_t)code_of(seq[j]) << (4 * (7 - (j - i)));
        w.push_back(x);
    }
    return w;
}

int build(pm_ctx* c, const char* json_text, const char* newick_c, const char* ref_c, PanmanTree& out) {
    std::string err;
    Json doc;
    if (!json_parse(json_text, doc, err)) return fail(c, PM_ERR_ARG, "PanGraph JSON: " + err);
    Pangraph pg;
    if (!load_pangraph(doc, pg, err)) return fail(c, PM_ERR_ARG, err);
    std::string newick(newick_c);
    const size_t nl = newick.find('\n');
    if (nl != std::string::npos) newick.resize(nl);
    Topology t;
    if (!parse_topology(newick, t, err)) return fail(c, PM_ERR_ARG, "Newick: " + err);
    const std::string reference = ref_c ? ref_c : "";
    const int32_t N = (int32_t)t.name.size();
    bool polytomy = false;
    for (const auto& k : t.kids) polytomy |= k.size() > 2;   // hasPolytomy (:621-631)

    // aligned block presence / strands per sequence (getAlignedSequences, :6427-6465)
    const std::vector<size_t>& topo = pg.topo;
    const size_t T = topo.size();
    std::unordered_map<std::string, std::vector<int>> aligned, aligned_strand;
    for (const auto& p : pg.int_sequences) {
        auto& a = aligned[p.first];
        size_t p1 = 0, p2 = 0;
        while (p1 < T && p2 < p.second.size()) {
            if (topo[p1] == p.second[p2]) {
                a.push_back((int)topo[p1]);
                ++p2;
            } else {
                a.push_back(-1);
            }
            ++p1;
        }
        a.resize(T, -1);
    }
    for (const auto& p : pg.int_sequences) {
        auto& a = aligned_strand[p.first];
        const auto& sp = pg.strand_paths[p.first];
        size_t p1 = 0, p2 = 0;
        while (p1 < T && p2 < p.second.size()) {
            if (topo[p1] == p.second[p2]) {
                a.push_back(p2 < sp.size() ? sp[p2] : 0);
                ++p2;
            } else {
                a.push_back(-1);
            }
            ++p1;
        }
        a.resize(T, -1);
    }
    // rows: the aligned sequences in their container order; tree leaves map to them by name
    std::vector<std::string> row_name;
    std::unordered_map<std::string, int32_t> row_of;
    for (const auto& u : aligned) {
        row_of[u.first] = (int32_t)row_name.size();
        row_name.push_back(u.first);
    }
    const int32_t R = (int32_t)row_name.size();
    std::vector<int32_t> node_row(N, -1);
    for (int32_t v = 0; v < N; ++v)
        if (t.kids[v].empty()) {
            auto it = row_of.find(t.name[v]);
            if (it != row_of.end()) node_row[v] = it->second;
        }
    // blockCounts (:984-997): the "number" of each present block of each sequence
    std::vector<std::vector<size_t>> block_count(R, std::vector<size_t>(T, 0));
    for (int32_t r = 0; r < R; ++r) {
        const auto& a = aligned[row_name[r]];
        const auto& nums = pg.block_numbers[row_name[r]];
        size_t ptr = 0;
        for (size_t i = 0; i < T; ++i)
            if (a[i] != -1) {
                if (ptr >= nums.size()) return fail(c, PM_ERR_ARG, "sequence " + row_name[r] + ": block numbers exhausted");
                block_count[r][i] = nums[ptr++];
            }
    }

    pm_tree tree{};
    std::vector<int32_t> off(N + 1, 0), idx;
    for (int32_t v = 0; v < N; ++v) {
        idx.insert(idx.end(), t.kids[v].begin(), t.kids[v].end());
        off[v + 1] = (int32_t)idx.size();
    }
    tree.num_nodes = N;
    tree.root = t.root;
    tree.child_offsets = off.data();
    tree.child_index = idx.data();
    int rc = pm_tree_upload(c, &tree);
    if (rc != PM_OK) return rc;

    // ---- block mutations (:870-982): one column per block, every aligned sequence present
    std::vector<std::vector<std::pair<int32_t, uint8_t>>> bmuts(N);
    {
        const int64_t stride = ((int64_t)T + 1) / 2;
        std::vector<uint8_t> codes((size_t)std::max(R, 1) * std::max<int64_t>(stride, 1), 0);
        std::vector<uint8_t> forced(T, 0);
        bool any_forced = false;
        for (size_t i = 0; i < T; ++i) {
            for (int32_t r = 0; r < R; ++r) {
                const int a = aligned[row_name[r]][i];
                const uint8_t code = a == -1 ? 0 : (aligned_strand[row_name[r]][i] ? 1 : 2);
                codes[(size_t)r * stride + i / 2] |= (uint8_t)(code << (4 * (i & 1)));
            }
            if (!reference.empty()) {   // last match in alignedSequences' (std) order
                int def = -1;
                for (const auto& u : aligned)
                    if (u.first.find(reference) != std::string::npos)
                        def = u.second[i] == -1 ? 0 : (aligned_strand[u.first][i] ? 1 : 2);
                if (def >= 0) {
                    forced[i] = (uint8_t)def;
                    any_forced = true;
                }
            }
        }
        // blocks without a forcing sequence keep the default rule: run them separately
        std::vector<size_t> cols[2];
        for (size_t i = 0; i < T; ++i) {
            bool f = false;
            if (any_forced) {
                for (const auto& u : aligned)
                    if (u.first.find(reference) != std::string::npos) f = true;
            }
            cols[f ? 1 : 0].push_back(i);
        }
        for (int f = 0; f < 2 && T > 0; ++f) {
            const auto& cs = cols[f];
            if (cs.empty()) continue;
            const int64_t S = (int64_t)cs.size(), st = (S + 1) / 2;
            std::vector<uint8_t> sub((size_t)std::max(R, 1) * st, 0), fc(cs.size());
            for (int32_t r = 0; r < R; ++r)
                for (int64_t s = 0; s < S; ++s) {
                    const size_t i = cs[s];
                    const uint8_t code = (codes[(size_t)r * stride + i / 2] >> (4 * (i & 1))) & 15;
                    sub[(size_t)r * st + s / 2] |= (uint8_t)(code << (4 * (s & 1)));
                }
            for (int64_t s = 0; s < S; ++s) fc[s] = forced[cs[s]];
            std::vector<uint8_t> cons_p = pack4(std::vector<uint8_t>(cs.size(), 0)), forced_p = pack4(fc);
            std::vector<pm_mut> recs;
            if ((rc = pm_leaves_upload(c, S, sub.data(), st, node_row.data(), nullptr, 0)) != PM_OK ||
                (rc = pm_sites_upload(c, cons_p.data(), f ? forced_p.data() : nullptr)) != PM_OK ||
                (rc = pm_run(c, polytomy ? PM_MODE_BLOCK_SANKOFF : PM_MODE_BLOCK_FITCH)) != PM_OK ||
                (rc = fetch_records(c, recs)) != PM_OK)
                return rc;
            for (const pm_mut& m : recs)
                bmuts[m.node].emplace_back((int32_t)cs[m.site_info >> 8], (uint8_t)(m.site_info & 0xFF));
        }
    }

    // ---- per-block sequences of every present row (:1005-1044) and the column list
    std::vector<Column> columns;
    std::vector<uint8_t> col_cons;                    // root parent code
    std::vector<std::vector<uint8_t>> leaf_codes(R);  // per row, per column
    std::vector<std::vector<uint8_t>> leaf_pres(R);
    std::vector<int32_t> col_forced;                  // forced code, -1 none
    out.block_primary.clear();
    for (size_t i = 0; i < T; ++i) {
        const std::string& sid = pg.int_to_string_id[topo[i]];
        const std::string& cseq = pg.consensus[sid];
        Seq base(cseq.size() + 1, {'-', {}});
        for (size_t j = 0; j < cseq.size(); ++j) base[j].first = cseq[j];
        for (const auto& g : pg.gaps[sid]) {
            if (g.first >= base.size()) return fail(c, PM_ERR_ARG, "block " + sid + ": gap position beyond the block");
            base[g.first].second.resize(g.second, '-');
        }
        // this block's sequences, in row order; absent rows stay empty
        std::vector<Seq> rows(R);
        std::vector<char> has(R, 0);
        for (int32_t r = 0; r < R; ++r) {
            if (aligned[row_name[r]][i] == -1) continue;
            Seq s = base;
            const size_t num = block_count[r][i];
            auto sit = pg.subs.find(sid);
            if (sit != pg.subs.end()) {
                auto a = sit->second.find(row_name[r]);
                if (a != sit->second.end()) {
                    auto b = a->second.find(num);
                    if (b != a->second.end())
                        for (const auto& v : b->second) {
                            if (v.first < 1 || v.first > s.size() || v.second.empty())
                                return fail(c, PM_ERR_ARG, "block " + sid + ": substitution out of range");
                            s[v.first - 1].first = v.second[0];
                        }
                }
            }
            auto iit = pg.ins.find(sid);
            if (iit != pg.ins.end()) {
                auto a = iit->second.find(row_name[r]);
                if (a != iit->second.end()) {
                    auto b = a->second.find(num);
                    if (b != a->second.end())
                        for (const auto& v : b->second) {
                            const size_t p = std::get<0>(v), o = std::get<1>(v);
                            const std::string& str = std::get<2>(v);
                            if (p >= s.size() || o + str.size() > s[p].second.size())
                                return fail(c, PM_ERR_ARG, "block " + sid + ": insertion outside its gap slots");
                            for (size_t j = 0; j < str.size(); ++j) s[p].second[o + j] = str[j];
                        }
                }
            }
            auto dit = pg.dels.find(sid);
            if (dit != pg.dels.end()) {
                auto a = dit->second.find(row_name[r]);
                if (a != dit->second.end()) {
                    auto b = a->second.find(num);
                    if (b != a->second.end())
                        for (const auto& v : b->second) {
                            if (v.first < 1 || v.first + v.second - 1 > s.size())
                                return fail(c, PM_ERR_ARG, "block " + sid + ": deletion out of range");
                            for (size_t j = v.first; j < v.first + v.second; ++j) s[j - 1].first = '-';
                        }
                }
            }
            rows[r] = std::move(s);
            has[r] = 1;
        }
        // forcing sequence of this block: the last present row in TBB order (main columns:
        // any row when no reference is given, :1131-1138) / the last reference match
        int32_t last_any = -1, last_ref = -1;
        uint64_t key_any = 0, key_ref = 0;
        for (int32_t r = 0; r < R; ++r) {
            if (!has[r]) continue;
            const uint64_t k = tbb_order_key(row_name[r]);
            if (last_any < 0 || k > key_any) { last_any = r; key_any = k; }
            if (!reference.empty() && row_name[r].find(reference) != std::string::npos && (last_ref < 0 || k > key_ref)) {
                last_ref = r;
                key_ref = k;
            }
        }
        auto add_col = [&](int32_t j, int32_t k, char cons_char, int32_t force_row) {
            columns.push_back(Column{(int32_t)i, j, k});
            col_cons.push_back(code_of(cons_char));
            for (int32_t r = 0; r < R; ++r) {
                char ch = '-';
                if (has[r]) ch = k < 0 ? rows[r][j].first : rows[r][j].second[k];
                leaf_codes[r].push_back(ch != '-' ? code_of(ch) : 0);
                leaf_pres[r].push_back(has[r]);
            }
            if (force_row >= 0) {
                const char ch = k < 0 ? rows[force_row][j].first : rows[force_row][j].second[k];
                col_forced.push_back(ch != '-' ? code_of(ch) : 0);
            } else {
                col_forced.push_back(-1);
            }
        };
        const int32_t main_force = polytomy ? last_ref : (reference.empty() ? last_any : last_ref);
        for (size_t j = 0; j < base.size(); ++j) {
            for (size_t k = 0; k < base[j].second.size(); ++k) add_col((int32_t)j, (int32_t)k, '-', last_ref);
            add_col((int32_t)j, -1, base[j].first, main_force);
        }
    }

    // ---- nucleotide columns on the device: forced and unforced columns as two runs
    const int mode = polytomy ? PM_MODE_SANKOFF : PM_MODE_FITCH;
    std::vector<std::vector<Tup>> main_t(N), gap_t(N);
    for (int f = 0; f < 2; ++f) {
        std::vector<int64_t> cs;
        for (size_t s = 0; s < columns.size(); ++s)
            if ((col_forced[s] >= 0) == (f == 1)) cs.push_back((int64_t)s);
        for (size_t c0 = 0; c0 < cs.size(); c0 += ((size_t)1 << 23)) {   // record format: < 2^24 sites per run
            const int64_t S = (int64_t)std::min(cs.size() - c0, (size_t)1 << 23);
            const int64_t st = (S + 1) / 2, pst = (S + 7) / 8;
            std::vector<uint8_t> codes((size_t)std::max(R, 1) * st, 0), pres((size_t)std::max(R, 1) * pst, 0);
            std::vector<uint8_t> cons_c(S), forced_c(S);
            for (int64_t s = 0; s < S; ++s) {
                const int64_t col = cs[c0 + s];
                cons_c[s] = col_cons[col];
                forced_c[s] = f ? (uint8_t)col_forced[col] : 0;
                for (int32_t r = 0; r < R; ++r) {
                    codes[(size_t)r * st + s / 2] |= (uint8_t)(leaf_codes[r][col] << (4 * (s & 1)));
                    if (leaf_pres[r][col]) pres[(size_t)r * pst + s / 8] |= (uint8_t)(1u << (s & 7));
                }
            }
            const std::vector<uint8_t> cons_p = pack4(cons_c), forced_p = pack4(forced_c);
            std::vector<pm_mut> recs;
            if ((rc = pm_leaves_upload(c, S, codes.data(), st, node_row.data(), pres.data(), pst)) != PM_OK ||
                (rc = pm_sites_upload(c, cons_p.data(), f ? forced_p.data() : nullptr)) != PM_OK ||
                (rc = pm_run(c, mode)) != PM_OK || (rc = fetch_records(c, recs)) != PM_OK)
                return rc;
            for (const pm_mut& m : recs) {
                const Column& col = columns[cs[c0 + (m.site_info >> 8)]];
                const Tup tu{col.block, col.pos, col.gap, (uint8_t)((m.site_info >> 4) & 15), (uint8_t)(m.site_info & 15)};
                (col.gap < 0 ? main_t : gap_t)[m.node].push_back(tu);
            }
        }
    }

    // ---- the PanMAT
    out.num_nodes = N;
    out.root = t.root;
    out.child_off = off;
    out.child_idx = idx;
    out.names_blob.clear();
    for (int32_t v = 0; v < N; ++v) {
        out.names_blob += t.name[v];
        out.names_blob.push_back('\0');
    }
    out.length = t.length;
    out.newick = newick_of(t);
    out.block_seq_off.assign(1, 0);
    out.gap_off.assign(1, 0);
    for (size_t i = 0; i < T; ++i) {
        const std::string& sid = pg.int_to_string_id[topo[i]];
        const std::vector<uint32_t> w = encode_block(pg.consensus[sid]);
        out.block_primary.push_back((int32_t)i);
        out.block_seq.insert(out.block_seq.end(), w.begin(), w.end());
        out.block_seq_off.push_back((int64_t)out.block_seq.size());
        out.gap_primary.push_back((int32_t)i);
        for (const auto& g : pg.gaps[sid]) {
            out.gap_pos.push_back((uint32_t)g.first);
            out.gap_len.push_back((uint32_t)g.second);
        }
        out.gap_off.push_back((int64_t)out.gap_pos.size());
    }
    out.bm_off.assign(N + 1, 0);
    out.nm_off.assign(N + 1, 0);
    for (int32_t v = 0; v < N; ++v) {
        auto& bl = bmuts[v];
        std::sort(bl.begin(), bl.end());   // block order (the reference's is TBB-scheduled)
        for (auto& bm : bl) {
            const int type = bm.second >> 4, code = bm.second & 15;
            out.bm_primary.push_back(bm.first);
            out.bm_info.push_back(type == PM_MUT_NI ? 1 : 0);
            out.bm_inv.push_back(type == PM_MUT_NI ? code == 2 : type == PM_MUT_NS);
        }
        out.bm_off[v + 1] = (int64_t)out.bm_primary.size();
        group(main_t[v], false, out);
        group(gap_t[v], true, out);
        out.nm_off[v + 1] = (int64_t)out.nm_primary.size();
    }
    out.circular.assign(N, -1);
    out.rotation.assign(N, 0);
    out.inverted.assign(N, 0);
    for (int32_t v = 0; v < N; ++v) {
        auto a = pg.circular.find(t.name[v]);
        if (a != pg.circular.end()) out.circular[v] = a->second;
        auto b = pg.rotation.find(t.name[v]);
        if (b != pg.rotation.end()) out.rotation[v] = b->second;
        auto d = pg.inverted.find(t.name[v]);
        if (d != pg.inverted.end()) out.inverted[v] = d->second;
    }
    return PM_OK;
}

}  // namespace
}  // namespace pm

extern "C" int pm_pangraph_build(pm_ctx* c, const char* json, const char* newick, const char* reference, pm_panman** out) {
    if (!c || !json || !newick || !out) return PM_ERR_ARG;
    *out = nullptr;
    (void)hipSetDevice(c->device);
    auto* res = new pm_panman();
    res->trees.resize(1);
    const int rc = pm::build(c, json, newick, reference, res->trees[0]);
    if (rc != PM_OK) {
        delete res;
        return rc;
    }
    *out = res;
    return PM_OK;
}
