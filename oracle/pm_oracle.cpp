// pm_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's small-parsimony path (faithokamoto/panman
// @ 2025-03-21).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / the timed
// CPU baseline.  The product path (panman_amd/libpanman_amd.so) never links,
// loads or calls it.
//
// Fidelity: every routine restates the reference algorithm with the
// reference's own data structures where they shape the cost (per-column
// std::unordered_map<std::string,...> keyed by node name, recursion over
// Node* children), so that its timing is a faithful stand-in for the
// reference's CPU path ("cpu_baseline.kind = port").
//
// Parity pin: the reference itself is unbuildable in this image without
// stand-ins for oneTBB / capnp / boost / jsoncpp headers (forbidden by the
// task rules), so this restatement is pinned against the known-answer tests
// the survey recorded from the compiled reference (SURVEY.md §8a', committed
// as tests/golden/kats.json) -- see DESIGN.md "Oracle".
//
// Reference anchors (file:line under /root/reference):
//   codes            src/panman.cpp:41-113 (getNucleotideFromCode / getCodeFromNucleotide)
//   complement       src/panman.cpp:171-204
//   Newick           src/panman.cpp:265-308 (stringSplit, stripString), :310-450
//   Fitch F1-F3      src/fitchSankoff.cpp:30-56, 96-129, 131-171
//   Sankoff S1-S3    src/fitchSankoff.cpp:359-405, 487-531, 676-703
//   block B1         src/fitchSankoff.cpp:224-308
//   block B2         src/fitchSankoff.cpp:707-818
//   M1 MSA driver    src/panman.cpp:1274-1466
//   M2 low-mem       src/panman.cpp:1467-1649 (readFastaInBatch :677-724)
//   E1 grouping      src/panman.cpp:1445-1466, src/panman.hpp:100-151

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stack>
#include <queue>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kSankoffInf = 100000001;      // src/common.hpp:16
constexpr int kNoDefault = 1 << 28;         // src/panman.hpp:851 default argument

enum NucType { NS = 0, ND = 1, NI = 2 };    // src/panman.hpp:46-61
enum BlockType { BD = 0, BI = 1 };          // src/panman.hpp:63-72

// ---------------------------------------------------------------- codes ----
int code_of(char c) {
    switch (c) {
        case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
        case 'R': return 5;  case 'Y': return 10; case 'S': return 6;  case 'W': return 9;
        case 'K': return 12; case 'M': return 3;  case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7;  case 'N': return 15;
        default: return 0;
    }
}

char char_of(int code) {
    static const char tab[16] = {'-', 'A', 'C', 'M', 'G', 'R', 'S', 'V',
                                 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
    return (code >= 0 && code < 16) ? tab[code] : '-';
}

char complement_of(char c) {
    switch (c) {
        case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
        case 'R': return 'Y'; case 'Y': return 'R'; case 'S': return 'S'; case 'W': return 'W';
        case 'K': return 'M'; case 'M': return 'K'; case 'B': return 'V'; case 'D': return 'H';
        case 'H': return 'D'; case 'V': return 'B';
        default: return 'N';
    }
}

// index of the highest set bit, as the reference's shift loop computes it
int log2_state(int s) {
    int code = 0;
    while (s > 0) { s >>= 1; ++code; }
    return code - 1;
}

int lowest_bit(int s) {
    int cur = 1;
    while (!(s & cur)) cur <<= 1;
    return cur;
}

// ----------------------------------------------------------------- tree ----
struct ONode {
    std::string id;
    ONode* parent = nullptr;
    std::vector<ONode*> children;
};

struct OTree {
    std::vector<ONode*> owned;
    ONode* root = nullptr;
    std::map<std::string, ONode*> all;   // name order, like Tree::allNodes
    size_t internal_counter = 0;
    ~OTree() { for (auto* n : owned) delete n; }
    ONode* make(const std::string& id, ONode* par) {
        ONode* n = new ONode();
        n->id = id;
        n->parent = par;
        if (par) par->children.push_back(n);
        owned.push_back(n);
        return n;
    }
};

// Quote-aware split that keeps ' ... ' groups whole (src/panman.cpp:265-296).
void split_keep_quotes(const std::string& s, char delim, std::vector<std::string>& out) {
    size_t start = 0, end = 0, hold = 0;
    while ((end = s.find(delim, start)) != std::string::npos) {
        if (end >= s.size()) break;
        if (hold == 0) {
            std::string piece = s.substr(start, end - start);
            if (std::count(piece.begin(), piece.end(), '\'') % 2 == 1) hold = start;
            else out.push_back(piece);
        } else {
            std::string piece = s.substr(hold, end - hold);
            if (std::count(piece.begin(), piece.end(), '\'') % 2 == 0) {
                hold = 0;
                out.push_back(piece);
            }
        }
        start = end + 1;
    }
    std::string tail = s.substr(start);
    if (!tail.empty()) out.push_back(tail);
}

std::string strip_spaces(std::string s) {
    while (!s.empty() && s.back() == ' ') s.pop_back();
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i] != ' ') return s.substr(i);
    return s;
}

// Newick -> tree, internal nodes named node_<k> in order of '(' (src/panman.cpp:310-450,
// src/panman.hpp:793-795).  Branch lengths are parsed but irrelevant to this path.
bool parse_newick(const std::string& text, OTree& t, std::string& err) {
    std::string nwk = strip_spaces(text);
    std::vector<std::string> pieces;
    split_keep_quotes(nwk, ',', pieces);
    std::vector<std::string> leaves;
    std::vector<size_t> opens, closes;
    long level = 0;
    for (const auto& s : pieces) {
        size_t no = 0, nc = 0;
        bool stop = false, in_quote = false, quoted = false;
        std::string leaf;
        for (char c : s) {
            if (in_quote) {
                leaf += c;
                if (c == '\'') in_quote = false;
            } else if (c == '\'') {
                in_quote = true; quoted = true; leaf += c;
            } else if (c == ':') {
                stop = true;
            } else if (c == '(') {
                ++no; ++level;
            } else if (c == ')') {
                stop = true; ++nc; --level;
            } else if (!stop) {
                leaf += c;
            }
        }
        if (quoted && leaf.size() >= 2 && leaf.front() == '\'' && leaf.back() == '\'')
            leaf = leaf.substr(1, leaf.size() - 2);
        leaves.push_back(leaf);
        opens.push_back(no);
        closes.push_back(nc);
    }
    if (level != 0) { err = "incorrect Newick format"; return false; }
    std::stack<ONode*> stack;
    for (size_t i = 0; i < leaves.size(); ++i) {
        for (size_t j = 0; j < opens[i]; ++j) {
            std::string nid = "node_" + std::to_string(++t.internal_counter);
            ONode* n = t.make(nid, stack.empty() ? nullptr : stack.top());
            if (stack.empty()) t.root = n;
            t.all[nid] = n;
            stack.push(n);
        }
        if (stack.empty()) { err = "leaf outside any clade"; return false; }
        ONode* lf = t.make(leaves[i], stack.top());
        t.all[leaves[i]] = lf;
        for (size_t j = 0; j < closes[i]; ++j) stack.pop();
    }
    if (!t.root) { err = "empty tree"; return false; }
    return true;
}

// ------------------------------------------------------ nucleotide Fitch ----
using StateMap = std::unordered_map<std::string, int>;
using CostMap = std::unordered_map<std::string, std::vector<int>>;
using NucMutMap = std::unordered_map<std::string, std::pair<int, char>>;
using BlockMutMap = std::unordered_map<std::string, std::pair<int, bool>>;

// F1: src/fitchSankoff.cpp:30-56
int fitch_up(ONode* n, StateMap& st, int ref_state) {
    if (n->children.empty()) {
        auto it = st.find(n->id);
        if (it == st.end()) return st[n->id] = 0;    // absent leaf poisons the AND
        return it->second;
    }
    std::vector<int> kids;
    kids.reserve(n->children.size());
    for (ONode* c : n->children) kids.push_back(fitch_up(c, st, ref_state));
    if (n->parent == nullptr && ref_state != -1) return st[n->id] = ref_state;
    int both = kids[0], either = 0;
    for (int k : kids) { either |= k; both &= k; }
    return st[n->id] = both ? both : either;
}

// F2: src/fitchSankoff.cpp:96-129
void fitch_down(ONode* n, ONode* root, StateMap& st, int parent_state, int forced) {
    if (n == root && forced != kNoDefault) {
        st[n->id] = forced;
    } else {
        int own = st[n->id];
        if (own == 0) return;
        if (n == root) st[n->id] = lowest_bit(own);
        else if (parent_state & own) st[n->id] = parent_state;
        else st[n->id] = lowest_bit(own);
    }
    int mine = st[n->id];
    for (ONode* c : n->children) fitch_down(c, root, st, mine, kNoDefault);
}

// F3: src/fitchSankoff.cpp:131-171
void fitch_assign(ONode* n, StateMap& st, NucMutMap& muts, int parent_state) {
    int own = st[n->id];
    if (own == 0) return;
    if (parent_state != own) {
        if (parent_state == 1) muts[n->id] = {NI, char_of(log2_state(own))};
        else if (own == 1) muts[n->id] = {ND, '-'};
        else muts[n->id] = {NS, char_of(log2_state(own))};
    }
    for (ONode* c : n->children) fitch_assign(c, st, muts, own);
}

// ---------------------------------------------------- nucleotide Sankoff ----
// S1: src/fitchSankoff.cpp:359-405
std::vector<int> sankoff_up(ONode* n, CostMap& cs) {
    if (n->children.empty()) {
        if (cs.find(n->id) == cs.end()) cs[n->id] = std::vector<int>(16, kSankoffInf);
        return cs[n->id];
    }
    std::vector<std::vector<int>> kids;
    for (ONode* c : n->children) kids.push_back(sankoff_up(c, cs));
    bool any_finite = false;
    for (auto& k : kids)
        for (int v : k)
            if (v < kSankoffInf) { any_finite = true; break; }
    if (!any_finite) return cs[n->id] = std::vector<int>(16, kSankoffInf);
    std::vector<int> cost(16, 0);
    for (int i = 0; i < 16; ++i) {
        for (auto& k : kids) {
            int best = kSankoffInf;
            for (int j = 0; j < 16; ++j) best = std::min(best, (i != j) + k[j]);
            if (best < kSankoffInf) cost[i] += best;
        }
    }
    return cs[n->id] = cost;
}

// S2: src/fitchSankoff.cpp:487-531
void sankoff_down(ONode* n, ONode* root, CostMap& cs, StateMap& st, int parent_ptr, int forced) {
    if (n == root && forced != kNoDefault) {
        st[n->id] = forced;
    } else if (n == root) {
        int best = kSankoffInf, arg = -1;
        const auto& c = cs[n->id];
        for (int i = 0; i < 16; ++i)
            if (c[i] < best) { best = c[i]; arg = i; }
        st[n->id] = arg;      // reference asserts arg != -1 (all-absent column)
    } else {
        st[n->id] = parent_ptr;
    }
    int mine = st[n->id];
    for (ONode* c : n->children) {
        if (mine == -1) { sankoff_down(c, root, cs, st, -1, kNoDefault); continue; }
        const auto& k = cs[c->id];
        int best = kSankoffInf, arg = -1;
        for (int i = 0; i < 16; ++i) {
            int v = (i != mine) + k[i];
            if (v < best) { best = v; arg = i; }
        }
        sankoff_down(c, root, cs, st, arg, kNoDefault);
    }
}

// S3: src/fitchSankoff.cpp:676-703
void sankoff_assign(ONode* n, StateMap& st, NucMutMap& muts, int parent_state) {
    int own = st[n->id];
    if (own == -1) return;
    if (parent_state != own) {
        if (parent_state == 0) muts[n->id] = {NI, char_of(own)};
        else if (own == 0) muts[n->id] = {ND, '-'};
        else muts[n->id] = {NS, char_of(own)};
    }
    for (ONode* c : n->children) sankoff_assign(c, st, muts, own);
}

// -------------------------------------------------------- block Fitch B1 ----
int block_fitch_up(ONode* n, StateMap& st) {             // :224-245
    if (n->children.empty()) {
        auto it = st.find(n->id);
        if (it == st.end()) return st[n->id] = 0;
        return it->second;
    }
    std::vector<int> kids;
    for (ONode* c : n->children) kids.push_back(block_fitch_up(c, st));
    int both = kids[0], either = 0;
    for (int k : kids) { either |= k; both &= k; }
    return st[n->id] = both ? both : either;
}

void block_fitch_down(ONode* n, ONode* root, StateMap& st, int parent_state, int forced) {  // :247-270
    if (n == root && forced != kNoDefault) {
        st[n->id] = forced;
    } else {
        int own = st[n->id];
        if (own == 0) return;
        st[n->id] = (parent_state & own) ? parent_state : lowest_bit(own);
    }
    int mine = st[n->id];
    for (ONode* c : n->children) block_fitch_down(c, root, st, mine, kNoDefault);
}

void block_fitch_assign(ONode* n, StateMap& st, BlockMutMap& muts, int parent_state) {  // :272-308
    int own = st[n->id];
    if (own == 0) return;
    if (parent_state != own) {
        if (parent_state == 1) muts[n->id] = {BI, log2_state(own) == 2};
        else if (own == 1) muts[n->id] = {BD, false};
        else muts[n->id] = {BD, true};
    }
    for (ONode* c : n->children) block_fitch_assign(c, st, muts, own);
}

// ------------------------------------------------------ block Sankoff B2 ----
std::vector<int> block_sankoff_up(ONode* n, CostMap& cs) {   // :707-735
    if (n->children.empty()) {
        if (cs.find(n->id) == cs.end()) cs[n->id] = {0, kSankoffInf, kSankoffInf};
        return cs[n->id];
    }
    std::vector<std::vector<int>> kids;
    for (ONode* c : n->children) kids.push_back(block_sankoff_up(c, cs));
    std::vector<int> cost(3, 0);
    for (int i = 0; i < 3; ++i)
        for (auto& k : kids) {
            int best = kSankoffInf;
            for (int j = 0; j < 3; ++j) best = std::min(best, (i != j) + k[j]);
            cost[i] += best;
        }
    return cs[n->id] = cost;
}

void block_sankoff_down(ONode* n, ONode* root, CostMap& cs, StateMap& st, int parent_ptr, int forced) {  // :737-786
    if (n == root && forced != kNoDefault) {
        st[n->id] = forced;
    } else if (n == root) {
        int best = kSankoffInf, arg = -1;
        const auto& c = cs[n->id];
        for (int i = 0; i < 3; ++i)
            if (c[i] < best) { best = c[i]; arg = i; }
        if (arg == -1) { st[n->id] = -1; return; }
        st[n->id] = arg;
    } else {
        bool finite = false;
        for (int v : cs[n->id]) if (v < kSankoffInf) finite = true;
        if (!finite) { st[n->id] = -1; return; }
        st[n->id] = parent_ptr;
    }
    int mine = st[n->id];
    for (ONode* c : n->children) {
        const auto& k = cs[c->id];
        int best = kSankoffInf, arg = -1;
        for (int i = 0; i < 3; ++i) {
            int v = (i != mine) + k[i];
            if (v < best) { best = v; arg = i; }
        }
        block_sankoff_down(c, root, cs, st, arg, kNoDefault);
    }
}

void block_sankoff_assign(ONode* n, StateMap& st, BlockMutMap& muts, int parent_state) {  // :788-818
    int own = st[n->id];
    if (own == -1) return;
    if (parent_state != own) {
        if (parent_state == 0) muts[n->id] = {BI, own == 2};
        else if (own == 0) muts[n->id] = {BD, false};
        else muts[n->id] = {BD, true};
    }
    for (ONode* c : n->children) block_sankoff_assign(c, st, muts, own);
}

// ------------------------------------------------------------ E1 grouping ----
// One NucMut as the reference stores it (src/panman.hpp:75-151).
struct ONucMut {
    int32_t pos;
    int32_t gap;
    uint8_t info;     // (len << 4) | type
    uint32_t nucs;    // code k at bits 4*(5-k)
};

using PosMut = std::tuple<int, int8_t, int8_t>;   // (position, type, code)

void group_runs(std::vector<PosMut>& v, std::vector<ONucMut>& out) {
    // src/panman.cpp:1445-1466
    std::sort(v.begin(), v.end());
    auto emit = [&](size_t a, size_t b) {
        ONucMut m;
        m.pos = std::get<0>(v[a]);
        m.gap = -1;
        m.info = (uint8_t)(((b - a) << 4) + std::get<1>(v[a]));
        m.nucs = 0;
        for (size_t k = a; k < b; ++k) m.nucs += (uint32_t)std::get<2>(v[k]) << (4 * (5 - (k - a)));
        out.push_back(m);
    };
    size_t start = 0;
    for (size_t i = 1; i < v.size(); ++i) {
        if (i - start == 6 || std::get<0>(v[i]) != std::get<0>(v[i - 1]) + 1 ||
            std::get<1>(v[i]) != std::get<1>(v[i - 1])) {
            emit(start, i);
            start = i;
        }
    }
    if (!v.empty()) emit(start, v.size());
}

// ------------------------------------------------------------ MSA readers ----
struct Msa {
    std::map<std::string, std::string> rows;
    size_t width = 0;
};

// M1 reader (src/panman.cpp:1285-1322), '\r'-tolerant.
bool read_msa_m1(const std::string& text, Msa& msa, std::string& err) {
    std::istringstream in(text);
    std::string line, seq, id;
    size_t width = 0;
    auto flush_named = [&](const std::string& name) {
        if (width == 0) width = seq.size();
        else if (width != seq.size()) { err = "sequence lengths don't match: " + name; return false; }
        msa.rows[name] = seq;
        return true;
    };
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        if (line[0] == '>') {
            if (!seq.empty()) {
                std::vector<std::string> sp;
                split_keep_quotes(id, '\r', sp);
                if (!flush_named(sp.empty() ? std::string() : sp[0])) return false;
            }
            std::vector<std::string> sp;
            split_keep_quotes(line, ' ', sp);
            id = sp.empty() ? std::string() : sp[0].substr(1);
            seq.clear();
        } else {
            std::vector<std::string> sp;
            split_keep_quotes(line, '\r', sp);
            seq += sp.empty() ? std::string() : sp[0];
        }
    }
    if (!seq.empty() && !flush_named(id)) return false;
    msa.width = width;
    return true;
}

// ------------------------------------------------------------ M1 / M2 ------
struct BuildOut {
    std::string consensus;
    std::map<std::string, std::vector<ONucMut>> node_muts;   // name order
    std::string root_id;
    std::string err;
};

using PerNode = std::unordered_map<std::string, std::vector<PosMut>>;

void collect(const NucMutMap& muts, int pos, PerNode& into) {
    for (auto& m : muts) into[m.first].emplace_back(pos, (int8_t)m.second.first, (int8_t)code_of(m.second.second));
}

void finish(OTree& t, PerNode& raw, BuildOut& out) {
    for (auto& kv : raw) {
        std::vector<ONucMut> recs;
        group_runs(kv.second, recs);
        out.node_muts[kv.first] = std::move(recs);
    }
    out.root_id = t.root->id;
}

// Column loop shared by M1/M2: run [lo,hi) columns, optionally on several threads
// (the reference M1 loop is sequential, src/panman.cpp:1380-1381; M2 is tbb::parallel_for,
// :1568; results are order-independent because every node's list is sorted later).
template <class Fn>
void run_columns(size_t lo, size_t hi, int threads, PerNode& raw, Fn&& body) {
    if (threads <= 1) {
        for (size_t i = lo; i < hi; ++i) body(i, raw);
        return;
    }
    std::vector<PerNode> parts(threads);
    std::atomic<size_t> next(lo);
    std::vector<std::thread> pool;
    for (int w = 0; w < threads; ++w)
        pool.emplace_back([&, w] {
            for (;;) {
                size_t i = next.fetch_add(1);
                if (i >= hi) break;
                body(i, parts[w]);
            }
        });
    for (auto& th : pool) th.join();
    for (auto& p : parts)
        for (auto& kv : p) {
            auto& dst = raw[kv.first];
            dst.insert(dst.end(), kv.second.begin(), kv.second.end());
        }
}

void build_msa_fitch(OTree& t, Msa& msa, const std::string& reference, int threads, BuildOut& out) {
    std::string consensus;
    if (!reference.empty()) {
        consensus = msa.rows[reference];
    } else {
        consensus.resize(msa.width);
        for (size_t i = 0; i < msa.width; ++i) {
            bool found = false;
            for (auto& r : msa.rows)
                if (r.second[i] != '-') { consensus[i] = r.second[i]; found = true; break; }
            if (!found) {
                // src/panman.cpp:1336-1361 drops the column from the rows but not from the
                // consensus, so the loop reads past the shortened rows: undefined behaviour.
                out.err = "all-gap column without reference (reference behaviour undefined)";
                return;
            }
        }
    }
    PerNode raw;
    run_columns(0, consensus.size(), threads, raw, [&](size_t i, PerNode& sink) {
        StateMap st;
        NucMutMap muts;
        for (const auto& r : msa.rows) {
            if (r.second[i] != '-') st.insert({r.first, 1 << code_of(r.second[i])});
            else st.insert({r.first, 1});
        }
        int ref_state = reference.empty() ? -1 : 1 << code_of(msa.rows.at(reference)[i]);
        fitch_up(t.root, st, ref_state);
        int cons_state = 1 << code_of(consensus[i]);
        fitch_down(t.root, t.root, st, cons_state, kNoDefault);
        fitch_assign(t.root, st, muts, cons_state);
        collect(muts, (int)i, sink);
    });
    out.consensus = consensus;
    finish(t, raw, out);
}

// M2 width probe (src/panman.cpp:1479-1500): only a header that follows a non-empty
// row sets the width, so the last row is never measured.
size_t m2_width(const std::string& text) {
    std::istringstream in(text);
    std::string line, seq;
    size_t width = 0;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        if (line[0] == '>') {
            if (!seq.empty() && width == 0) width = seq.size();
            seq.clear();
        } else {
            seq += line;
        }
    }
    return width;
}

// readFastaInBatch (src/panman.cpp:677-724), without the length check it also does.
void read_batch(const std::string& text, size_t start, size_t batch, Msa& msa) {
    std::istringstream in(text);
    std::string line, seq, id;
    auto put = [&](const std::string& name) {
        size_t take = start + batch > seq.size() ? seq.size() - start : batch;
        msa.rows[name] = seq.substr(start, take);
    };
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        if (line[0] == '>') {
            if (!seq.empty()) put(id);
            std::vector<std::string> sp;
            split_keep_quotes(line, ' ', sp);
            id = sp.empty() ? std::string() : sp[0].substr(1);
            seq.clear();
        } else {
            seq += line;
        }
    }
    if (!seq.empty()) put(id);
}

void build_msa_sankoff(OTree& t, const std::string& text, const std::string& reference,
                       int threads, size_t batch, BuildOut& out) {
    size_t width = m2_width(text);
    std::string consensus(width, '\0');
    PerNode raw;
    for (size_t start = 0; start < width;) {
        Msa msa;
        read_batch(text, start, batch, msa);
        size_t n = 0;
        if (!msa.rows.empty()) n = msa.rows.rbegin()->second.size();
        if (n == 0) break;
        if (!reference.empty()) {
            auto it = msa.rows.find(reference);
            if (it == msa.rows.end()) { out.err = "Reference not found in the sequence"; return; }
            for (size_t i = 0; i < n; ++i) {
                if (it->second[i] == '-') {
                    for (auto& r : msa.rows)
                        if (r.second[i] != '-') { consensus[start + i] = r.second[i]; break; }
                } else {
                    consensus[start + i] = it->second[i];
                }
            }
        } else {
            for (size_t i = 0; i < n; ++i) {
                bool found = false;
                for (auto& r : msa.rows)
                    if (r.second[i] != '-') { consensus[start + i] = r.second[i]; found = true; break; }
                if (!found) { out.err = "all-gap column without reference (reference exits)"; return; }
            }
        }
        run_columns(0, n, threads, raw, [&](size_t i, PerNode& sink) {
            CostMap cs;
            StateMap st;
            NucMutMap muts;
            for (const auto& r : msa.rows) {
                std::vector<int> v(16, kSankoffInf);
                v[r.second[i] != '-' ? code_of(r.second[i]) : 0] = 0;
                cs[r.first] = v;
            }
            int forced = -1;
            if (!reference.empty()) {
                char rc = msa.rows.at(reference)[i];
                forced = rc != '-' ? code_of(rc) : 0;
            }
            sankoff_up(t.root, cs);
            int cons_code = code_of(consensus[start + i]);
            sankoff_down(t.root, t.root, cs, st, cons_code, forced != -1 ? forced : kNoDefault);
            sankoff_assign(t.root, st, muts, cons_code);
            collect(muts, (int)(start + i), sink);
        });
        start += n;
    }
    out.consensus = consensus;
    finish(t, raw, out);
}

char* dup_string(const std::string& s) {
    char* p = (char*)std::malloc(s.size() + 1);
    std::memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    return p;
}

// Canonical text dump shared with the product's host driver (byte-identical format).
std::string dump_build(const BuildOut& b) {
    std::ostringstream os;
    if (!b.err.empty()) { os << "#error\t" << b.err << "\n"; return os.str(); }
    os << "#consensus\t" << b.consensus << "\n";
    os << "#blockmut\t" << b.root_id << "\t0\t-1\t1\t0\n";   // root BlockMut(0, BI, false)
    for (auto& kv : b.node_muts) {
        for (auto& m : kv.second) {
            char buf[96];
            std::snprintf(buf, sizeof buf, "\t%d\t%d\t%u\t%06x\n", m.pos, m.gap, (unsigned)m.info,
                          (unsigned)m.nucs);
            os << kv.first << buf;
        }
    }
    return os.str();
}

// ---------------------------------------------------------- CSR trees -------
// Bench / parity entry: a tree given as CSR with names, leaf columns as codes.
struct CsrTree {
    OTree t;
    std::vector<ONode*> by_index;
};

void csr_to_tree(int32_t n, const int32_t* child_off, const int32_t* child_idx, int32_t root,
                 const char* names, CsrTree& ct) {
    ct.by_index.assign(n, nullptr);
    const char* p = names;
    std::vector<std::string> nm(n);
    for (int32_t i = 0; i < n; ++i) { nm[i] = p; p += nm[i].size() + 1; }
    for (int32_t i = 0; i < n; ++i) {
        ONode* x = new ONode();
        x->id = nm[i];
        ct.t.owned.push_back(x);
        ct.by_index[i] = x;
        ct.t.all[x->id] = x;
    }
    for (int32_t i = 0; i < n; ++i)
        for (int32_t e = child_off[i]; e < child_off[i + 1]; ++e) {
            ONode* c = ct.by_index[child_idx[e]];
            c->parent = ct.by_index[i];
            ct.by_index[i]->children.push_back(c);
        }
    ct.t.root = ct.by_index[root];
}

}  // namespace

// ------------------------------------------------------------- R1-R3 replay ----
// Restatement of Tree::printFASTAUltraFast (src/fasta.cpp:1981-2099) with
// getNodesFromTipToRoot (:1753-1764), getBlockSequence (:1766-1787),
// printFASTAUltraFastHelper (:1789-1979) and printSequenceLinesNew (:155-254).

struct RBlockMut { int32_t primary; int32_t secondary; bool info; bool inversion; };
struct RNucMut { int32_t pos; int32_t gap; int32_t primary; int32_t secondary; uint8_t info; uint32_t nucs;
                 int length() const { return info >> 4; }
                 uint32_t type() const { return info & 0x7; }
                 int code(int i) const { return (nucs >> (4 * (5 - i))) & 0xF; } };
struct RNode { std::string id; RNode* parent = nullptr; std::vector<RNode*> children;
               std::vector<RBlockMut> bmuts; std::vector<RNucMut> nmuts; float len = 1.0f; };
struct RBlock { int32_t primary; std::vector<uint32_t> seq; };
struct RGap { int32_t primary; std::vector<uint32_t> pos, len; };
using Seq = std::vector<std::vector<std::pair<char, std::vector<char>>>>;

struct RTree {
    std::vector<std::unique_ptr<RNode>> nodes;
    RNode* root = nullptr;
    size_t internal_counter = 0;          // m_currInternalNode after the Newick parse
    std::map<std::string, RNode*> all;
    std::vector<RBlock> blocks;
    std::vector<RGap> gaps;
    std::unordered_map<std::string, int> circular, rotation;
    std::unordered_map<std::string, bool> inverted;
};

std::string print_lines(const Seq& seq, std::unordered_map<int, int>& block_len, const std::vector<bool>& exists,
                        const std::vector<bool>& strand, size_t width, bool aligned, int offset) {
    std::string line;
    for (size_t i = 0; i < exists.size(); ++i) {
        if (exists[i]) {
            if (strand[i]) {
                for (size_t j = 0; j < seq[i].size(); ++j) {
                    for (char g : seq[i][j].second) {
                        if (g != '-') line += g;
                        else if (aligned) line += '-';
                    }
                    const char m = seq[i][j].first;
                    if (m != '-' && m != 'x') line += m;
                    else if (aligned && m != 'x') line += '-';
                }
            } else {
                for (size_t j = seq[i].size(); j-- > 0;) {
                    const char m = seq[i][j].first;
                    if (m != '-' && m != 'x') line += complement_of(m);
                    else if (aligned && m != 'x') line += '-';
                    const auto& g = seq[i][j].second;
                    for (size_t k = g.size(); k-- > 0;) {
                        if (g[k] != '-') line += complement_of(g[k]);
                        else if (aligned) line += '-';
                    }
                }
            }
        } else if (aligned) {
            line.append((size_t)block_len[(int)i], '-');   // indexed by print position (:207-210)
        }
    }
    size_t start = 0;
    if (offset != 0) {
        for (size_t i = 0; i < line.size(); ++i) {
            if (line[i] != '-') {
                if (start == (size_t)offset) { start = i; break; }
                ++start;
            }
        }
    }
    std::string out;
    size_t col = 0;
    auto put = [&](char ch) {
        out += ch;
        if (++col == width) { out += '\n'; col = 0; }
    };
    for (size_t i = start; i < line.size(); ++i) put(line[i]);
    for (size_t i = 0; i < start; ++i) put(line[i]);
    return out;
}

std::string leaf_record(RTree& t, RNode* leaf, bool aligned) {
    std::vector<RNode*> path;
    for (RNode* n = leaf; n; n = n->parent) path.push_back(n);
    std::reverse(path.begin(), path.end());
    const size_t nb = t.blocks.size() + 1;
    std::vector<bool> present(nb, false);
    for (RNode* n : path)
        for (auto& m : n->bmuts) {
            if (m.info) present[m.primary] = true;
            else if (!m.inversion) present[m.primary] = false;
        }
    std::unordered_map<int, int> block_len;
    Seq seq(nb);
    std::vector<bool> exists(nb, false), strand(nb, true);
    int32_t max_id = 0;
    for (auto& b : t.blocks) {
        block_len[b.primary] = 0;
        max_id = std::max(max_id, b.primary);
        int len = 0;
        bool end = false;
        for (size_t j = 0; j < b.seq.size() && !end; ++j)
            for (int k = 0; k < 8; ++k) {
                const int code = (b.seq[j] >> (4 * (7 - k))) & 15;
                if (code == 0) { end = true; break; }
                if (present[b.primary]) seq[b.primary].push_back({char_of(code), {}});
                ++len;
            }
        if (present[b.primary]) seq[b.primary].push_back({'x', {}});
        else block_len[b.primary] += len;
    }
    seq.resize(max_id + 1);
    exists.resize(max_id + 1);
    strand.resize(max_id + 1);
    for (auto& g : t.gaps) {
        if (present[g.primary]) {
            for (size_t j = 0; j < g.pos.size(); ++j) seq[g.primary][g.pos[j]].second.resize(g.len[j], '-');
        } else {
            int len = 0;
            for (auto l : g.len) len += (int)l;
            block_len[g.primary] += len;
        }
    }
    for (RNode* n : path) {
        for (auto& m : n->bmuts) {
            if (!present[m.primary]) continue;
            if (m.info) { exists[m.primary] = true; strand[m.primary] = !m.inversion; }
            else if (m.inversion) { strand[m.primary] = !strand[m.primary]; }
            else { exists[m.primary] = false; strand[m.primary] = true; }
        }
        for (auto& m : n->nmuts) {
            if (!present[m.primary]) continue;
            const uint32_t type = m.type();
            auto& blk = seq[m.primary];
            if (type < 3) {
                for (int j = 0; j < m.length(); ++j) {
                    const char v = type == ND ? '-' : char_of(m.code(j));   // NS / NI write the code
                    if (m.gap != -1) blk[m.pos].second[m.gap + j] = v;
                    else blk[m.pos + j].first = v;
                }
            } else if (type <= 5) {
                const char v = type == 5 ? '-' : char_of(m.code(0));
                if (m.gap != -1) blk[m.pos].second[m.gap] = v;
                else blk[m.pos].first = v;
            }
        }
    }
    int offset = 0;
    if (!aligned) {
        auto it = t.circular.find(leaf->id);
        if (it != t.circular.end()) offset = it->second;
    }
    auto rit = t.rotation.find(leaf->id);
    if (rit != t.rotation.end() && rit->second != 0) {
        int ctr = -1;
        size_t at = 0;
        for (size_t i = 0; i < exists.size(); ++i) {
            if (exists[i]) ++ctr;
            if (ctr == rit->second) { at = i; break; }
        }
        std::rotate(seq.begin(), seq.begin() + at, seq.end());
        std::vector<bool> e2(exists), s2(strand);
        std::rotate(e2.begin(), e2.begin() + at, e2.end());
        std::rotate(s2.begin(), s2.begin() + at, s2.end());
        exists = e2;
        strand = s2;
    }
    auto iit = t.inverted.find(leaf->id);
    if (iit != t.inverted.end() && iit->second) {
        std::reverse(seq.begin(), seq.end());
        std::vector<bool> e2(exists.rbegin(), exists.rend()), s2(strand.rbegin(), strand.rend());
        exists = e2;
        strand = s2;
    }
    return ">" + leaf->id + "\n" + print_lines(seq, block_len, exists, strand, 70, aligned, offset) + "\n";
}

// ===================================================================== C API ==
extern "C" {

void oracle_free(void* p) { std::free(p); }

// M1 (mode 0: FILE_TYPE::MSA, Fitch) / M2 (mode 1: FILE_TYPE::MSA_OPTIMIZE, Sankoff).
// Returns the canonical dump (malloc'd; release with oracle_free).
char* oracle_msa_build(const char* newick, const char* msa_text, const char* reference, int mode,
                       int threads) {
    BuildOut out;
    OTree t;
    std::string err;
    std::string first_line(newick);
    size_t nl = first_line.find('\n');
    if (nl != std::string::npos) first_line.resize(nl);
    if (!parse_newick(first_line, t, err)) { out.err = err; return dup_string(dump_build(out)); }
    std::string ref = reference ? reference : "";
    if (mode == 0) {
        Msa msa;
        if (!read_msa_m1(msa_text, msa, err)) { out.err = err; return dup_string(dump_build(out)); }
        build_msa_fitch(t, msa, ref, threads, out);
    } else {
        build_msa_sankoff(t, msa_text, ref, threads, 20000, out);
    }
    return dup_string(dump_build(out));
}

// One column through the per-column routines on a Newick tree (KAT driver).
// algo: 0 nuc Fitch, 1 nuc Sankoff, 2 block Fitch, 3 block Sankoff.
// leaves: "name=V,name=V" -- V is a nucleotide char (algo 0/1) or a state digit
// (algo 2: 1/2/4, algo 3: 0/1/2).  Leaves not listed are absent.
// forced: refState (algo 0, forward) / defaultState (others); -1 = none.
// parent: the root's parent state passed to backward/assign (algo 0: a char code is
// converted to 1<<code by the caller, i.e. pass the state).
char* oracle_column(const char* newick, const char* leaves, int algo, int forced, int parent) {
    OTree t;
    std::string err;
    std::ostringstream os;
    if (!parse_newick(newick, t, err)) { os << "#error\t" << err << "\n"; return dup_string(os.str()); }
    std::vector<std::pair<std::string, std::string>> kv;
    {
        std::vector<std::string> items;
        split_keep_quotes(leaves, ',', items);
        for (auto& it : items) {
            size_t eq = it.rfind('=');
            kv.emplace_back(it.substr(0, eq), it.substr(eq + 1));
        }
    }
    StateMap st;
    CostMap cs;
    NucMutMap nm;
    BlockMutMap bm;
    if (algo == 0) {
        for (auto& p : kv) st[p.first] = p.second[0] != '-' ? 1 << code_of(p.second[0]) : 1;
        fitch_up(t.root, st, forced);
        for (auto& n : t.all) os << "F\t" << n.first << "\t" << st[n.first] << "\n";
        fitch_down(t.root, t.root, st, parent, kNoDefault);
        for (auto& n : t.all) os << "B\t" << n.first << "\t" << st[n.first] << "\n";
        fitch_assign(t.root, st, nm, parent);
    } else if (algo == 1) {
        for (auto& p : kv) {
            std::vector<int> v(16, kSankoffInf);
            v[p.second[0] != '-' ? code_of(p.second[0]) : 0] = 0;
            cs[p.first] = v;
        }
        sankoff_up(t.root, cs);
        for (auto& n : t.all) {
            os << "F\t" << n.first << "\t";
            for (int i = 0; i < 16; ++i) os << (i ? "," : "") << cs[n.first][i];
            os << "\n";
        }
        sankoff_down(t.root, t.root, cs, st, parent, forced == -1 ? kNoDefault : forced);
        for (auto& n : t.all) os << "B\t" << n.first << "\t" << st[n.first] << "\n";
        sankoff_assign(t.root, st, nm, parent);
    } else if (algo == 2) {
        for (auto& p : kv) st[p.first] = std::atoi(p.second.c_str());
        block_fitch_up(t.root, st);
        for (auto& n : t.all) os << "F\t" << n.first << "\t" << st[n.first] << "\n";
        block_fitch_down(t.root, t.root, st, parent, forced == -1 ? kNoDefault : forced);
        for (auto& n : t.all) os << "B\t" << n.first << "\t" << st[n.first] << "\n";
        block_fitch_assign(t.root, st, bm, parent);
    } else {
        for (auto& p : kv) {
            std::vector<int> v(3, kSankoffInf);
            v[std::atoi(p.second.c_str())] = 0;
            cs[p.first] = v;
        }
        block_sankoff_up(t.root, cs);
        for (auto& n : t.all) {
            os << "F\t" << n.first << "\t";
            for (int i = 0; i < 3; ++i) os << (i ? "," : "") << cs[n.first][i];
            os << "\n";
        }
        block_sankoff_down(t.root, t.root, cs, st, parent, forced == -1 ? kNoDefault : forced);
        for (auto& n : t.all) os << "B\t" << n.first << "\t" << st[n.first] << "\n";
        block_sankoff_assign(t.root, st, bm, parent);
    }
    std::map<std::string, std::string> sorted;
    for (auto& m : nm) sorted[m.first] = std::to_string(m.second.first) + "\t" + m.second.second;
    for (auto& m : bm) sorted[m.first] = std::to_string(m.second.first) + "\t" + (m.second.second ? "1" : "0");
    for (auto& m : sorted) os << "M\t" << m.first << "\t" << m.second << "\n";
    return dup_string(os.str());
}

// Column block on a CSR tree (bench baseline + full-size parity samples).
//   child_off[n+1], child_idx[]: children in order; names: n NUL-terminated strings.
//   leaf_codes: row r holds `sites` 4-bit codes, one byte per site; node_row[i] is the
//   row of leaf i, or -1 for a leaf absent from the alignment.
//   cons: per-site consensus code; ref: per-site forced root code or NULL.
//   algo 0 = Fitch (M1 semantics, ref -> refState=1<<code), 1 = Sankoff (M2 semantics,
//   ref -> defaultState=code), 2 = block Fitch, 3 = block Sankoff (codes 0 absent block,
//   1 forward, 2 reverse; ref -> defaultValue; records carry (blockMutInfo, inversion)).
//   Output: *out_recs = malloc'd uint32 quads (node, site, type, code), *out_n = count,
//   sorted by (node, site).  Returns wall seconds of the column loop.
double oracle_csr_columns(int32_t n, const int32_t* child_off, const int32_t* child_idx, int32_t root,
                          const char* names, const uint8_t* leaf_codes, int64_t row_stride,
                          const int32_t* node_row, int64_t sites, const uint8_t* cons,
                          const uint8_t* ref, int algo, int threads, uint32_t** out_recs,
                          int64_t* out_n, uint8_t* out_root /* nullable: root final code per site, 255 = unresolved */) {
    CsrTree ct;
    csr_to_tree(n, child_off, child_idx, root, names, ct);
    std::unordered_map<std::string, int32_t> index_of;
    for (int32_t i = 0; i < n; ++i) index_of[ct.by_index[i]->id] = i;
    std::vector<std::pair<int32_t, int32_t>> present;   // (node, row)
    for (int32_t i = 0; i < n; ++i)
        if (child_off[i] == child_off[i + 1] && node_row[i] >= 0) present.emplace_back(i, node_row[i]);

    std::vector<std::vector<uint32_t>> parts(std::max(1, threads));
    std::atomic<int64_t> next(0);
    auto t0 = std::chrono::steady_clock::now();
    auto worker = [&](int w) {
        for (;;) {
            int64_t s = next.fetch_add(1);
            if (s >= sites) break;
            NucMutMap muts;
            if (algo == 0) {
                StateMap st;
                for (auto& pr : present) {
                    int c = leaf_codes[(int64_t)pr.second * row_stride + s];
                    st.insert({ct.by_index[pr.first]->id, 1 << c});
                }
                int ref_state = ref ? 1 << ref[s] : -1;
                fitch_up(ct.t.root, st, ref_state);
                int cs = 1 << cons[s];
                fitch_down(ct.t.root, ct.t.root, st, cs, kNoDefault);
                fitch_assign(ct.t.root, st, muts, cs);
                if (out_root) {
                    const int r = st[ct.t.root->id];
                    out_root[s] = r ? (uint8_t)log2_state(r) : (uint8_t)255;
                }
            } else if (algo == 1) {
                CostMap costs;
                StateMap st;
                for (auto& pr : present) {
                    std::vector<int> v(16, kSankoffInf);
                    v[leaf_codes[(int64_t)pr.second * row_stride + s]] = 0;
                    costs[ct.by_index[pr.first]->id] = v;
                }
                sankoff_up(ct.t.root, costs);
                sankoff_down(ct.t.root, ct.t.root, costs, st, cons[s], ref ? (int)ref[s] : kNoDefault);
                sankoff_assign(ct.t.root, st, muts, cons[s]);
                if (out_root) {
                    const int r = st[ct.t.root->id];
                    out_root[s] = r >= 0 ? (uint8_t)r : (uint8_t)255;
                }
            } else if (algo == 2) {
                // block Fitch (B1), driven like src/panman.cpp:873-911
                StateMap st;
                BlockMutMap bm;
                for (auto& pr : present)
                    st[ct.by_index[pr.first]->id] = 1 << leaf_codes[(int64_t)pr.second * row_stride + s];
                block_fitch_up(ct.t.root, st);
                block_fitch_down(ct.t.root, ct.t.root, st, 1 << cons[s], ref ? 1 << ref[s] : kNoDefault);
                block_fitch_assign(ct.t.root, st, bm, 1 << cons[s]);
                for (auto& m : bm) muts[m.first] = {m.second.first, m.second.second ? '1' : '0'};
                if (out_root) {
                    const int r = st[ct.t.root->id];
                    out_root[s] = r ? (uint8_t)log2_state(r) : (uint8_t)255;
                }
            } else {
                // block Sankoff (B2), driven like src/panman.cpp:912-960
                CostMap costs;
                StateMap st;
                BlockMutMap bm;
                for (auto& pr : present) {
                    std::vector<int> v(3, kSankoffInf);
                    v[leaf_codes[(int64_t)pr.second * row_stride + s]] = 0;
                    costs[ct.by_index[pr.first]->id] = v;
                }
                block_sankoff_up(ct.t.root, costs);
                block_sankoff_down(ct.t.root, ct.t.root, costs, st, cons[s], ref ? (int)ref[s] : kNoDefault);
                block_sankoff_assign(ct.t.root, st, bm, cons[s]);
                for (auto& m : bm) muts[m.first] = {m.second.first, m.second.second ? '1' : '0'};
                if (out_root) {
                    const int r = st[ct.t.root->id];
                    out_root[s] = r >= 0 ? (uint8_t)r : (uint8_t)255;
                }
            }
            for (auto& m : muts) {
                auto& o = parts[w];
                o.push_back((uint32_t)index_of[m.first]);
                o.push_back((uint32_t)s);
                o.push_back((uint32_t)m.second.first);
                // nucleotide: code of the char; block: inversion flag
                o.push_back(algo >= 2 ? (uint32_t)(m.second.second == '1') : (uint32_t)code_of(m.second.second));
            }
        }
    };
    if (threads <= 1) {
        worker(0);
    } else {
        std::vector<std::thread> pool;
        for (int w = 0; w < threads; ++w) pool.emplace_back(worker, w);
        for (auto& th : pool) th.join();
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<std::array<uint32_t, 4>> all;
    for (auto& p : parts)
        for (size_t i = 0; i < p.size(); i += 4) all.push_back({p[i], p[i + 1], p[i + 2], p[i + 3]});
    std::sort(all.begin(), all.end());
    *out_n = (int64_t)all.size();
    *out_recs = (uint32_t*)std::malloc(sizeof(uint32_t) * 4 * (all.size() + 1));
    for (size_t i = 0; i < all.size(); ++i) std::memcpy(*out_recs + 4 * i, all[i].data(), 16);
    return secs;
}

// PanMAT description shared with the product's pm_panmat (same field order / types).
struct OraclePanmat {
    int32_t num_nodes;
    int32_t root;
    const int32_t* child_offsets;
    const int32_t* child_index;
    const char* names;                 // num_nodes NUL-terminated strings back to back
    int32_t num_blocks;
    const int32_t* block_primary;
    const int64_t* block_seq_offsets;
    const uint32_t* block_seq;
    int32_t num_gaps;
    const int32_t* gap_primary;
    const int64_t* gap_offsets;
    const uint32_t* gap_position;
    const uint32_t* gap_length;
    const int64_t* block_mut_offsets;
    const int32_t* block_mut_primary;
    const uint8_t* block_mut_info;
    const uint8_t* block_mut_inversion;
    const int64_t* nuc_mut_offsets;
    const int32_t* nuc_mut_primary;
    const int32_t* nuc_mut_secondary;
    const int32_t* nuc_mut_position;
    const int32_t* nuc_mut_gap_position;
    const uint8_t* nuc_mut_info;
    const uint32_t* nuc_mut_nucs;
    const int32_t* circular_offset;    // nullable, [num_nodes]; < 0 = none
    const int32_t* rotation_index;     // nullable
    const uint8_t* sequence_inverted;  // nullable
    const float* branch_length;        // nullable
};

void build_rtree(const OraclePanmat* p, RTree& t) {
    const char* nm = p->names;
    for (int32_t i = 0; i < p->num_nodes; ++i) {
        auto n = std::make_unique<RNode>();
        n->id = nm;
        nm += n->id.size() + 1;
        if (p->branch_length) n->len = p->branch_length[i];
        t.nodes.push_back(std::move(n));
    }
    for (int32_t i = 0; i < p->num_nodes; ++i) {
        RNode* n = t.nodes[i].get();
        t.all[n->id] = n;
        for (int32_t e = p->child_offsets[i]; e < p->child_offsets[i + 1]; ++e) {
            RNode* c = t.nodes[p->child_index[e]].get();
            c->parent = n;
            n->children.push_back(c);
        }
        if (p->child_offsets[i + 1] > p->child_offsets[i]) ++t.internal_counter;
        for (int64_t k = p->block_mut_offsets[i]; k < p->block_mut_offsets[i + 1]; ++k)
            n->bmuts.push_back({p->block_mut_primary[k], -1, p->block_mut_info[k] != 0, p->block_mut_inversion[k] != 0});
        for (int64_t k = p->nuc_mut_offsets[i]; k < p->nuc_mut_offsets[i + 1]; ++k)
            n->nmuts.push_back({p->nuc_mut_position[k], p->nuc_mut_gap_position[k], p->nuc_mut_primary[k],
                                p->nuc_mut_secondary[k], p->nuc_mut_info[k], p->nuc_mut_nucs[k]});
        if (p->circular_offset && p->circular_offset[i] >= 0) t.circular[n->id] = p->circular_offset[i];
        if (p->rotation_index && p->rotation_index[i] != 0) t.rotation[n->id] = p->rotation_index[i];
        if (p->sequence_inverted && p->sequence_inverted[i]) t.inverted[n->id] = true;
    }
    t.root = t.nodes[p->root].get();
    for (int32_t b = 0; b < p->num_blocks; ++b)
        t.blocks.push_back({p->block_primary[b], std::vector<uint32_t>(p->block_seq + p->block_seq_offsets[b],
                                                                      p->block_seq + p->block_seq_offsets[b + 1])});
    for (int32_t g = 0; g < p->num_gaps; ++g) {
        RGap gl{p->gap_primary[g], {}, {}};
        for (int64_t k = p->gap_offsets[g]; k < p->gap_offsets[g + 1]; ++k) {
            gl.pos.push_back(p->gap_position[k]);
            gl.len.push_back(p->gap_length[k]);
        }
        t.gaps.push_back(gl);
    }
}

// ---------------------------------------------------------------- M4 reroot ----
// R4 getSequenceFromReference (src/panman.cpp:4676-5000) with rotateSequence = false:
// every block expanded (absent ones keep the consensus), gap slots resized, block
// mutations over the whole path, then nucleotide mutations of blocks that exist.
bool sequence_from_reference(RTree& t, RNode* ref, Seq& seq, std::vector<bool>& exists, std::vector<bool>& strand,
                             std::string& err) {
    std::vector<RNode*> path;
    for (RNode* it = ref; it != t.root; it = it->parent) path.push_back(it);
    path.push_back(t.root);
    seq.assign(t.blocks.size() + 1, {});
    exists.assign(t.blocks.size() + 1, false);
    strand.assign(t.blocks.size() + 1, true);
    int32_t max_id = 0;
    for (auto& b : t.blocks) {
        max_id = std::max(max_id, b.primary);
        if ((size_t)b.primary >= seq.size()) { err = "block id beyond the block count"; return false; }
        bool end = false;
        for (size_t j = 0; j < b.seq.size() && !end; ++j)
            for (int k = 0; k < 8; ++k) {
                const int code = (b.seq[j] >> (4 * (7 - k))) & 15;
                if (code == 0) { end = true; break; }
                seq[b.primary].push_back({char_of(code), {}});
            }
        seq[b.primary].push_back({'x', {}});
    }
    seq.resize(max_id + 1);
    exists.resize(max_id + 1);
    strand.resize(max_id + 1);
    for (auto& g : t.gaps)
        for (size_t j = 0; j < g.pos.size(); ++j) {
            if (g.pos[j] >= seq[g.primary].size()) { err = "gap position beyond the block"; return false; }
            seq[g.primary][g.pos[j]].second.resize(g.len[j], '-');
        }
    for (auto it = path.rbegin(); it != path.rend(); ++it)
        for (auto& m : (*it)->bmuts) {
            if (m.info) { exists[m.primary] = true; strand[m.primary] = !m.inversion; }
            else if (m.inversion) strand[m.primary] = !strand[m.primary];
            else { exists[m.primary] = false; strand[m.primary] = true; }
        }
    for (auto it = path.rbegin(); it != path.rend(); ++it)
        for (auto& m : (*it)->nmuts) {
            if (!exists[m.primary]) continue;
            auto& blk = seq[m.primary];
            const uint32_t type = m.type();
            auto put = [&](int32_t pos, int32_t gap, char v) {
                if (pos < 0 || (size_t)pos >= blk.size()) return false;
                if (gap != -1) {
                    if (gap < 0 || (size_t)gap >= blk[pos].second.size()) return false;
                    blk[pos].second[gap] = v;
                } else {
                    blk[pos].first = v;
                }
                return true;
            };
            bool ok = true;
            if (type < 3) {
                for (int j = 0; j < m.length() && ok; ++j) {
                    const char v = type == ND ? '-' : char_of(m.code(j));
                    ok = m.gap != -1 ? put(m.pos, m.gap + j, v) : put(m.pos + j, -1, v);
                }
            } else if (type <= 5) {
                ok = put(m.pos, m.gap, type == 5 ? '-' : char_of(m.code(0)));
            }
            if (!ok) { err = "mutation outside its block"; return false; }
        }
    return true;
}

// transformHelper (src/panman.cpp:5831-5865)
RNode* transform_helper(RTree& t, RNode* node, bool& ok) {
    if (node == t.root) {
        if (node->children.size() > 1) {
            node->len = 0;
            return node;
        }
        if (node->children.empty()) { ok = false; return node; }   // reference: children[0] of an empty list
        RNode* c = node->children[0];
        c->len = 0;
        t.all.erase(node->id);
        node->children.clear();
        return c;
    }
    RNode* par = node->parent;
    par->children.erase(std::find(par->children.begin(), par->children.end(), node));
    node->parent = nullptr;
    const float old = node->len;
    node->len = 0;
    RNode* c = transform_helper(t, par, ok);
    node->children.push_back(c);
    c->parent = node;
    c->len = old;
    return node;
}

// transform (src/panman.cpp:5867-5906)
bool transform(RTree& t, RNode* node) {
    RNode* par = node->parent;
    if (!par) return true;
    if (par == t.root) { node->len = 0; return true; }
    par->children.erase(std::find(par->children.begin(), par->children.end(), node));
    node->parent = nullptr;
    const float old = node->len;
    auto nr = std::make_unique<RNode>();
    nr->id = "node_" + std::to_string(++t.internal_counter);
    nr->len = 0;
    nr->children.push_back(node);
    node->parent = nr.get();
    node->len = 0;
    bool ok = true;
    RNode* sib = transform_helper(t, par, ok);
    nr->children.push_back(sib);
    sib->parent = nr.get();
    sib->len = old;
    t.root = nr.get();
    t.all[nr->id] = nr.get();
    t.nodes.push_back(std::move(nr));
    return ok;
}

// getNewickString (src/panman.cpp:1921-2029) -- the level walk there prints exactly this
// recursive form: "(children)name:len", leaves "name:len", lengths with "%f".
void newick_rec(RNode* n, std::string& out) {
    char buf[64];
    std::snprintf(buf, sizeof buf, ":%f", (double)n->len);
    if (!n->children.empty()) {
        out += '(';
        for (size_t i = 0; i < n->children.size(); ++i) {
            if (i) out += ',';
            newick_rec(n->children[i], out);
        }
        out += ')';
    }
    out += n->id;
    if (n->len >= 0) out += buf;
}

ONode* mirror(OTree& o, RNode* n, ONode* par) {
    ONode* x = o.make(n->id, par);
    o.all[x->id] = x;
    for (RNode* c : n->children) mirror(o, c, x);
    return x;
}

using Tup6 = std::tuple<int, int, int, int, int, int>;   // block, secondary, pos, gap, type, code

// NucMut runs (src/reroot.cpp:228-262, NucMut(vector<tuple6>, start, end) src/panman.hpp:150-180)
void group6(std::vector<Tup6>& v, bool gap, std::vector<RNucMut>& out) {
    std::sort(v.begin(), v.end());
    auto emit = [&](size_t a, size_t b) {
        RNucMut m{std::get<2>(v[a]), std::get<3>(v[a]), std::get<0>(v[a]), std::get<1>(v[a]),
                  (uint8_t)(((b - a) << 4) + std::get<4>(v[a])), 0};
        for (size_t i = a; i < b; ++i) m.nucs += (uint32_t)std::get<5>(v[i]) << (4 * (5 - (i - a)));
        out.push_back(m);
    };
    size_t start = 0;
    for (size_t i = 1; i < v.size(); ++i) {
        const bool brk = i - start == 6 || std::get<0>(v[i]) != std::get<0>(v[i - 1]) ||
                         std::get<1>(v[i]) != std::get<1>(v[i - 1]) ||
                         (gap ? (std::get<2>(v[i]) != std::get<2>(v[i - 1]) || std::get<3>(v[i]) != std::get<3>(v[i - 1]) + 1)
                              : std::get<2>(v[i]) != std::get<2>(v[i - 1]) + 1) ||
                         std::get<4>(v[i]) != std::get<4>(v[i - 1]);
        if (brk) { emit(start, i); start = i; }
    }
    if (!v.empty()) emit(start, v.size());
}

// Tree::reroot (src/reroot.cpp:4-262), columns in sequence; returns the dump (or "#error").
std::string reroot_dump(RTree& t, const std::string& name) {
    auto it = t.all.find(name);
    if (it == t.all.end()) return "#error\tSequence with name " + name + " not found!\n";
    RNode* new_root = it->second;
    if (!new_root->children.empty()) return "#error\tNode with id " + name + " is not a tip!\n";
    std::string err;
    Seq seq;
    std::vector<bool> bex, bst;
    if (!sequence_from_reference(t, new_root, seq, bex, bst, err)) return "#error\t" + err + "\n";
    std::map<std::string, Seq> leaf_seq;
    std::map<std::string, std::vector<bool>> leaf_ex, leaf_st;
    for (auto& kv : t.all)
        if (kv.second->children.empty()) {
            Seq s2;
            std::vector<bool> e2, st2;
            if (!sequence_from_reference(t, kv.second, s2, e2, st2, err)) return "#error\t" + err + "\n";
            leaf_seq[kv.first] = std::move(s2);
            leaf_ex[kv.first] = std::move(e2);
            leaf_st[kv.first] = std::move(st2);
        }
    if (!transform(t, new_root)) return "#error\tunary root\n";
    for (auto& kv : t.all) { kv.second->bmuts.clear(); kv.second->nmuts.clear(); }
    OTree o;
    o.root = mirror(o, t.root, nullptr);
    // block mutations (src/reroot.cpp:53-125)
    for (size_t i = 0; i < bex.size(); ++i) {
        StateMap st;
        BlockMutMap muts;
        for (auto& kv : leaf_ex) st[kv.first] = !kv.second[i] ? 1 : (leaf_st[kv.first][i] ? 2 : 4);
        const int def = !bex[i] ? 1 : (bst[i] ? 2 : 4);
        block_fitch_up(o.root, st);
        block_fitch_down(o.root, o.root, st, 1, def);
        block_fitch_assign(o.root, st, muts, 1);
        for (auto& m : muts) t.all[m.first]->bmuts.push_back({(int32_t)i, -1, m.second.first == BI, m.second.second});
    }
    // nucleotide mutations (src/reroot.cpp:130-226)
    std::map<std::string, std::vector<Tup6>> non_gap, gap;
    for (size_t i = 0; i < seq.size(); ++i) {
        const RBlock* blk = nullptr;
        for (auto& b : t.blocks)
            if (b.primary == (int32_t)i) { blk = &b; break; }
        if (!blk) return "#error\tBlock with id " + std::to_string(i) + " -1 not found!\n";
        std::string cons;
        bool end = false;
        for (size_t j = 0; j < blk->seq.size() && !end; ++j)
            for (int k = 0; k < 8; ++k) {
                const int code = (blk->seq[j] >> (4 * (7 - k))) & 15;
                if (code == 0) { end = true; break; }
                cons += char_of(code);
            }
        cons += '-';
        if (cons.size() != seq[i].size()) return "#error\tconsensus length mismatch\n";
        auto state_of = [](char ch) { return ch != '-' && ch != 'x' ? 1 << code_of(ch) : 1; };
        for (size_t k = 0; k < seq[i].size(); ++k) {
            for (size_t w = 0; w < seq[i][k].second.size(); ++w) {
                StateMap st;
                NucMutMap muts;
                for (auto& kv : leaf_seq) st[kv.first] = state_of(kv.second[i][k].second[w]);
                const int code = state_of(seq[i][k].second[w]);
                fitch_up(o.root, st, code);
                fitch_down(o.root, o.root, st, code, code);
                fitch_assign(o.root, st, muts, 1);
                for (auto& m : muts)
                    gap[m.first].emplace_back((int)i, -1, (int)k, (int)w, m.second.first, code_of(m.second.second));
            }
            StateMap st;
            NucMutMap muts;
            for (auto& kv : leaf_seq) st[kv.first] = state_of(kv.second[i][k].first);
            const int code = state_of(seq[i][k].first);
            fitch_up(o.root, st, code);
            fitch_down(o.root, o.root, st, code, code);
            fitch_assign(o.root, st, muts, 1 << code_of(cons[k]));
            for (auto& m : muts)
                non_gap[m.first].emplace_back((int)i, -1, (int)k, -1, m.second.first, code_of(m.second.second));
        }
    }
    for (auto& kv : non_gap) group6(kv.second, false, t.all[kv.first]->nmuts);
    for (auto& kv : gap) group6(kv.second, true, t.all[kv.first]->nmuts);
    std::string out = "newick\t";
    newick_rec(t.root, out);
    out += ";\n";
    char buf[160];
    for (auto& kv : t.all) {
        auto bm = kv.second->bmuts;
        std::sort(bm.begin(), bm.end(), [](const RBlockMut& a, const RBlockMut& b) { return a.primary < b.primary; });
        for (auto& m : bm) {
            std::snprintf(buf, sizeof buf, "\tB\t%d\t%d\t%d\n", m.primary, (int)m.info, (int)m.inversion);
            out += kv.first + buf;
        }
        for (auto& m : kv.second->nmuts) {
            std::snprintf(buf, sizeof buf, "\tN\t%d\t%d\t%d\t%u\t%06x\n", m.primary, m.pos, m.gap, (unsigned)m.info,
                          m.nucs);
            out += kv.first + buf;
        }
    }
    return out;
}

// FASTA records of every leaf (printFASTAUltraFast), sorted by leaf name; at most
// `leaf_limit` leaves (<= 0: all) and, when `seconds` is set, the replay wall time.
// `threads` > 1: the leaves are replayed in parallel, as the reference's
// tbb::parallel_for_each over leaves does (src/fasta.cpp:1993), then joined in name order.
char* oracle_fasta(const OraclePanmat* p, int aligned, int leaf_limit, int threads, double* seconds) {
    RTree t;
    build_rtree(p, t);
    std::vector<RNode*> leaves;
    for (auto& kv : t.all) {
        if (!kv.second->children.empty()) continue;
        if (leaf_limit > 0 && (int)leaves.size() >= leaf_limit) break;
        leaves.push_back(kv.second);
    }
    std::vector<std::string> rec(leaves.size());
    auto t0 = std::chrono::steady_clock::now();
    const int nt = std::max(1, std::min(threads, (int)leaves.size()));
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t i = next++; i < leaves.size(); i = next++) rec[i] = leaf_record(t, leaves[i], aligned != 0);
    };
    std::vector<std::thread> pool;
    for (int k = 1; k < nt; ++k) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::string out;
    for (auto& r : rec) out += r;
    return dup_string(out);
}

// Reroot at `leaf` (Tree::reroot) and dump the new tree: "newick\t<text>" then per node
// in name order its block mutations (sorted by block) and nucleotide mutations (list
// order) -- see reroot_dump.
// ---------------------------------------------------------------- summary ----
// Tree::printSummary (src/summary.cpp:257-273): counts by getTotalParsimonyParallelHelper
// (:3-59) -- NS counted by length, NI / ND by record, block insertions of any strand into
// "Insertions", non-inverting block deletions into "Deletions", every block mutation with
// the inversion flag into "Inversions" -- and the Newick parser's leaf depths
// (src/panman.cpp:372-394: float sum in Newick leaf order / leaf count).  Then
// getBlockMutationsParallel (:203-250, printed to std::cout): block insertions / deletions /
// inversions and the duplication / translocation walk getOtherBlockMutationsParallelHelper
// (:111-193) over blocks grouped by identical consensusSeq.  Returns "<out part>\0<cout part>".
struct SummaryWalk {
    std::vector<bool> exists, strand;
    std::vector<std::vector<uint32_t>> dups;
    std::vector<uint32_t> dups_pos;
    long long dup = 0, trans = 0;
    void visit(RNode* n) {
        std::vector<bool> exists_parent = exists;
        std::vector<std::tuple<int32_t, bool, bool>> undo;
        for (auto& m : n->bmuts) {
            const int32_t b = m.primary;
            if (m.info) {
                undo.emplace_back(b, exists[b], strand[b]);
                exists[b] = true;
                strand[b] = !m.inversion;
            } else {
                undo.emplace_back(b, exists[b], strand[b]);
                if (m.inversion) {
                    strand[b] = !strand[b];
                } else {
                    exists[b] = false;
                    strand[b] = true;
                }
            }
        }
        for (auto& m : n->bmuts) {
            if (!m.info) continue;
            for (uint32_t d : dups[dups_pos[m.primary]]) {
                if (d != (uint32_t)m.primary && exists[d] && exists_parent[d]) { ++dup; break; }
                if (d != (uint32_t)m.primary && !exists[d] && exists_parent[d]) { ++trans; break; }
            }
        }
        for (RNode* c : n->children) visit(c);
        for (auto it = undo.rbegin(); it != undo.rend(); ++it) {
            exists[std::get<0>(*it)] = std::get<1>(*it);
            strand[std::get<0>(*it)] = std::get<2>(*it);
        }
    }
};

static std::string summary_text(RTree& t, std::string& cout_part) {
    long long ns = 0, ni = 0, nd = 0, bi = 0, bd = 0, inv = 0, bdi = 0;
    size_t leaves = 0, max_depth = 0;
    float mean_depth = 0.f;
    // pre-order, children in order = the Newick string's leaf order
    std::vector<std::pair<RNode*, size_t>> stack{{t.root, 0}};
    while (!stack.empty()) {
        auto [n, depth] = stack.back();
        stack.pop_back();
        for (auto& m : n->nmuts) {
            if (m.type() == 0) ns += m.length();
            else if (m.type() == 2) ++ni;
            else if (m.type() == 1) ++nd;
        }
        for (auto& m : n->bmuts) {
            if (m.info) ++bi;
            if (!m.info && !m.inversion) ++bd;
            if (m.inversion) ++inv;
            if (!m.info && m.inversion) ++bdi;
        }
        if (n->children.empty()) {
            ++leaves;
            max_depth = std::max(max_depth, depth);
            mean_depth += depth;
        }
        for (auto it = n->children.rbegin(); it != n->children.rend(); ++it) stack.push_back({*it, depth + 1});
    }
    mean_depth /= leaves;
    std::ostringstream out;
    out << "Total Nodes in Tree: " << t.internal_counter + leaves << std::endl;
    out << "Total Samples in Tree: " << leaves << std::endl;
    out << "Total Substitutions: " << ns << std::endl;
    out << "Total Insertions: " << ni + bi << std::endl;
    out << "Total Deletions: " << nd + bd << std::endl;
    out << "Total Inversions: " << inv << std::endl;
    out << "Max Tree Depth: " << max_depth << std::endl;
    out << "Mean Tree Depth: " << mean_depth << std::endl;
    SummaryWalk w;
    std::map<std::vector<uint32_t>, std::vector<uint32_t>> by_seq;   // grouping only: order-free counts
    for (auto& b : t.blocks) by_seq[b.seq].push_back((uint32_t)b.primary);
    w.dups_pos.assign(t.blocks.size(), 0);
    for (auto& kv : by_seq) {
        for (uint32_t b : kv.second) w.dups_pos[b] = (uint32_t)w.dups.size();
        w.dups.push_back(kv.second);
    }
    w.exists.assign(t.blocks.size(), false);
    w.strand.assign(t.blocks.size(), true);
    w.visit(t.root);
    std::ostringstream co;
    co << "Total Block Insertions: " << bi << std::endl;
    co << "Total Block Deletions: " << bd << std::endl;
    co << "Total Block Inversion: " << bdi << std::endl;
    co << "Total Block Duplications: " << w.dup << std::endl;
    co << "Total Block Translocation: " << w.trans << std::endl;
    cout_part = co.str();
    return out.str();
}

char* oracle_summary(const OraclePanmat* p) {
    RTree t;
    build_rtree(p, t);
    std::string co;
    const std::string out = summary_text(t, co);
    return dup_string(out + std::string(1, '\0') + co);
}

char* oracle_reroot(const OraclePanmat* p, const char* leaf) {
    RTree t;
    build_rtree(p, t);
    return dup_string(reroot_dump(t, leaf));
}

// ------------------------------------------------------------- M3 PanGraph ----
// Restatement of Tree(json, newick, FILE_TYPE::PANGRAPH, reference) (src/panman.cpp:820-1273)
// with Pangraph (:6200-6476), chain_align (src/chaining.cpp) and rotate_sample
// (src/rotation.cpp), on the reference's containers.  The PanGraph JSON arrives flattened
// by the test (one record per line, see tests/_pangraph.py); oneTBB's concurrent map order
// of individualSequences is restated as ascending bit-reversed tbb_hasher(name) | 1.
namespace pgo {

struct Range {
    std::pair<int, int> point;
    Range* left = nullptr;
    Range* right = nullptr;
};

Range* range_tree(std::vector<std::pair<int, int>>& pts, int a, int b, std::vector<std::unique_ptr<Range>>& own) {
    if (a > b) return nullptr;
    std::sort(pts.begin() + a, pts.begin() + b + 1,
              [](const std::pair<int, int>& x, const std::pair<int, int>& y) { return x.first < y.first; });
    const int mid = (a + b) / 2;
    own.push_back(std::make_unique<Range>());
    Range* r = own.back().get();
    r->point = pts[mid];
    r->left = range_tree(pts, a, mid - 1, own);
    r->right = range_tree(pts, mid + 1, b, own);
    return r;
}

void query(Range* r, std::pair<int, int> lo, std::pair<int, int> hi, std::vector<std::pair<int, int>>& out) {
    if (!r) return;
    if (r->point.first >= lo.first && r->point.first <= hi.first && r->point.second >= lo.second &&
        r->point.second <= hi.second)
        out.push_back(r->point);
    if (r->left && lo.first <= r->point.first) query(r->left, lo, hi, out);
    if (r->right && hi.first >= r->point.first) query(r->right, lo, hi, out);
}

struct PairHash {
    size_t operator()(const std::pair<int, int>& p) const {
        const size_t a = std::hash<int>{}(p.first), b = std::hash<int>{}(p.second);
        return a != b ? a ^ b : a;
    }
};

std::vector<std::pair<int, int>> chaining(std::vector<std::string>& cons, std::vector<std::string>& sample) {
    std::vector<std::pair<int, int>> chain, pts;
    for (size_t i = 0; i < cons.size(); ++i)
        for (size_t j = 0; j < sample.size(); ++j)
            if (cons[i] == sample[j]) pts.emplace_back((int)i, (int)j);
    std::sort(pts.begin(), pts.end());
    std::vector<std::unique_ptr<Range>> own;
    Range* root = range_tree(pts, 0, (int)pts.size() - 1, own);
    if (pts.empty()) return chain;
    std::unordered_map<std::pair<int, int>, std::pair<int, std::pair<int, int>>, PairHash> map;
    const std::pair<int, int> origin(-1, -1);
    for (auto p : pts) map[p] = {-1, origin};
    const int K = 4000, match = 50;
    for (auto point : pts) {
        if (point.first == 0 && point.second == 0) { map[point] = {match, {-1, -1}}; continue; }
        std::vector<std::pair<int, int>> res;
        query(root, {point.first - K > 0 ? point.first - K : 0, point.second - K > 0 ? point.second - K : 0},
              {point.first - 1, point.second - 1}, res);
        int score = 10, xb = -1, yb = -1;
        std::pair<int, int> node = origin;
        for (auto it = res.rbegin(); it != res.rend(); ++it) {
            auto p = *it;
            if (p.first <= xb && p.second <= yb) continue;
            const int cost = -(point.first - p.first + point.second - p.second);
            if (cost + map[p].first + match > score) { score = cost + map[p].first + match; node = p; }
            if (xb < p.first) xb = p.first - 1;
            if (yb < p.second) yb = p.second - 1;
        }
        map[point] = {score, node};
    }
    int best = -1;
    std::pair<int, int> seed{};
    for (auto& m : map)
        if (m.second.first > best) { best = m.second.first; seed = m.first; }
    while (true) {
        chain.push_back(seed);
        seed = map[seed].second;
        if (seed == origin) break;
    }
    return chain;
}

std::pair<int, int> rotate_alignment(const std::vector<std::string>& c, const std::vector<std::string>& s) {
    std::vector<std::pair<int, int>> score(s.size(), {-1, -1}), next(s.size(), {-1, -1});
    std::pair<int, int> mx(0, 0);
    for (size_t i = 0; i < c.size(); ++i) {
        for (size_t j = 0; j < s.size(); ++j) {
            const size_t up = j == 0 ? s.size() - 1 : j - 1, diag = up, left = j;
            int lv = score[left].first - 1, dv = score[diag].first, uv = j == 0 ? -1 : next[up].first - 1;
            dv = c[i] == s[j] ? dv + 5 : dv - 2;
            if (dv >= lv) {
                if (dv >= uv) next[j] = {dv, score[diag].second == -1 ? (int)j : score[diag].second};
                else next[j] = {uv, j == 0 ? -1 : next[up].second};
            } else {
                if (lv >= uv) next[j] = {lv, score[left].second};
                else next[j] = {uv, j == 0 ? -1 : next[up].second};
            }
            if (next[j].first > mx.first) mx = next[j];
        }
        for (size_t z = 0; z < s.size(); ++z) score[z] = next[z];
    }
    return mx;
}

uint64_t tbb_key(const std::string& s) {
    uint64_t h = 0;
    for (char c : s) h = (uint64_t)(int64_t)c ^ (h * 0x9E3779B97F4A7C15ull);
    uint64_t r = 0;
    for (int b = 0; b < 64; ++b) r |= ((h >> b) & 1ull) << (63 - b);
    return r | 1ull;
}

std::vector<std::string> split_tabs(const std::string& line) {
    std::vector<std::string> f;
    size_t a = 0;
    for (size_t b; (b = line.find('\t', a)) != std::string::npos; a = b + 1) f.push_back(line.substr(a, b - a));
    f.push_back(line.substr(a));
    return f;
}

using Item = std::pair<char, std::vector<char>>;

// `rt` (nullable) receives the built Tree in the R1 replay's form (blocks packed 8 codes per
// u32, gap slots, per-node mutations, rotation / inversion / circular offsets), so the
// oracle's printFASTAUltraFast restatement can replay what this driver built.
std::string build_dump(const std::string& flat, const std::string& newick, const std::string& reference, bool tbb_order,
                       RTree* rt = nullptr) {
    // --- Pangraph (:6200-6425) ---
    std::unordered_map<std::string, std::vector<std::string>> paths;
    std::unordered_map<std::string, std::vector<int>> strand_paths;
    std::unordered_map<std::string, std::vector<size_t>> block_numbers, int_sequences;
    std::unordered_map<std::string, int> circular, rotation;
    std::unordered_map<std::string, bool> inverted;
    std::unordered_map<std::string, std::string> consensus;
    std::unordered_map<std::string, std::vector<std::pair<size_t, size_t>>> gaps;
    std::unordered_map<std::string, std::unordered_map<std::string, std::unordered_map<size_t,
        std::vector<std::pair<size_t, std::string>>>>> subs;
    std::unordered_map<std::string, std::unordered_map<std::string, std::unordered_map<size_t,
        std::vector<std::tuple<size_t, size_t, std::string>>>>> ins;
    std::unordered_map<std::string, std::unordered_map<std::string, std::unordered_map<size_t,
        std::vector<std::pair<size_t, size_t>>>>> dels;
    bool circ = false;
    std::istringstream in(flat);
    std::string line;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        const auto f = split_tabs(line);
        if (f[0] == "P") {
            for (size_t k = 5; k < f.size(); ++k) {
                const size_t colon = f[k].rfind(':');
                paths[f[1]].push_back(f[k].substr(0, colon));
                strand_paths[f[1]].push_back(f[k].substr(colon + 1) == "1");
            }
            if (f[2] == "1") { circ = true; circular[f[1]] = -std::stoi(f[3]); }
        } else if (f[0] == "B") {
            consensus[f[1]] = f[2];
        } else if (f[0] == "G") {
            gaps[f[1]].emplace_back((size_t)std::stol(f[2]), (size_t)std::stol(f[3]));
        } else if (f[0] == "S") {
            subs[f[1]][f[2]][(size_t)std::stol(f[3])].emplace_back((size_t)std::stol(f[4]), f[5]);
        } else if (f[0] == "I") {
            ins[f[1]][f[2]][(size_t)std::stol(f[3])].emplace_back((size_t)std::stol(f[4]), (size_t)std::stol(f[5]), f[6]);
        } else if (f[0] == "D") {
            dels[f[1]][f[2]][(size_t)std::stol(f[3])].emplace_back((size_t)std::stol(f[4]), (size_t)std::stol(f[5]));
        }
    }
    if (circ) {
        std::vector<std::string> base;
        int count = 0;
        for (auto& p : paths) {
            std::unordered_map<std::string, size_t> bn;
            for (auto& b : p.second) { block_numbers[p.first].push_back(bn[b] + 1); bn[b]++; }
            if (count == 0) {
                inverted[p.first] = false;
                rotation[p.first] = 0;
                base = p.second;
            } else {
                auto sample = p.second;
                const int rot = rotate_alignment(base, sample).second;
                std::vector<std::string> out;
                std::vector<int> ns;
                std::vector<size_t> nn;
                auto& st = strand_paths[p.first];
                auto& num = block_numbers[p.first];
                for (size_t i = 0; i < sample.size(); ++i) {
                    const size_t k = (i + rot) % sample.size();
                    out.push_back(sample[k]);
                    ns.push_back(st[k]);
                    nn.push_back(num[k]);
                }
                st = ns;
                num = nn;
                inverted[p.first] = false;
                rotation[p.first] = (int)((sample.size() - rot) % sample.size());
                p.second = out;
            }
            ++count;
        }
    } else {
        for (auto p : paths) {
            std::unordered_map<std::string, size_t> bn;
            inverted[p.first] = false;
            rotation[p.first] = 0;
            for (auto& b : p.second) { block_numbers[p.first].push_back(bn[b] + 1); bn[b]++; }
        }
    }
    size_t num_nodes = 0;
    std::unordered_map<int, std::string> int_to_string;
    std::vector<std::string> cons;
    std::vector<size_t> int_cons;
    int count = 0;
    for (auto& p : paths) {
        if (count == 0) {
            for (auto& b : p.second) {
                cons.push_back(b);
                int_to_string[(int)num_nodes] = b;
                int_sequences[p.first].push_back(num_nodes);
                int_cons.push_back(num_nodes);
                ++num_nodes;
            }
        } else {
            std::vector<std::string> sample = p.second, cons_new;
            std::vector<size_t> int_sample, int_new;
            auto chain = chaining(cons, sample);
            int pc = -1, ps = -1;
            for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
                for (int j = pc + 1; j < it->first; ++j) { cons_new.push_back(cons[j]); int_new.push_back(int_cons[j]); }
                for (int j = ps + 1; j < it->second; ++j) {
                    cons_new.push_back(sample[j]);
                    int_sample.push_back(num_nodes);
                    int_to_string[(int)num_nodes] = sample[j];
                    int_new.push_back(num_nodes);
                    ++num_nodes;
                }
                cons_new.push_back(cons[it->first]);
                int_sample.push_back(int_cons[it->first]);
                int_new.push_back(int_cons[it->first]);
                pc = it->first;
                ps = it->second;
            }
            for (int j = pc + 1; j < (int)cons.size(); ++j) { cons_new.push_back(cons[j]); int_new.push_back(int_cons[j]); }
            for (int j = ps + 1; j < (int)sample.size(); ++j) {
                cons_new.push_back(sample[j]);
                int_sample.push_back(num_nodes);
                int_to_string[(int)num_nodes] = sample[j];
                int_new.push_back(num_nodes);
                ++num_nodes;
            }
            for (auto b : int_sample) int_sequences[p.first].push_back(b);
            cons = cons_new;
            int_cons = int_new;
        }
        ++count;
    }
    std::unordered_map<int, int> order;
    std::unordered_map<size_t, std::string> id_of;
    std::vector<size_t> topo;
    int reorder = 0;
    for (auto i : int_cons) {
        order[(int)i] = reorder;
        id_of[reorder] = int_to_string[(int)i];
        topo.push_back(reorder);
        ++reorder;
    }
    for (auto& m : int_sequences)
        for (auto& x : m.second) x = order[(int)x];

    // --- driver (:820-1273) ---
    OTree t;
    std::string err;
    if (!parse_newick(newick, t, err)) return "#error\t" + err + "\n";
    std::function<bool(ONode*)> has_polytomy = [&](ONode* n) {
        if (n->children.size() > 2) return true;
        for (ONode* c : n->children)
            if (has_polytomy(c)) return true;
        return false;
    };
    const bool polytomy = has_polytomy(t.root);
    std::unordered_map<std::string, std::vector<int>> aligned, aligned_strand;
    for (auto p : int_sequences) {
        size_t p1 = 0, p2 = 0;
        while (p1 < topo.size() && p2 < p.second.size()) {
            if (topo[p1] == p.second[p2]) { aligned[p.first].push_back((int)topo[p1]); ++p2; }
            else aligned[p.first].push_back(-1);
            ++p1;
        }
        while (aligned[p.first].size() < topo.size()) aligned[p.first].push_back(-1);
    }
    for (auto p : int_sequences) {
        size_t p1 = 0, p2 = 0;
        while (p1 < topo.size() && p2 < p.second.size()) {
            if (topo[p1] == p.second[p2]) { aligned_strand[p.first].push_back(strand_paths[p.first][p2]); ++p2; }
            else aligned_strand[p.first].push_back(-1);
            ++p1;
        }
        while (aligned_strand[p.first].size() < topo.size()) aligned_strand[p.first].push_back(-1);
    }
    std::map<std::string, std::vector<RBlockMut>> block_muts;
    for (size_t i = 0; i < topo.size(); ++i) {
        if (!polytomy) {
            StateMap st;
            BlockMutMap muts;
            int def = -1;
            for (auto& u : aligned) {
                if (reference.length() && u.first.find(reference) != std::string::npos)
                    def = u.second[i] == -1 ? 1 : (aligned_strand[u.first][i] ? 2 : 4);
                st[u.first] = u.second[i] == -1 ? 1 : (aligned_strand[u.first][i] ? 2 : 4);
            }
            block_fitch_up(t.root, st);
            block_fitch_down(t.root, t.root, st, 1, def != -1 ? def : kNoDefault);
            block_fitch_assign(t.root, st, muts, 1);
            for (auto& m : muts) block_muts[m.first].push_back({(int32_t)i, -1, m.second.first == BI, m.second.second});
        } else {
            CostMap cs;
            StateMap st;
            BlockMutMap muts;
            int def = -1;
            for (auto& u : aligned) {
                if (reference.length() && u.first.find(reference) != std::string::npos)
                    def = u.second[i] == -1 ? 0 : (aligned_strand[u.first][i] ? 1 : 2);
                std::vector<int> v(3, kSankoffInf);
                v[u.second[i] == -1 ? 0 : (aligned_strand[u.first][i] ? 1 : 2)] = 0;
                cs[u.first] = v;
            }
            block_sankoff_up(t.root, cs);
            block_sankoff_down(t.root, t.root, cs, st, 0, def != -1 ? def : kNoDefault);
            block_sankoff_assign(t.root, st, muts, 0);
            for (auto& m : muts) block_muts[m.first].push_back({(int32_t)i, -1, m.second.first == BI, m.second.second});
        }
    }
    std::unordered_map<std::string, std::vector<size_t>> block_counts;
    for (auto& u : aligned) {
        block_counts[u.first].resize(u.second.size(), 0);
        int ptr = 0;
        for (size_t i = 0; i < u.second.size(); ++i)
            if (u.second[i] != -1) block_counts[u.first][i] = block_numbers[u.first][ptr++];
    }
    std::map<std::string, std::vector<std::tuple<int, int, int, int, int, int>>> non_gap, gap_m;
    for (size_t i = 0; i < topo.size(); ++i) {
        const std::string sid = id_of[topo[i]];
        const std::string cseq = consensus[sid];
        std::vector<Item> seq(cseq.size() + 1, {'-', {}});
        for (size_t j = 0; j < cseq.size(); ++j) seq[j].first = cseq[j];
        for (auto& g : gaps[sid]) seq[g.first].second.resize(g.second, '-');
        std::vector<std::pair<std::string, std::vector<Item>>> indiv;   // iterated in TBB order below
        for (auto& u : aligned) {
            if (u.second[i] == -1) continue;
            auto cur = seq;
            const size_t num = block_counts[u.first][i];
            for (auto& v : subs[sid][u.first][num]) cur[v.first - 1].first = v.second[0];
            for (auto& v : ins[sid][u.first][num])
                for (size_t j = 0; j < std::get<2>(v).size(); ++j) cur[std::get<0>(v)].second[std::get<1>(v) + j] = std::get<2>(v)[j];
            for (auto& v : dels[sid][u.first][num])
                for (size_t j = v.first; j < v.first + v.second; ++j) cur[j - 1].first = '-';
            indiv.emplace_back(u.first, cur);
        }
        if (tbb_order) {
            std::sort(indiv.begin(), indiv.end(), [](const auto& a, const auto& b) { return tbb_key(a.first) < tbb_key(b.first); });
        } else {   // the survey's serial stand-in: a std::unordered_map filled in alignedSequences order
            std::unordered_map<std::string, std::vector<Item>> m;
            for (auto& u : indiv) m[u.first] = u.second;
            indiv.assign(m.begin(), m.end());
        }
        auto state_of = [](char ch) { return ch != '-' ? 1 << code_of(ch) : 1; };
        for (size_t j = 0; j < seq.size(); ++j) {
            for (size_t k = 0; k < seq[j].second.size(); ++k) {
                NucMutMap muts;
                StateMap st;
                if (!polytomy) {
                    int def = -1;
                    for (auto& u : indiv) {
                        if (reference.length() && u.first.find(reference) != std::string::npos)
                            def = state_of(u.second[j].second[k]);
                        st[u.first] = state_of(u.second[j].second[k]);
                    }
                    fitch_up(t.root, st, -1);
                    const int par = 1 << code_of(seq[j].second[k]);
                    fitch_down(t.root, t.root, st, par, def != -1 ? def : kNoDefault);
                    fitch_assign(t.root, st, muts, par);
                } else {
                    CostMap cs;
                    int def = -1;
                    for (auto& u : indiv) {
                        const char ch = u.second[j].second[k];
                        if (reference.length() && u.first.find(reference) != std::string::npos)
                            def = ch != '-' ? code_of(ch) : 0;
                        std::vector<int> v(16, kSankoffInf);
                        v[ch != '-' ? code_of(ch) : 0] = 0;
                        cs[u.first] = v;
                    }
                    sankoff_up(t.root, cs);
                    sankoff_down(t.root, t.root, cs, st, code_of(seq[j].second[k]), def != -1 ? def : kNoDefault);
                    sankoff_assign(t.root, st, muts, code_of(seq[j].second[k]));
                }
                for (auto& m : muts)
                    gap_m[m.first].emplace_back((int)i, -1, (int)j, (int)k, m.second.first, code_of(m.second.second));
            }
            NucMutMap muts;
            StateMap st;
            if (!polytomy) {
                int def = -1;
                for (auto& u : indiv) {
                    if (u.first.find(reference) != std::string::npos) def = state_of(u.second[j].first);   // unguarded
                    st[u.first] = state_of(u.second[j].first);
                }
                fitch_up(t.root, st, -1);
                const int par = 1 << code_of(seq[j].first);
                fitch_down(t.root, t.root, st, par, def != -1 ? def : kNoDefault);
                fitch_assign(t.root, st, muts, par);
            } else {
                CostMap cs;
                int def = -1;
                for (auto& u : indiv) {
                    const char ch = u.second[j].first;
                    if (reference.length() && u.first.find(reference) != std::string::npos)
                        def = ch != '-' ? code_of(ch) : 0;
                    std::vector<int> v(16, kSankoffInf);
                    v[ch != '-' ? code_of(ch) : 0] = 0;
                    cs[u.first] = v;
                }
                sankoff_up(t.root, cs);
                sankoff_down(t.root, t.root, cs, st, code_of(seq[j].first), def != -1 ? def : kNoDefault);
                sankoff_assign(t.root, st, muts, code_of(seq[j].first));
            }
            for (auto& m : muts)
                non_gap[m.first].emplace_back((int)i, -1, (int)j, -1, m.second.first, code_of(m.second.second));
        }
    }
    std::map<std::string, std::vector<RNucMut>> nuc;
    for (auto& kv : non_gap) group6(kv.second, false, nuc[kv.first]);
    for (auto& kv : gap_m) group6(kv.second, true, nuc[kv.first]);
    if (rt) {
        std::unordered_map<const ONode*, RNode*> of;
        for (ONode* o : t.owned) {
            auto n = std::make_unique<RNode>();
            n->id = o->id;
            of[o] = n.get();
            rt->nodes.push_back(std::move(n));
        }
        for (ONode* o : t.owned) {
            RNode* n = of[o];
            if (o->parent) n->parent = of[o->parent];
            for (ONode* ch : o->children) n->children.push_back(of[ch]);
            rt->all[n->id] = n;
        }
        rt->root = of[t.root];
        rt->internal_counter = t.internal_counter;
        for (size_t i = 0; i < topo.size(); ++i) {
            const std::string& seq = consensus[id_of[topo[i]]];
            RBlock b{(int32_t)i, std::vector<uint32_t>((seq.size() + 8) / 8, 0u)};   // a 0 code ends the block
            for (size_t k = 0; k < seq.size(); ++k) b.seq[k / 8] |= (uint32_t)code_of(seq[k]) << (4 * (7 - k % 8));
            rt->blocks.push_back(std::move(b));
            RGap g{(int32_t)i, {}, {}};
            for (auto& gp : gaps[id_of[topo[i]]]) {
                g.pos.push_back((uint32_t)gp.first);
                g.len.push_back((uint32_t)gp.second);
            }
            rt->gaps.push_back(std::move(g));
        }
        for (auto& kv : block_muts)
            if (rt->all.count(kv.first)) rt->all[kv.first]->bmuts = kv.second;
        for (auto& kv : nuc)
            if (rt->all.count(kv.first)) rt->all[kv.first]->nmuts = kv.second;
        for (auto& kv : circular) rt->circular[kv.first] = kv.second;
        for (auto& kv : rotation)
            if (kv.second != 0) rt->rotation[kv.first] = kv.second;
        for (auto& kv : inverted)
            if (kv.second) rt->inverted[kv.first] = true;
    }
    // dump: blocks, then per node (name order) block and nucleotide mutations
    std::string out;
    char buf[200];
    for (size_t i = 0; i < topo.size(); ++i) {
        const std::string sid = id_of[topo[i]];
        out += "block\t" + std::to_string(i) + "\t" + consensus[sid];
        for (auto& g : gaps[sid]) out += "\t" + std::to_string(g.first) + ":" + std::to_string(g.second);
        out += "\n";
    }
    for (auto& kv : t.all) {
        auto bm = block_muts[kv.first];
        std::sort(bm.begin(), bm.end(), [](const RBlockMut& a, const RBlockMut& b) { return a.primary < b.primary; });
        for (auto& m : bm) {
            std::snprintf(buf, sizeof buf, "\tB\t%d\t%d\t%d\n", m.primary, (int)m.info, (int)m.inversion);
            out += kv.first + buf;
        }
        for (auto& m : nuc[kv.first]) {
            std::snprintf(buf, sizeof buf, "\tN\t%d\t%d\t%d\t%u\t%06x\n", m.primary, m.pos, m.gap, (unsigned)m.info, m.nucs);
            out += kv.first + buf;
        }
    }
    return out;
}

}  // namespace pgo

// M3 then R1 (src/panman.cpp:820-1273, src/fasta.cpp:1981-2099): the FASTA records of every
// leaf of the Tree the PanGraph driver builds, sorted by leaf name -- the round trip that
// test/sars_20.fa pins (the input genomes come back).
char* oracle_pangraph_fasta(const char* flat, const char* newick, const char* reference, int tbb_order, int aligned) {
    std::string nwk(newick);
    const size_t nl = nwk.find('\n');
    if (nl != std::string::npos) nwk.resize(nl);
    RTree t;
    const std::string dump = pgo::build_dump(flat, nwk, reference ? reference : "", tbb_order != 0, &t);
    if (dump.rfind("#error", 0) == 0 || !t.root) return dup_string(dump);
    std::string out;
    for (auto& kv : t.all)
        if (kv.second->children.empty()) out += leaf_record(t, kv.second, aligned != 0);
    return dup_string(out);
}

char* oracle_pangraph(const char* flat, const char* newick, const char* reference, int tbb_order) {
    std::string nwk(newick);
    const size_t nl = nwk.find('\n');
    if (nl != std::string::npos) nwk.resize(nl);
    return dup_string(pgo::build_dump(flat, nwk, reference ? reference : "", tbb_order != 0));
}

}  // extern "C"
