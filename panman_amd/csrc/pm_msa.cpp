// pm_msa.cpp -- MSA -> per-node mutations on the GPU: the column drivers of the
// reference's Tree(msa, newick, FILE_TYPE::MSA | MSA_OPTIMIZE, reference) constructor
// (src/panman.cpp:1274-1466 Fitch "M1", :1467-1649 low-mem Sankoff "M2"), with the
// per-column recursion replaced by one pm_run over all columns, followed by the
// reference's NucMut grouping (src/panman.cpp:1445-1466, src/panman.hpp:100-151).
//
// Exposed as pm_msa_build(); the canonical text dump it returns is the one the tests
// compare against the CPU oracle byte for byte.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <stack>
#include <string>
#include <vector>

#include "pm_internal.h"

namespace pm {
namespace {

int nuc_code(char c) {
    switch (c) {
        case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
        case 'R': return 5;  case 'Y': return 10; case 'S': return 6;  case 'W': return 9;
        case 'K': return 12; case 'M': return 3;  case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7;  case 'N': return 15;
        default: return 0;   // gap, lowercase, anything else (src/panman.cpp:78-113)
    }
}

// Split on `delim`, re-joining pieces while a single quote is open (src/panman.cpp:265-296).
std::vector<std::string> split_quoted(const std::string& s, char delim) {
    std::vector<std::string> out;
    size_t start = 0, open_at = 0;
    bool open = false;
    for (size_t end; (end = s.find(delim, start)) != std::string::npos; start = end + 1) {
        const size_t from = open ? open_at : start;
        const std::string piece = s.substr(from, end - from);
        const bool odd = std::count(piece.begin(), piece.end(), '\'') % 2 == 1;
        if (!open && odd) { open = true; open_at = start; }
        else if (!open) out.push_back(piece);
        else if (!odd) { open = false; out.push_back(piece); }
    }
    if (start < s.size()) out.push_back(s.substr(start));
    return out;
}

// Newick topology, nodes numbered in creation (pre-)order; internal nodes are named
// node_<k> in order of '(' and internal labels are ignored (src/panman.cpp:310-450).
struct Topology {
    std::vector<std::string> name;
    std::vector<std::vector<int32_t>> kids;
    int32_t root = -1;
};

bool parse_topology(std::string text, Topology& t, std::string& err) {
    while (!text.empty() && text.back() == ' ') text.pop_back();
    const size_t first = text.find_first_not_of(' ');
    text = first == std::string::npos ? std::string() : text.substr(first);
    struct Tok { std::string leaf; size_t opens = 0, closes = 0; };
    std::vector<Tok> toks;
    long depth = 0;
    for (const std::string& piece : split_quoted(text, ',')) {
        Tok k;
        bool stop = false, quote = false, quoted = false;
        for (char ch : piece) {
            if (quote) { k.leaf += ch; quote = ch != '\''; }
            else if (ch == '\'') { quote = quoted = true; k.leaf += ch; }
            else if (ch == ':') stop = true;
            else if (ch == '(') { ++k.opens; ++depth; }
            else if (ch == ')') { stop = true; ++k.closes; --depth; }
            else if (!stop) k.leaf += ch;
        }
        if (quoted && k.leaf.size() >= 2 && k.leaf.front() == '\'' && k.leaf.back() == '\'')
            k.leaf = k.leaf.substr(1, k.leaf.size() - 2);
        toks.push_back(std::move(k));
    }
    if (depth != 0) { err = "incorrect Newick format"; return false; }
    std::stack<int32_t> open;
    int internal = 0;
    auto add = [&](const std::string& nm) {
        t.name.push_back(nm);
        t.kids.emplace_back();
        const int32_t id = (int32_t)t.name.size() - 1;
        if (!open.empty()) t.kids[open.top()].push_back(id);
        return id;
    };
    for (const Tok& k : toks) {
        for (size_t j = 0; j < k.opens; ++j) {
            const int32_t id = add("node_" + std::to_string(++internal));
            if (t.root < 0) t.root = id;
            open.push(id);
        }
        if (open.empty()) { err = "leaf outside any clade"; return false; }
        add(k.leaf);
        for (size_t j = 0; j < k.closes && !open.empty(); ++j) open.pop();
    }
    if (t.root < 0) { err = "empty tree"; return false; }
    return true;
}

// M1 reader: rows keyed (and ordered) by name, '\r' stripped, equal lengths required
// (src/panman.cpp:1285-1322).
bool read_rows(const std::string& text, std::map<std::string, std::string>& rows, size_t& width, std::string& err) {
    std::istringstream in(text);
    std::string line, seq, id;
    width = 0;
    auto flush = [&](const std::string& nm) {
        if (width == 0) width = seq.size();
        else if (width != seq.size()) { err = "sequence lengths don't match: " + nm; return false; }
        rows[nm] = seq;
        return true;
    };
    bool have = false;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        if (line[0] == '>') {
            if (have && !seq.empty() && !flush(split_quoted(id, '\r').empty() ? std::string() : split_quoted(id, '\r')[0]))
                return false;
            const auto sp = split_quoted(line, ' ');
            id = sp.empty() ? std::string() : sp[0].substr(1);
            seq.clear();
            have = true;
        } else {
            const auto sp = split_quoted(line, '\r');
            seq += sp.empty() ? std::string() : sp[0];
        }
    }
    if (!seq.empty() && !flush(id)) return false;
    return true;
}

struct Grouped {
    int32_t pos;
    uint32_t info;
    uint32_t nucs;
};

// NucMut runs: a new record starts after 6 codes, at a position gap or a type change.
void group_node(const pm_mut* r, int64_t n, std::vector<Grouped>& out) {
    auto pos = [&](int64_t i) { return (int32_t)(r[i].site_info >> 8); };
    auto typ = [&](int64_t i) { return (r[i].site_info >> 4) & 15u; };
    int64_t start = 0;
    auto emit = [&](int64_t a, int64_t b) {
        Grouped g{pos(a), (uint32_t)(((b - a) << 4) + typ(a)), 0};
        for (int64_t k = a; k < b; ++k) g.nucs += (r[k].site_info & 15u) << (4 * (5 - (k - a)));
        out.push_back(g);
    };
    for (int64_t i = 1; i < n; ++i)
        if (i - start == 6 || pos(i) != pos(i - 1) + 1 || typ(i) != typ(i - 1)) { emit(start, i); start = i; }
    if (n > 0) emit(start, n);
}

std::string dump_error(const std::string& e) { return "#error\t" + e + "\n"; }

struct CtxGuard {
    pm_ctx* c = nullptr;
    ~CtxGuard() { pm_destroy(c); }
};

std::string build(const char* newick_c, const char* msa_c, const char* ref_c, int mode, int device) {
    std::string newick(newick_c), err;
    const size_t nl = newick.find('\n');
    if (nl != std::string::npos) newick.resize(nl);
    Topology t;
    if (!parse_topology(newick, t, err)) return dump_error(err);
    const std::string reference = ref_c ? ref_c : "";

    std::map<std::string, std::string> rows;
    size_t width = 0;
    if (!read_rows(msa_c, rows, width, err)) return dump_error(err);
    if (mode == PM_MODE_SANKOFF && rows.size() == 1) width = 0;   // M2 never measures the last row

    std::string consensus(width, '\0');
    std::vector<uint8_t> forced;
    const std::string* ref_row = nullptr;
    if (!reference.empty()) {
        auto it = rows.find(reference);
        if (it == rows.end()) {
            if (mode == PM_MODE_SANKOFF) return dump_error("Reference not found in the sequence");
            width = 0;   // M1 indexes an empty reference row: zero columns
            consensus.clear();
        } else {
            ref_row = &it->second;
        }
    }
    for (size_t i = 0; i < width; ++i) {
        char pick = '\0';
        bool found = false;
        if (ref_row && (mode == PM_MODE_FITCH || (*ref_row)[i] != '-')) {
            pick = (*ref_row)[i];      // M1: the reference row (:1332); M2: unless a gap (:1530)
            found = true;
        } else {
            for (auto& r : rows)
                if (r.second[i] != '-') { pick = r.second[i]; found = true; break; }
        }
        if (!found && !ref_row)
            return dump_error(mode == PM_MODE_FITCH
                                  ? "all-gap column without reference (reference behaviour undefined)"
                                  : "all-gap column without reference (reference exits)");
        consensus[i] = pick;
    }

    std::string dump = "#consensus\t" + consensus + "\n";
    dump += "#blockmut\t" + t.name[t.root] + "\t0\t-1\t1\t0\n";
    if (width == 0) return dump;

    // CSR + leaf rows (rows in name order; leaves missing from the alignment are absent)
    const int32_t N = (int32_t)t.name.size();
    std::vector<int32_t> off(N + 1, 0), idx;
    for (int32_t i = 0; i < N; ++i) {
        idx.insert(idx.end(), t.kids[i].begin(), t.kids[i].end());
        off[i + 1] = (int32_t)idx.size();
    }
    std::map<std::string, int32_t> row_of;
    std::vector<const std::string*> row_seq;
    for (auto& r : rows) {
        row_of[r.first] = (int32_t)row_seq.size();
        row_seq.push_back(&r.second);
    }
    std::vector<int32_t> node_row(N, -1);
    for (int32_t i = 0; i < N; ++i)
        if (t.kids[i].empty()) {
            auto it = row_of.find(t.name[i]);
            if (it != row_of.end()) node_row[i] = it->second;
        }
    const int64_t S = (int64_t)width;
    const int64_t stride = (S + 1) / 2;
    std::vector<uint8_t> codes(row_seq.size() * stride, 0);
    for (size_t r = 0; r < row_seq.size(); ++r)
        for (int64_t s = 0; s < S; ++s)
            codes[r * stride + s / 2] |= (uint8_t)(nuc_code((*row_seq[r])[s]) << (4 * (s & 1)));
    std::vector<uint8_t> cons4(stride, 0), force4;
    for (int64_t s = 0; s < S; ++s) cons4[s / 2] |= (uint8_t)(nuc_code(consensus[s]) << (4 * (s & 1)));
    if (ref_row) {
        // M1: refState = 1 << code(ref) (:1419); M2: defaultState = code, gap -> 0 (:1583-1596)
        force4.assign(stride, 0);
        for (int64_t s = 0; s < S; ++s) force4[s / 2] |= (uint8_t)(nuc_code((*ref_row)[s]) << (4 * (s & 1)));
    }

    CtxGuard g;
    int rc = pm_create(device, &g.c);
    if (rc != PM_OK) return dump_error("no HIP device");
    pm_tree tree{N, t.root, off.data(), idx.data()};
    if ((rc = pm_tree_upload(g.c, &tree)) != PM_OK ||
        (rc = pm_leaves_upload(g.c, S, codes.data(), stride, node_row.data(), nullptr, 0)) != PM_OK ||
        (rc = pm_sites_upload(g.c, cons4.data(), ref_row ? force4.data() : nullptr)) != PM_OK ||
        (rc = pm_run(g.c, mode)) != PM_OK)
        return dump_error(pm_last_error(g.c));
    int64_t n = 0;
    if ((rc = pm_mutation_count(g.c, &n)) != PM_OK) return dump_error(pm_last_error(g.c));
    std::vector<pm_mut> recs((size_t)std::max<int64_t>(n, 1));
    if ((rc = pm_mutations_fetch(g.c, recs.data(), n, &n)) != PM_OK) return dump_error(pm_last_error(g.c));

    std::map<std::string, std::vector<Grouped>> per_node;
    for (int64_t a = 0; a < n;) {
        int64_t b = a;
        while (b < n && recs[b].node == recs[a].node) ++b;
        group_node(recs.data() + a, b - a, per_node[t.name[recs[a].node]]);
        a = b;
    }
    std::ostringstream os;
    for (auto& kv : per_node)
        for (auto& m : kv.second) {
            char buf[96];
            std::snprintf(buf, sizeof buf, "\t%d\t-1\t%u\t%06x\n", m.pos, m.info, m.nucs);
            os << kv.first << buf;
        }
    return dump + os.str();
}

}  // namespace
}  // namespace pm

extern "C" {

char* pm_msa_build(const char* newick, const char* msa_text, const char* reference, int mode, int device) {
    std::string out;
    if (!newick || !msa_text || (mode != PM_MODE_FITCH && mode != PM_MODE_SANKOFF)) out = "#error\tbad arguments\n";
    else out = pm::build(newick, msa_text, reference, mode, device);
    char* p = static_cast<char*>(std::malloc(out.size() + 1));
    if (!p) return nullptr;
    std::memcpy(p, out.data(), out.size() + 1);
    return p;
}

void pm_free(void* p) { std::free(p); }

}  // extern "C"
