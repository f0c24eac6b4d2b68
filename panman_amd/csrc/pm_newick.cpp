// pm_newick.cpp -- Newick parsing with the reference's semantics (src/panman.cpp:265-450).
#include "pm_newick.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <stack>
#include <string>
#include <vector>

namespace pm {

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

bool parse_topology(std::string text, Topology& t, std::string& err) {
    while (!text.empty() && text.back() == ' ') text.pop_back();
    const size_t first = text.find_first_not_of(' ');
    text = first == std::string::npos ? std::string() : text.substr(first);
    struct Tok { std::string leaf; size_t opens = 0, closes = 0; };
    std::vector<Tok> toks;
    // Branch lengths: every ')' and every piece end pushes the digits seen after the last
    // ':' of the piece (stale if a clade has none; 1 if none at all; 0 becomes 1) onto a
    // FIFO per depth; nodes pop their depth's FIFO in creation order (:339-376, :408-435).
    std::vector<std::vector<float>> fifo;
    std::vector<size_t> fifo_head;
    auto push_len = [&](long lvl, const std::string& digits) -> bool {
        float len = 1.0f;
        if (!digits.empty()) {
            char* end = nullptr;
            len = std::strtof(digits.c_str(), &end);
            if (end == digits.c_str()) return false;   // std::stof would throw
        }
        if (len == 0) len = 1.0f;
        if ((long)fifo.size() <= lvl) fifo.resize(lvl + 1), fifo_head.resize(lvl + 1, 0);
        fifo[lvl].push_back(len);
        return true;
    };
    long depth = 0;
    for (const std::string& piece : split_quoted(text, ',')) {
        Tok k;
        bool stop = false, quote = false, quoted = false, branch_start = false;
        std::string branch;
        for (char ch : piece) {
            if (quote) { k.leaf += ch; quote = ch != '\''; }
            else if (ch == '\'') { quote = quoted = true; k.leaf += ch; }
            else if (ch == ':') { stop = true; branch.clear(); branch_start = true; }
            else if (ch == '(') { ++k.opens; ++depth; }
            else if (ch == ')') {
                stop = true;
                ++k.closes;
                if (depth < 0 || !push_len(depth, branch)) { err = "incorrect Newick format"; return false; }
                --depth;
                branch_start = false;
            }
            else if (!stop) { k.leaf += ch; branch_start = false; }
            else if (branch_start && (std::isdigit((unsigned char)ch) || ch == '.')) branch += ch;
        }
        if (quoted && k.leaf.size() >= 2 && k.leaf.front() == '\'' && k.leaf.back() == '\'')
            k.leaf = k.leaf.substr(1, k.leaf.size() - 2);
        if (depth < 0 || !push_len(depth, branch)) { err = "incorrect Newick format"; return false; }
        toks.push_back(std::move(k));
    }
    if (depth != 0) { err = "incorrect Newick format"; return false; }
    long level = 0;
    auto pop_len = [&](float& len) {
        if (level >= (long)fifo.size() || fifo_head[level] >= fifo[level].size()) return false;
        len = fifo[level][fifo_head[level]++];
        return true;
    };
    std::stack<int32_t> open;
    int internal = 0;
    auto add = [&](const std::string& nm) {
        t.name.push_back(nm);
        t.kids.emplace_back();
        t.length.push_back(1.0f);
        const int32_t id = (int32_t)t.name.size() - 1;
        if (!open.empty()) t.kids[open.top()].push_back(id);
        return id;
    };
    for (const Tok& k : toks) {
        for (size_t j = 0; j < k.opens; ++j) {
            const int32_t id = add("node_" + std::to_string(++internal));
            if (t.root < 0) t.root = id;
            open.push(id);
            if (!pop_len(t.length[id])) { err = "incorrect Newick format"; return false; }
            ++level;
        }
        if (open.empty()) { err = "leaf outside any clade"; return false; }
        const int32_t leaf = add(k.leaf);
        if (!pop_len(t.length[leaf])) { err = "incorrect Newick format"; return false; }
        for (size_t j = 0; j < k.closes && !open.empty(); ++j) {
            open.pop();
            --level;
        }
    }
    if (t.root < 0) { err = "empty tree"; return false; }
    t.length[t.root] = 0.0f;
    return true;
}

std::string newick_of(const Topology& t) {
    if (t.kids[t.root].empty()) return t.name[t.root];   // single node: the bare identifier
    auto len_of = [&](int32_t v) {
        const float len = t.length.empty() ? (v == t.root ? 0.0f : 1.0f) : t.length[v];
        std::string s;
        if (len >= 0) {
            char buf[64];
            std::snprintf(buf, sizeof buf, ":%f", (double)len);
            s = buf;
        }
        return s;
    };
    std::string out;
    std::vector<std::pair<int32_t, size_t>> st{{t.root, 0}};
    while (!st.empty()) {
        auto& top = st.back();
        const int32_t v = top.first;
        const auto& k = t.kids[v];
        if (k.empty()) {
            out += t.name[v] + len_of(v);
            st.pop_back();
            continue;
        }
        if (top.second == 0) out += '(';
        if (top.second < k.size()) {
            if (top.second > 0) out += ',';
            const int32_t c = k[top.second++];
            st.emplace_back(c, 0);
        } else {
            out += ')' + t.name[v] + len_of(v);
            st.pop_back();
        }
    }
    return out + ";";
}

}  // namespace pm
