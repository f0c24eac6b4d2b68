// pm_newick.cpp -- Newick parsing with the reference's semantics (src/panman.cpp:265-450).
#include "pm_newick.h"

#include <algorithm>
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

std::string newick_of(const Topology& t) {
    std::string out;
    std::vector<std::pair<int32_t, size_t>> st{{t.root, 0}};
    while (!st.empty()) {
        auto& top = st.back();
        const int32_t v = top.first;
        const auto& k = t.kids[v];
        if (k.empty()) {
            out += t.name[v];
            st.pop_back();
            continue;
        }
        if (top.second == 0) out += '(';
        if (top.second < k.size()) {
            if (top.second > 0) out += ',';
            const int32_t c = k[top.second++];
            st.emplace_back(c, 0);
        } else {
            out += ')';
            st.pop_back();
        }
    }
    return out + ";";
}

}  // namespace pm
