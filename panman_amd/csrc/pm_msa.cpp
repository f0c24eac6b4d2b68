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
#include <thread>
#include <vector>

#include "pm_internal.h"
#include "pm_newick.h"

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

struct MsaResult {
    std::string err;
    Topology t;
    std::string consensus;
    std::vector<std::vector<Grouped>> muts;   // per node id, NucMut runs in list order
};

// The constructor body: returns the tree, consensus block and per-node NucMut lists.
MsaResult build_result(const char* newick_c, const char* msa_c, const char* ref_c, int mode,
                       const std::vector<int>& devices) {
    MsaResult res;
    PhaseClock clock;
    std::string newick(newick_c), err;
    const size_t nl = newick.find('\n');
    if (nl != std::string::npos) newick.resize(nl);
    auto dump_error = [&](const std::string& e) {
        res.err = e;
        return res;
    };
    Topology& t = res.t;
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

    res.consensus = consensus;
    res.muts.assign(t.name.size(), {});
    clock.lap("msa.parse");
    if (width == 0) return res;

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

    // columns split into contiguous even-aligned ranges, one host thread + context per
    // device; each range's records are (node, site)-sorted, so appending
    // the ranges in site order and stable-sorting by node gives the global (node, site) order.
    // Distinct devices form one RCCL communicator (pm_comm_init_all) and the per-site
    // (score, root code) are reassembled with one all-gather (pm_multi_run); repeated
    // devices (several shards on one GPU) run their shards independently.
    const int G = (int)devices.size();
    std::vector<std::vector<pm_mut>> part(G);
    std::vector<std::string> msg(G);
    std::vector<int64_t> lo(G + 1);
    for (int g = 0; g <= G; ++g) lo[g] = std::min<int64_t>(S, (S * g / G + 1) / 2 * 2);
    lo[G] = S;
    bool distinct = G > 1;
    for (int g = 0; g < G; ++g)
        for (int h = 0; h < g; ++h) distinct &= devices[g] != devices[h];
    for (int g = 0; g < G && distinct; ++g) distinct &= lo[g + 1] > lo[g];
    clock.lap("msa.pack_columns");
    std::vector<CtxGuard> cg(G);
    for (int g = 0; g < G; ++g)
        if (pm_create(devices[g], &cg[g].c) != PM_OK) return dump_error("no HIP device " + std::to_string(devices[g]));
    clock.lap("hip.create_contexts");
    auto each = [&](auto&& fn) {   // one host thread per shard
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g)
            th.emplace_back([&, g]() {
                if (lo[g + 1] > lo[g] && msg[g].empty()) fn(g);
            });
        for (auto& x : th) x.join();
        for (int g = 0; g < G; ++g)
            if (!msg[g].empty()) return false;
        return true;
    };
    const bool uploaded = each([&](int g) {
        const int64_t a = lo[g], ns = lo[g + 1] - lo[g];
        pm_tree tree{N, t.root, off.data(), idx.data()};
        if (pm_tree_upload(cg[g].c, &tree) != PM_OK ||
            pm_leaves_upload(cg[g].c, ns, codes.data() + a / 2, stride, node_row.data(), nullptr, 0) != PM_OK ||
            pm_sites_upload(cg[g].c, cons4.data() + a / 2, ref_row ? force4.data() + a / 2 : nullptr) != PM_OK ||
            (!distinct && pm_run(cg[g].c, mode) != PM_OK))
            msg[g] = pm_last_error(cg[g].c);
    });
    clock.lap("msa.upload");
    if (uploaded && !distinct)
        each([&](int g) {
            if (hipStreamSynchronize(cg[g].c->stream) != hipSuccess) msg[g] = "GPU run failed";
        });
    std::vector<int32_t> score;
    if (uploaded && distinct) {
        std::vector<pm_ctx*> ctxs(G);
        for (int g = 0; g < G; ++g) ctxs[g] = cg[g].c;
        score.assign(S, 0);
        if (pm_comm_init_all(ctxs.data(), G) != PM_OK ||
            pm_multi_run(ctxs.data(), G, mode, lo.data(), S, score.data(), nullptr) != PM_OK)
            return dump_error(std::string("multi-GPU run: ") + pm_last_error(ctxs[0]));
    }
    clock.lap("msa.gpu_run");
    if (uploaded)
        each([&](int g) {
            int64_t n = 0;
            if (pm_mutation_count(cg[g].c, &n) != PM_OK) {
                msg[g] = pm_last_error(cg[g].c);
                return;
            }
            part[g].resize((size_t)std::max<int64_t>(n, 1));
            if (pm_mutations_fetch(cg[g].c, part[g].data(), n, &n) != PM_OK) {
                msg[g] = pm_last_error(cg[g].c);
                return;
            }
            part[g].resize((size_t)n);
            for (pm_mut& m : part[g]) m.site_info += (uint32_t)lo[g] << 8;
        });
    for (int g = 0; g < G; ++g)
        if (!msg[g].empty()) return dump_error(msg[g]);
    if (!score.empty()) {   // the gathered score counts every non-root record exactly once
        int64_t total = 0, nonroot = 0;
        for (int32_t v : score) total += v;
        for (auto& v : part)
            for (const pm_mut& m : v) nonroot += m.node != (uint32_t)t.root;
        if (total != nonroot) return dump_error("gathered parsimony score disagrees with the shards' records");
    }
    clock.lap("msa.fetch_records");
    std::vector<pm_mut> recs;
    for (auto& v : part) recs.insert(recs.end(), v.begin(), v.end());
    if (G > 1) std::stable_sort(recs.begin(), recs.end(), [](const pm_mut& x, const pm_mut& y) { return x.node < y.node; });
    const int64_t n = (int64_t)recs.size();

    for (int64_t a = 0; a < n;) {
        int64_t b = a;
        while (b < n && recs[b].node == recs[a].node) ++b;
        group_node(recs.data() + a, b - a, res.muts[recs[a].node]);
        a = b;
    }
    clock.lap("msa.group");
    return res;
}

std::string build(const char* newick_c, const char* msa_c, const char* ref_c, int mode, int device) {
    MsaResult r = build_result(newick_c, msa_c, ref_c, mode, {device});
    if (!r.err.empty()) return dump_error(r.err);
    std::string dump = "#consensus\t" + r.consensus + "\n";
    dump += "#blockmut\t" + r.t.name[r.t.root] + "\t0\t-1\t1\t0\n";
    std::map<std::string, const std::vector<Grouped>*> by_name;   // nodes in name order
    for (size_t v = 0; v < r.muts.size(); ++v)
        if (!r.muts[v].empty()) by_name[r.t.name[v]] = &r.muts[v];
    std::ostringstream os;
    for (auto& kv : by_name)
        for (auto& m : *kv.second) {
            char buf[96];
            std::snprintf(buf, sizeof buf, "\t%d\t-1\t%u\t%06x\n", m.pos, m.info, m.nucs);
            os << kv.first << buf;
        }
    return dump + os.str();
}

// Block(0, consensus): 8 codes per word, MSB nibble first (src/panman.cpp:246-257).
std::vector<uint32_t> encode_block(const std::string& seq) {
    std::vector<uint32_t> w;
    for (size_t i = 0; i < seq.size(); i += 8) {
        uint32_t x = 0;
        for (size_t j = i; j < std::min(i + 8, seq.size()); ++j) x ^= (uint32_t)nuc_code(seq[j]) << (4 * (7 - (j - i)));
        w.push_back(x);
    }
    return w;
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

int pm_msa_to_panman(const char* newick, const char* msa_text, const char* reference, int mode, int device,
                     const char* out_path, char* err, int64_t err_len) {
    return pm_msa_to_panman_multi(newick, msa_text, reference, mode, &device, 1, out_path, err, err_len);
}

int pm_msa_to_panman_multi(const char* newick, const char* msa_text, const char* reference, int mode,
                           const int* devices, int num_devices, const char* out_path, char* err, int64_t err_len) {
    auto set_err = [&](const std::string& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
    };
    if (!newick || !msa_text || !out_path || (mode != PM_MODE_FITCH && mode != PM_MODE_SANKOFF) || !devices ||
        num_devices < 1) {
        set_err("bad arguments");
        return PM_ERR_ARG;
    }
    pm::MsaResult r = pm::build_result(newick, msa_text, reference, mode,
                                       std::vector<int>(devices, devices + num_devices));
    if (!r.err.empty()) {
        set_err(r.err);
        return PM_ERR_ARG;
    }
    const auto t_conv = std::chrono::steady_clock::now();
    const int32_t N = (int32_t)r.t.name.size();
    std::vector<int32_t> off(N + 1, 0), idx;
    std::string names;
    for (int32_t i = 0; i < N; ++i) {
        idx.insert(idx.end(), r.t.kids[i].begin(), r.t.kids[i].end());
        off[i + 1] = (int32_t)idx.size();
        names += r.t.name[i];
        names.push_back('\0');
    }
    const std::vector<uint32_t> words = pm::encode_block(r.consensus);
    const int32_t block_primary = 0;
    const int64_t seq_off[2] = {0, (int64_t)words.size()};
    const int64_t gap_off[1] = {0};
    std::vector<int64_t> bm_off(N + 1, 0), nm_off(N + 1, 0);
    for (int32_t v = 0; v < N; ++v) bm_off[v + 1] = bm_off[v] + (v == r.t.root ? 1 : 0);
    const int32_t bm_primary = 0;
    const uint8_t bm_info = 1, bm_inv = 0;   // root: BlockMut(0, BI, false)
    std::vector<int32_t> np, ns, npos, ngap;
    std::vector<uint8_t> ninfo;
    std::vector<uint32_t> nnucs;
    for (int32_t v = 0; v < N; ++v) {
        for (auto& m : r.muts.empty() ? std::vector<pm::Grouped>() : r.muts[v]) {
            np.push_back(0);
            ns.push_back(-1);
            npos.push_back(m.pos);
            ngap.push_back(-1);
            ninfo.push_back((uint8_t)m.info);
            nnucs.push_back(m.nucs);
        }
        nm_off[v + 1] = (int64_t)np.size();
    }
    pm_panmat p{};
    p.num_nodes = N;
    p.root = r.t.root;
    p.child_offsets = off.data();
    p.child_index = idx.data();
    p.names = names.data();
    p.num_blocks = 1;
    p.block_primary = &block_primary;
    p.block_seq_offsets = seq_off;
    p.block_seq = words.data();
    p.num_gaps = 0;
    p.gap_offsets = gap_off;
    p.block_mut_offsets = bm_off.data();
    p.block_mut_primary = &bm_primary;
    p.block_mut_info = &bm_info;
    p.block_mut_inversion = &bm_inv;
    p.nuc_mut_offsets = nm_off.data();
    p.nuc_mut_primary = np.data();
    p.nuc_mut_secondary = ns.data();
    p.nuc_mut_position = npos.data();
    p.nuc_mut_gap_position = ngap.data();
    p.nuc_mut_info = ninfo.data();
    p.nuc_mut_nucs = nnucs.data();
    p.branch_length = r.t.length.data();
    const pm_panmat* list[1] = {&p};
    pm::phase_add("msa.to_panmat", std::chrono::duration<double>(std::chrono::steady_clock::now() - t_conv).count());
    const int rc = pm_panman_write(out_path, list, 1, 1);
    if (rc != PM_OK) set_err(std::string("cannot write ") + out_path);
    return rc;
}

}  // extern "C"
