// panman_tree.hpp -- header-only C++ facade over panman_gpu.h shaped like the reference's
// panmanUtils::Tree / TreeGroup (src/panman.hpp:819-1271), for the commands on the GPU
// path.  A caller of the reference swaps the include and the namespace:
//
//   panmanUtils::Tree T(msa, nwk, FILE_TYPE::MSA, ref)        -> panman_gpu::Tree T(msa, nwk, panman_gpu::MSA, ref)
//   panmanUtils::TreeGroup TG(fin)                            -> panman_gpu::TreeGroup TG(fin)
//   TG.trees[i].printFASTAUltraFast(out, aligned)             (unchanged)
//   TG.trees[i].printSummary(out) / reroot(name) / getNewickString()
//
// Everything runs through the C-ABI (include/panman_gpu.h): parsimony, replay and the
// summary reduction on the GPU; no CPU fallback.  Errors throw panman_gpu::Error where the
// reference would exit().
#ifndef PANMAN_TREE_HPP
#define PANMAN_TREE_HPP

#include <cstdio>
#include <fstream>
#include <iostream>
#include <iterator>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unistd.h>
#include <vector>

#include "panman_gpu.h"

namespace panman_gpu {

// src/common.hpp:35-42
enum FILE_TYPE { PANMAT = 0, GFA = 1, PANGRAPH = 2, MSA = 3, MSA_OPTIMIZE = 4 };

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

namespace detail {

inline std::string slurp(std::istream& in) {
    return std::string(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
}

struct Ctx {   // one pm_ctx per facade object that computes
    pm_ctx* c = nullptr;
    explicit Ctx(int device) {
        if (pm_create(device, &c) != PM_OK) throw Error("no HIP device " + std::to_string(device));
    }
    ~Ctx() { pm_destroy(c); }
    Ctx(const Ctx&) = delete;
    Ctx& operator=(const Ctx&) = delete;
    void check(int rc, const char* what) const {
        if (rc != PM_OK) throw Error(std::string(what) + ": " + pm_last_error(c));
    }
};

using File = std::shared_ptr<pm_panman>;

inline File own(pm_panman* f) { return File(f, [](pm_panman* p) { pm_panman_free(p); }); }

inline File load(const std::string& path) {
    pm_panman* f = nullptr;
    char err[512] = {0};
    if (pm_panman_load(path.c_str(), &f, err, sizeof err) != PM_OK) throw Error(err[0] ? err : "cannot load " + path);
    return own(f);
}

// A scratch file for the builders that write a .panman (removed when it goes out of scope).
struct TempPath {
    std::string path;
    TempPath() {
        char tmpl[] = "/tmp/panman_gpu_XXXXXX";
        const int fd = mkstemp(tmpl);
        if (fd < 0) throw Error("cannot create a temporary file");
        close(fd);
        path = tmpl;
    }
    ~TempPath() { std::remove(path.c_str()); }
};

}  // namespace detail

class Tree {
  public:
    // Tree(std::ifstream& fin, std::ifstream& secondFin, FILE_TYPE ftype, std::string reference)
    // (src/panman.hpp:825-826): MSA / MSA_OPTIMIZE -- fin = aligned FASTA, secondFin = Newick
    // (src/panman.cpp:1274-1649); PANGRAPH -- fin = PanGraph JSON, secondFin = Newick
    // (:820-1273).  GFA input is not on the GPU path.
    Tree(std::istream& fin, std::istream& secondFin, FILE_TYPE ftype, const std::string& reference = "",
         int device = 0)
        : device_(device) {
        const std::string first = detail::slurp(fin), newick = detail::slurp(secondFin);
        if (ftype == MSA || ftype == MSA_OPTIMIZE) {
            detail::TempPath tmp;
            char err[512] = {0};
            const int mode = ftype == MSA ? PM_MODE_FITCH : PM_MODE_SANKOFF;
            if (pm_msa_to_panman(newick.c_str(), first.c_str(), reference.c_str(), mode, device, tmp.path.c_str(), err,
                                 sizeof err) != PM_OK)
                throw Error(err[0] ? err : "PanMAN construction failed");
            file_ = detail::load(tmp.path);
        } else if (ftype == PANGRAPH) {
            detail::Ctx ctx(device);
            pm_panman* out = nullptr;
            ctx.check(pm_pangraph_build(ctx.c, first.c_str(), newick.c_str(), reference.c_str(), &out),
                      "pm_pangraph_build");
            file_ = detail::own(out);
        } else {
            throw Error("this FILE_TYPE is not on the GPU path");
        }
    }

    // One tree of a loaded PanMAN (TreeGroup::trees[index]).
    Tree(detail::File file, int index, int device = 0) : file_(std::move(file)), index_(index), device_(device) {}

    // Tree::printFASTAUltraFast(fout, aligned) (src/fasta.cpp:1981-2099), replayed on the GPU.
    void printFASTAUltraFast(std::ostream& fout, bool aligned = false) const {
        detail::Ctx ctx(device_);
        pm_panmat v = view();
        char* text = nullptr;
        int64_t len = 0;
        ctx.check(pm_fasta(ctx.c, &v, aligned ? 1 : 0, &text, &len), "pm_fasta");
        fout.write(text, (std::streamsize)len);
        pm_free(text);
    }

    // Tree::printSummary(out) (src/summary.cpp:257-273); the block lines go to std::cout as
    // getBlockMutationsParallel prints them (:203-250).
    void printSummary(std::ostream& out) const {
        detail::Ctx ctx(device_);
        pm_panmat v = view();
        pm_summary s;
        ctx.check(pm_summary_compute(ctx.c, &v, &s), "pm_summary_compute");
        out << "Total Nodes in Tree: " << s.nodes << std::endl;
        out << "Total Samples in Tree: " << s.samples << std::endl;
        out << "Total Substitutions: " << s.substitutions << std::endl;
        out << "Total Insertions: " << s.insertions << std::endl;
        out << "Total Deletions: " << s.deletions << std::endl;
        out << "Total Inversions: " << s.inversions << std::endl;
        out << "Max Tree Depth: " << s.max_depth << std::endl;
        out << "Mean Tree Depth: " << s.mean_depth << std::endl;
        std::cout << "Total Block Insertions: " << s.block_insertions << std::endl;
        std::cout << "Total Block Deletions: " << s.block_deletions << std::endl;
        std::cout << "Total Block Inversion: " << s.block_inversions << std::endl;
        std::cout << "Total Block Duplications: " << s.block_duplications << std::endl;
        std::cout << "Total Block Translocation: " << s.block_translocations << std::endl;
    }

    // Tree::reroot(sequenceName) (src/reroot.cpp:4-262): the tree is replaced by the rerooted one.
    void reroot(const std::string& sequenceName) {
        detail::Ctx ctx(device_);
        pm_panmat v = view();
        pm_panman* out = nullptr;
        ctx.check(pm_reroot(ctx.c, &v, sequenceName.c_str(), &out), "pm_reroot");
        file_ = detail::own(out);
        index_ = 0;
    }

    // Newick of the tree as stored (Tree::getNewickString, src/panman.cpp:1921-2029).
    std::string getNewickString() const { return pm_panman_newick(file_.get(), index_); }

    // The flat view every C-ABI entry point takes (valid while this Tree lives).
    pm_panmat view() const {
        pm_panmat v;
        if (pm_panman_tree(file_.get(), index_, &v) != PM_OK) throw Error("bad tree index");
        return v;
    }

  private:
    detail::File file_;
    int index_ = 0;
    int device_ = 0;
    friend class TreeGroup;
};

class TreeGroup {
  public:
    std::vector<Tree> trees;

    // TreeGroup(std::istream& fin) (src/panman.hpp:1260; src/panman.cpp:6847-6877): an xz-compressed
    // Cap'n Proto PanMAN read from a stream.
    explicit TreeGroup(std::istream& fin, int device = 0) {
        detail::TempPath tmp;
        {
            std::ofstream out(tmp.path, std::ios::binary);
            out << fin.rdbuf();
        }
        init(detail::load(tmp.path), device);
    }
    TreeGroup(const std::string& path, int device) { init(detail::load(path), device); }
    explicit TreeGroup(std::vector<Tree> t) : trees(std::move(t)) {}

    // TreeGroup::writeToFile + writePanMAN's xz stream (src/panman.cpp:6885-7015,
    // src/panmanUtils.cpp:271-299).
    void writeToFile(const std::string& path, bool compress = true) const {
        std::vector<pm_panmat> views;
        views.reserve(trees.size());
        for (const Tree& t : trees) views.push_back(t.view());
        std::vector<const pm_panmat*> list;
        for (const pm_panmat& v : views) list.push_back(&v);
        if (pm_panman_write(path.c_str(), list.data(), (int)list.size(), compress ? 1 : 0) != PM_OK)
            throw Error("cannot write " + path);
    }

  private:
    void init(detail::File f, int device) {
        const int n = pm_panman_tree_count(f.get());
        for (int i = 0; i < n; ++i) trees.emplace_back(f, i, device);
    }
};

}  // namespace panman_gpu

#endif  // PANMAN_TREE_HPP
