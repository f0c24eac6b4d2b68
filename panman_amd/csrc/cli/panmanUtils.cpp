// panmanUtils-compatible command line for the GPU path (src/panmanUtils.cpp:128-182 option
// table, :1302-1325 PanMAN load, :1409-1465 MSA build, :271-299 writePanMAN, :385-415 and
// :458-490 FASTA / aligned FASTA, :766-786 Newick).  Only the commands on the accelerated
// path are implemented; any other reference command is rejected with a message.
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "panman_gpu.h"

namespace {

using Clock = std::chrono::high_resolution_clock;

long long ns_since(Clock::time_point t0) {
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
}

struct Options {
    std::map<std::string, std::string> values;   // long name -> value ("" for flags)
    bool has(const char* k) const { return values.count(k) != 0; }
    const std::string& get(const char* k) const { return values.at(k); }
};

struct Spec {
    const char* name;
    char shortc;
    bool takes_value;
    const char* help;
};

const Spec kSpecs[] = {
    {"help", 'h', false, "Print help messages"},
    {"input-panman", 'I', true, "Input PanMAN file path"},
    {"input-msa", 'M', true, "Input MSA file (FASTA format) to build a PanMAN"},
    {"input-pangraph", 'P', true, "Input PanGraph JSON file to build a PanMAN"},
    {"input-newick", 'N', true, "Input tree topology as Newick string"},
    {"summary", 's', false, "Print PanMAN summary"},
    {"newick", 't', false, "Print newick string of all trees in a PanMAN"},
    {"fasta", 'f', false, "Print tip sequences (FASTA format)"},
    {"fasta-aligned", 'm', false, "Print MSA of sequences for each PanMAT in a PanMAN (FASTA format)"},
    {"reroot", 'r', false, "Reroot a PanMAT in a PanMAN based on the input sequence id (--reference)"},
    {"treeID", 'd', true, "Tree ID, required for --reroot"},
    {"protobuf2capnp", 0, false, "Converts a Google Protobuf PanMAN (-I) to a Cap'n Proto PanMAN (-o)"},
    {"low-mem-mode", 0, false, "Build with the Sankoff driver (the reference's batched low-memory mode)"},
    {"reference", 'n', true, "Identifier of reference sequence for PanMAN construction (optional) or reroot (required)"},
    {"output-file", 'o', true, "Prefix of the output file name"},
    {"threads", 0, true, "Accepted for compatibility (the build runs on the GPU)"},
    {"device", 0, true, "First HIP device ordinal (default 0)"},
    {"gpus", 0, true, "Number of GPUs (devices device..device+N-1): MSA columns / FASTA leaves are split across them"},
    {"backend", 0, true, "Compute backend: hip (the only one; there is no CPU product path)"},
};

// Reference commands outside the accelerated path: recognised so the error is explicit.
const char* const kOther[] = {"input-gfa", "impute", "create-network", "printTips",
                              "subnet", "vcf", "gfa", "maf", "annotate",
                              "aa-translation", "extended-newick", "printMutations", "acr", "index",
                              "toUsher"};

void usage(std::ostream& os) {
    os << "Allowed options:\n";
    for (const Spec& s : kSpecs) {
        std::string flag = "  --" + std::string(s.name);
        if (s.shortc) flag += std::string(" [ -") + s.shortc + " ]";
        if (s.takes_value) flag += " arg";
        os << flag << std::string(flag.size() < 36 ? 36 - flag.size() : 1, ' ') << s.help << "\n";
    }
}

const Spec* find_long(const std::string& n) {
    for (const Spec& s : kSpecs)
        if (n == s.name) return &s;
    return nullptr;
}

const Spec* find_short(char c) {
    for (const Spec& s : kSpecs)
        if (s.shortc == c) return &s;
    return nullptr;
}

bool parse(int argc, char** argv, Options& o, std::string& err) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        const Spec* s = nullptr;
        std::string inline_value;
        bool has_inline = false;
        if (a.rfind("--", 0) == 0) {
            std::string n = a.substr(2);
            const size_t eq = n.find('=');
            if (eq != std::string::npos) {
                inline_value = n.substr(eq + 1);
                n.resize(eq);
                has_inline = true;
            }
            s = find_long(n);
            if (!s) {
                for (const char* other : kOther)
                    if (n == other) {
                        err = "--" + n + " is not part of the GPU path of this build";
                        return false;
                    }
                err = "unrecognised option '" + a + "'";
                return false;
            }
        } else if (a.size() >= 2 && a[0] == '-') {
            s = find_short(a[1]);
            if (!s) {
                err = "unrecognised option '" + a + "'";
                return false;
            }
            if (a.size() > 2) {
                inline_value = a.substr(2);
                has_inline = true;
            }
        } else {
            o.values["input-panman"] = a;   // positional argument (src/panmanUtils.cpp:183)
            continue;
        }
        if (s->takes_value) {
            if (has_inline) {
                o.values[s->name] = inline_value;
            } else if (i + 1 < argc) {
                o.values[s->name] = argv[++i];
            } else {
                err = std::string("the required argument for option '--") + s->name + "' is missing";
                return false;
            }
        } else {
            o.values[s->name] = "";
        }
    }
    return true;
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    std::ostringstream ss;
    ss << in.rdbuf();
    out = ss.str();
    return true;
}

// a CLI phase in the same log as the library's (PANMAN_PHASES)
void cli_phase(const char* name, Clock::time_point t0) {
    if (const char* ph = std::getenv("PANMAN_PHASES"); ph && ph[0] == '1')
        std::cerr << name << "\t" << ns_since(t0) * 1e-9 << "\n";
}

void print_error(const std::string& e) { std::cerr << "\033[1;31mError: " << e << "\033[0m\n"; }

int build_from_msa(const Options& o, const std::vector<int>& devices) {
    if (!o.has("input-newick")) {
        print_error("File containing newick string not provided!");
        return 1;
    }
    if (!o.has("output-file")) {
        print_error("Output file not provided!");
        usage(std::cout);
        return 1;
    }
    std::string msa, newick;
    const auto r0 = Clock::now();
    if (!read_file(o.get("input-msa"), msa)) {
        print_error("cannot read " + o.get("input-msa"));
        return 1;
    }
    if (!read_file(o.get("input-newick"), newick)) {
        print_error("cannot read " + o.get("input-newick"));
        return 1;
    }
    cli_phase("cli.read_inputs", r0);
    const std::string ref = o.has("reference") ? o.get("reference") : "";
    const int mode = o.has("low-mem-mode") ? PM_MODE_SANKOFF : PM_MODE_FITCH;
    std::cout << "Creating PanMAN from MSA and Newick" << std::endl;
    ::mkdir("./panman", 0777);
    const std::string out = "./panman/" + o.get("output-file") + ".panman";
    const auto t0 = Clock::now();
    char err[512] = {0};
    const int rc = pm_msa_to_panman_multi(newick.c_str(), msa.c_str(), ref.c_str(), mode, devices.data(),
                                          (int)devices.size(), out.c_str(), err, sizeof err);
    if (rc != PM_OK) {
        print_error(err[0] ? err : "PanMAN construction failed");
        return 1;
    }
    // Construction and the xz write are one call here; both lines report its time.
    const long long t = ns_since(t0);
    std::cout << "Data load time: " << t << " nanoseconds \n";
    std::cout << "Writing PanMAN" << std::endl;
    std::cout << "\nNetwork Write execution time: " << t << " nanoseconds\n";
    return 0;
}

int reroot(const Options& o, const pm_panman* file, int device) {
    if (!o.has("treeID")) {
        print_error("TreeID not provided!");
        usage(std::cout);
        return 1;
    }
    const int tree_id = std::atoi(o.get("treeID").c_str());
    if (tree_id < 0 || tree_id >= pm_panman_tree_count(file)) {
        print_error("TreeID out of range");
        return 1;
    }
    if (!o.has("reference")) {
        print_error("Refence ID not provided!");
        usage(std::cout);
        return 1;
    }
    if (!o.has("output-file")) {
        print_error("Output file not provided!");
        return 1;
    }
    pm_ctx* ctx = nullptr;
    if (pm_create(device, &ctx) != PM_OK) {
        print_error("no HIP device");
        return 1;
    }
    pm_panmat view;
    pm_panman* res = nullptr;
    const auto t0 = Clock::now();
    int rc = pm_panman_tree(file, tree_id, &view);
    if (rc == PM_OK) rc = pm_reroot(ctx, &view, o.get("reference").c_str(), &res);
    if (rc != PM_OK) {
        print_error(pm_last_error(ctx));
        pm_destroy(ctx);
        return 1;
    }
    std::cout << "\nReroot execution time: " << ns_since(t0) << " nanoseconds\n";
    std::vector<pm_panmat> views(pm_panman_tree_count(file));
    std::vector<const pm_panmat*> list;
    for (int i = 0; i < (int)views.size(); ++i) {
        if (i == tree_id) pm_panman_tree(res, 0, &views[i]);
        else pm_panman_tree(file, i, &views[i]);
        list.push_back(&views[i]);
    }
    std::cout << "Writing PanMAN" << std::endl;
    ::mkdir("./panman", 0777);
    const std::string out = "./panman/" + o.get("output-file") + ".panman";
    const auto w0 = Clock::now();
    rc = pm_panman_write(out.c_str(), list.data(), (int)list.size(), 1);
    std::cout << "\nNetwork Write execution time: " << ns_since(w0) << " nanoseconds\n";
    pm_panman_free(res);
    pm_destroy(ctx);
    if (rc != PM_OK) {
        print_error("cannot write " + out);
        return 1;
    }
    return 0;
}

// -P pangraph.json -N tree.nwk -o out [-n ref] (src/panmanUtils.cpp:1364-1407)
int build_from_pangraph(const Options& o, int device) {
    if (!o.has("input-newick")) {
        print_error("File containing newick string not provided!");
        return 1;
    }
    if (!o.has("output-file")) {
        print_error("Output file not provided!");
        usage(std::cout);
        return 1;
    }
    std::string json, newick;
    if (!read_file(o.get("input-pangraph"), json)) {
        print_error("cannot read " + o.get("input-pangraph"));
        return 1;
    }
    if (!read_file(o.get("input-newick"), newick)) {
        print_error("cannot read " + o.get("input-newick"));
        return 1;
    }
    std::cout << "Creating PanMAN from PanGraph and Newick" << std::endl;
    pm_ctx* ctx = nullptr;
    if (pm_create(device, &ctx) != PM_OK) {
        print_error("no HIP device");
        return 1;
    }
    const auto t0 = Clock::now();
    pm_panman* res = nullptr;
    const std::string ref = o.has("reference") ? o.get("reference") : "";
    if (pm_pangraph_build(ctx, json.c_str(), newick.c_str(), ref.c_str(), &res) != PM_OK) {
        print_error(pm_last_error(ctx));
        pm_destroy(ctx);
        return 1;
    }
    std::cout << "Data load time: " << ns_since(t0) << " nanoseconds \n";
    std::cout << "Writing PanMAN" << std::endl;
    ::mkdir("./panman", 0777);
    const std::string out = "./panman/" + o.get("output-file") + ".panman";
    pm_panmat view;
    pm_panman_tree(res, 0, &view);
    const pm_panmat* list[1] = {&view};
    const auto w0 = Clock::now();
    const int rc = pm_panman_write(out.c_str(), list, 1, 1);
    std::cout << "\nNetwork Write execution time: " << ns_since(w0) << " nanoseconds\n";
    pm_panman_free(res);
    pm_destroy(ctx);
    if (rc != PM_OK) {
        print_error("cannot write " + out);
        return 1;
    }
    return 0;
}

// --protobuf2capnp -I old.panman -o out (src/panmanUtils.cpp:939-952, 1267-1268): the older
// Protobuf PanMAN read and written back as ./panman/<out>.panman (writePanMAN, :271-299).
int protobuf2capnp(const Options& o) {
    if (!o.has("output-file")) {
        print_error("Output file not provided!");
        usage(std::cout);
        return 1;
    }
    const std::string path = o.get("input-panman");
    std::cout << "starting reading panman" << std::endl;
    pm_panman* file = nullptr;
    char err[512] = {0};
    if (pm_panman_load_old(path.c_str(), &file, err, sizeof err) != PM_OK) {
        print_error(err[0] ? err : ("cannot load " + path));
        return 1;
    }
    std::vector<pm_panmat> views(pm_panman_tree_count(file));
    std::vector<const pm_panmat*> list;
    for (int i = 0; i < (int)views.size(); ++i) {
        pm_panman_tree(file, i, &views[i]);
        list.push_back(&views[i]);
    }
    std::cout << "Writing PanMAN" << std::endl;
    ::mkdir("./panman", 0777);
    const std::string out = "./panman/" + o.get("output-file") + ".panman";
    const auto w0 = Clock::now();
    const int rc = pm_panman_write(out.c_str(), list.data(), (int)list.size(), 1);
    std::cout << "\nNetwork Write execution time: " << ns_since(w0) << " nanoseconds\n";
    pm_panman_free(file);
    if (rc != PM_OK) {
        print_error("cannot write " + out);
        return 1;
    }
    return 0;
}

int from_panman(const Options& o, const std::vector<int>& devices) {
    const int device = devices[0];
    const std::string path = o.get("input-panman");
    if (o.has("protobuf2capnp")) return protobuf2capnp(o);
    std::cout << "starting reading panman" << std::endl;
    const auto t0 = Clock::now();
    pm_panman* file = nullptr;
    char err[512] = {0};
    if (pm_panman_load(path.c_str(), &file, err, sizeof err) != PM_OK) {
        print_error(err[0] ? err : ("cannot load " + path));
        return 1;
    }
    std::cout << "Data load time: " << ns_since(t0) << " nanoseconds \n";
    ::mkdir("./info", 0777);
    const int trees = pm_panman_tree_count(file);
    const bool to_file = o.has("output-file");
    auto sink = [&](const char* ext, int i, const char* data, size_t n) -> bool {
        if (!to_file) {   // (stdio straight to fd 1: a 5 GB FASTA text through iostream costs seconds)
            std::cout.flush();
            return std::fwrite(data, 1, n, stdout) == n && std::fflush(stdout) == 0;
        }
        const std::string p = "./info/" + o.get("output-file") + "_" + std::to_string(i) + ext;
        std::ofstream f(p, std::ios::binary);
        f.write(data, (std::streamsize)n);
        return (bool)f;
    };
    int status = 0;
    if (o.has("reroot")) {   // src/panmanUtils.cpp:855-892, then writePanMAN
        status = reroot(o, file, device);
        pm_panman_free(file);
        return status;
    }
    if (o.has("summary")) {   // src/panmanUtils.cpp:356-384, Tree::printSummary (src/summary.cpp:257-273)
        pm_ctx* ctx = nullptr;
        if (pm_create(device, &ctx) != PM_OK) {
            print_error("no HIP device");
            pm_panman_free(file);
            return 1;
        }
        const auto s0 = Clock::now();
        for (int i = 0; i < trees && status == 0; ++i) {
            pm_panmat view;
            pm_summary sm;
            if (pm_panman_tree(file, i, &view) != PM_OK || pm_summary_compute(ctx, &view, &sm) != PM_OK) {
                print_error(pm_last_error(ctx));
                status = 1;
                break;
            }
            std::ostringstream out;
            out << "Total Nodes in Tree: " << sm.nodes << std::endl;
            out << "Total Samples in Tree: " << sm.samples << std::endl;
            out << "Total Substitutions: " << sm.substitutions << std::endl;
            out << "Total Insertions: " << sm.insertions << std::endl;
            out << "Total Deletions: " << sm.deletions << std::endl;
            out << "Total Inversions: " << sm.inversions << std::endl;
            out << "Max Tree Depth: " << sm.max_depth << std::endl;
            out << "Mean Tree Depth: " << sm.mean_depth << std::endl;
            const std::string text = out.str();
            if (!sink(".summary", i, text.data(), text.size())) status = 1;
            // getBlockMutationsParallel prints to std::cout whatever the output file (:203-250)
            std::cout << "Total Block Insertions: " << sm.block_insertions << std::endl;
            std::cout << "Total Block Deletions: " << sm.block_deletions << std::endl;
            std::cout << "Total Block Inversion: " << sm.block_inversions << std::endl;
            std::cout << "Total Block Duplications: " << sm.block_duplications << std::endl;
            std::cout << "Total Block Translocation: " << sm.block_translocations << std::endl;
        }
        std::cout << "\nSummary creation time: " << ns_since(s0) << " nanoseconds\n";
        pm_destroy(ctx);
    }
    if (o.has("newick")) {
        for (int i = 0; i < trees; ++i) {
            std::string s = pm_panman_newick(file, i);
            s += "\n";
            if (!sink(".newick", i, s.data(), s.size())) status = 1;
        }
    }
    for (int aligned = 0; aligned < 2 && status == 0; ++aligned) {
        if (!o.has(aligned ? "fasta-aligned" : "fasta")) continue;
        const auto f0 = Clock::now();
        for (int i = 0; i < trees && status == 0; ++i) {
            pm_panmat view;
            int64_t len = 0;
            char err[512] = {0};
            // the text streams from the device(s) straight to stdout or the output file
            // (pm_fasta_multi_fd): no host copy of the whole text, the write overlaps the download
            int fd = 1;
            if (to_file) {
                const std::string p = "./info/" + o.get("output-file") + "_" + std::to_string(i) + (aligned ? ".msa" : ".fasta");
                fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
                if (fd < 0) {
                    print_error("cannot write " + p);
                    status = 1;
                    break;
                }
            } else {
                std::cout.flush();
                std::fflush(stdout);
            }
            const auto w0 = Clock::now();
            if (pm_panman_tree(file, i, &view) != PM_OK ||
                pm_fasta_multi_fd(&view, aligned, devices.data(), (int)devices.size(), fd, &len, err, sizeof err) != PM_OK) {
                print_error(err[0] ? err : "FASTA extraction failed");
                status = 1;
            }
            if (to_file && ::close(fd) != 0) status = 1;
            cli_phase("cli.fasta_stream", w0);
            if (status) break;
        }
        std::cout << "\nFASTA execution time: " << ns_since(f0) << " nanoseconds\n";
    }
    pm_panman_free(file);
    return status;
}

int run(int argc, char** argv);

}  // namespace

// Builds whose tools write their results at exit always take the normal exit: sanitizers
// (LeakSanitizer's report) are detected; a coverage build (gcc defines no macro for
// --coverage) adds -DPM_CLI_NORMAL_EXIT.
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__) || defined(PM_CLI_NORMAL_EXIT)
constexpr bool kFastExitAllowed = false;
#elif defined(__has_feature)
#if __has_feature(address_sanitizer) || __has_feature(thread_sanitizer) || __has_feature(memory_sanitizer)
constexpr bool kFastExitAllowed = false;
#else
constexpr bool kFastExitAllowed = true;
#endif
#else
constexpr bool kFastExitAllowed = true;
#endif

// PANMAN_PHASES=1: the library's phase log (pm_phase_report: HIP init, parse, upload, GPU
// run, grouping, capnp, xz, download ...) and the CLI's own wall time, on stderr.
int main(int argc, char** argv) {
    pm_phase_reset();
    const auto t0 = Clock::now();
    const int rc = run(argc, argv);
    const char* ph = std::getenv("PANMAN_PHASES");
    if (ph && ph[0] == '1') {
        std::vector<char> buf((size_t)pm_phase_report(nullptr, 0));
        pm_phase_report(buf.data(), (int64_t)buf.size());
        std::cerr << "#phases\n" << buf.data() << "cli.total\t" << ns_since(t0) * 1e-9 << "\n";
    }
    // Every output file is closed and every context destroyed by now; what a normal exit adds
    // is the HIP / HSA runtime's own teardown in static destructors, which the kernel driver
    // does anyway when the process ends.  Skipped, unless a profiler whose results are written
    // at exit is preloaded, the build carries a sanitizer or coverage (kFastExitAllowed), or
    // PM_CLI_FULL_EXIT=1.
    const char* pre = std::getenv("LD_PRELOAD");
    const char* full = std::getenv("PM_CLI_FULL_EXIT");
    if (kFastExitAllowed && !(full && full[0] == '1') && !(pre && std::strstr(pre, "rocprof"))) {
        std::cout.flush();
        std::cerr.flush();
        std::fflush(nullptr);
        _exit(rc);
    }
    return rc;
}

namespace {

int run(int argc, char** argv) {
    Options o;
    std::string err;
    if (!parse(argc, argv, o, err)) {
        print_error(err);
        usage(std::cerr);
        return 1;
    }
    if (o.has("help") || argc == 1) {
        usage(std::cout);
        return 0;
    }
    if (o.has("backend") && o.get("backend") != "hip") {
        print_error("--backend " + o.get("backend") + ": this build computes on the GPU only (use --backend hip)");
        return 1;
    }
    const int device = o.has("device") ? std::atoi(o.get("device").c_str()) : 0;
    const int gpus = o.has("gpus") ? std::atoi(o.get("gpus").c_str()) : 1;
    if (gpus < 1 || gpus > 64) {
        print_error("--gpus must be between 1 and 64");
        return 1;
    }
    std::vector<int> devices;
    for (int g = 0; g < gpus; ++g) devices.push_back(device + g);
    // -I: HIP initialisation and the code objects' load (~0.1 s) on a thread of their own,
    // while this one reads and xz-decodes the PanMAN (C5: 0.3 s; measured 0.06-0.08 s off the
    // command).  Not for -M, whose input is parsed in ~10 ms: there the extra code-object
    // loads only delayed the build (PM_CLI_NO_WARMUP=1: never).
    struct Warm {
        std::thread t;
        ~Warm() {
            if (t.joinable()) t.join();
        }
    } warm;
    if (const char* nw = std::getenv("PM_CLI_NO_WARMUP");
        !(nw && nw[0] == '1') && o.has("input-panman") && !o.has("input-msa") && !o.has("input-pangraph"))
        warm.t = std::thread([device] { (void)pm_warmup(device); });
    if (o.has("input-pangraph")) return build_from_pangraph(o, device);
    if (o.has("input-msa")) return build_from_msa(o, devices);
    if (o.has("input-panman")) return from_panman(o, devices);
    print_error("no input: give -I <file.panman> or -M <msa> -N <newick>");
    usage(std::cerr);
    return 1;
}

}  // namespace
