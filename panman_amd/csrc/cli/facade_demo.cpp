// facade_demo -- exercises include/panman_tree.hpp the way a reference caller would use
// panmanUtils::Tree / TreeGroup (tests/test_facade.py runs it on the GPU):
//   facade_demo msa     <msa.fa> <tree.nwk> <out.panman> [reference]   Tree(MSA) -> writeToFile
//   facade_demo fasta   <in.panman> <aligned 0|1>                     TreeGroup(istream) -> printFASTAUltraFast
//   facade_demo summary <in.panman>                                   printSummary(std::cout)
//   facade_demo reroot  <in.panman> <leaf> <out.panman>               reroot(leaf) -> writeToFile
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>

#include "panman_tree.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::cerr << "usage: facade_demo msa|fasta|summary|reroot ...\n";
        return 2;
    }
    const std::string cmd = argv[1];
    try {
        if (cmd == "msa" && argc >= 5) {
            std::ifstream msa(argv[2]), nwk(argv[3]);
            panman_gpu::Tree T(msa, nwk, panman_gpu::MSA, argc > 5 ? argv[5] : "");
            panman_gpu::TreeGroup TG(std::vector<panman_gpu::Tree>{T});
            TG.writeToFile(argv[4]);
            std::cout << T.getNewickString() << "\n";
            return 0;
        }
        std::ifstream in(argv[2], std::ios::binary);
        panman_gpu::TreeGroup TG(in);
        if (cmd == "fasta" && argc >= 4) {
            for (auto& T : TG.trees) T.printFASTAUltraFast(std::cout, std::atoi(argv[3]) != 0);
            return 0;
        }
        if (cmd == "summary") {
            for (auto& T : TG.trees) T.printSummary(std::cout);
            return 0;
        }
        if (cmd == "reroot" && argc >= 5) {
            TG.trees[0].reroot(argv[3]);
            TG.writeToFile(argv[4]);
            return 0;
        }
    } catch (const panman_gpu::Error& e) {
        std::cerr << "Error: " << e.what() << "\n";
        return 1;
    }
    std::cerr << "bad arguments\n";
    return 2;
}
