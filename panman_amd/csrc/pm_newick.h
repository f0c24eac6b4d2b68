// pm_newick.h -- Newick topology with the reference's node naming (shared by the MSA
// drivers and the PanMAN loader).
#pragma once

#include <string>
#include <vector>

namespace pm {

// Nodes numbered in creation order, which is the pre-order of the Newick text; internal
// nodes are named node_<k> in order of '(' and internal labels are ignored
// (src/panman.cpp:310-450, src/panman.hpp:793-795).
struct Topology {
    std::vector<std::string> name;
    std::vector<std::vector<int32_t>> kids;
    std::vector<float> length;   // branch length per node (root 0)
    int32_t root = -1;
};

std::vector<std::string> split_quoted(const std::string& s, char delim);
bool parse_topology(std::string text, Topology& t, std::string& err);
// Tree::getNewickString (src/panman.cpp:1921-2029): leaves "name:len", clades
// "(...)name:len", lengths printed with "%f", terminated by ';'.  Empty `length` prints
// the parser's defaults (1 for every node, 0 for the root).
std::string newick_of(const Topology& t);

}  // namespace pm
