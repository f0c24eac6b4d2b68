// pm_panman_tree.h -- owned PanMAT storage behind pm_panman handles (loader, reroot).
#pragma once

#include <string>
#include <vector>

#include "../../include/panman_gpu.h"

namespace pm {

// One loaded tree, owning the arrays a pm_panmat view points into.
struct PanmanTree {
    std::string names_blob;
    std::vector<int32_t> child_off, child_idx;
    int32_t root = 0;
    std::vector<int32_t> block_primary;
    std::vector<int64_t> block_seq_off;
    std::vector<uint32_t> block_seq;
    std::vector<int32_t> gap_primary;
    std::vector<int64_t> gap_off;
    std::vector<uint32_t> gap_pos, gap_len;
    std::vector<int64_t> bm_off;
    std::vector<int32_t> bm_primary;
    std::vector<uint8_t> bm_info, bm_inv;
    std::vector<int64_t> nm_off;
    std::vector<int32_t> nm_primary, nm_secondary, nm_pos, nm_gap;
    std::vector<uint8_t> nm_info;
    std::vector<uint32_t> nm_nucs;
    std::vector<int32_t> circular, rotation;
    std::vector<uint8_t> inverted;
    std::vector<float> length;
    std::string newick;
    int32_t num_nodes = 0;

    void view(pm_panmat& v) const {
        v.num_nodes = num_nodes;
        v.root = root;
        v.child_offsets = child_off.data();
        v.child_index = child_idx.data();
        v.names = names_blob.data();
        v.num_blocks = (int32_t)block_primary.size();
        v.block_primary = block_primary.data();
        v.block_seq_offsets = block_seq_off.data();
        v.block_seq = block_seq.data();
        v.num_gaps = (int32_t)gap_primary.size();
        v.gap_primary = gap_primary.data();
        v.gap_offsets = gap_off.data();
        v.gap_position = gap_pos.data();
        v.gap_length = gap_len.data();
        v.block_mut_offsets = bm_off.data();
        v.block_mut_primary = bm_primary.data();
        v.block_mut_info = bm_info.data();
        v.block_mut_inversion = bm_inv.data();
        v.nuc_mut_offsets = nm_off.data();
        v.nuc_mut_primary = nm_primary.data();
        v.nuc_mut_secondary = nm_secondary.data();
        v.nuc_mut_position = nm_pos.data();
        v.nuc_mut_gap_position = nm_gap.data();
        v.nuc_mut_info = nm_info.data();
        v.nuc_mut_nucs = nm_nucs.data();
        v.circular_offset = circular.data();
        v.rotation_index = rotation.data();
        v.sequence_inverted = inverted.data();
        v.branch_length = length.data();
    }
};

}  // namespace pm

struct pm_panman {
    std::vector<pm::PanmanTree> trees;
    std::string err;
};
