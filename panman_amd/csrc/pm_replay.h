// pm_replay.h -- replay state shared by the FASTA path (pm_replay.cpp) and the reroot
// driver (pm_reroot.cpp).
#pragma once

#include <string>
#include <vector>

#include "pm_internal.h"

namespace pm {

struct ReplayState {
    // topology
    int32_t num_nodes = 0;
    std::vector<std::string> names;
    std::vector<int32_t> parent;
    std::vector<int32_t> leaves;                 // leaf node ids, increasing
    // blocks, indexed by primary id (0..max_id)
    int32_t max_id = -1;
    std::vector<uint8_t> is_block;               // [max_id+1]
    std::vector<int64_t> col_start, width;       // canonical columns per block
    std::vector<int64_t> absent_len;             // blockLengths when absent (len + sum of gap lengths)
    int64_t columns = 0;
    // per leaf (host, for the formatter)
    std::vector<std::vector<uint8_t>> present;   // [leaf][max_id+1]
    std::vector<std::vector<uint8_t>> exists, strand;
    std::vector<int32_t> circular, rotation;
    std::vector<uint8_t> inverted;
    int64_t edits = 0;
    // canonical layout (host): consensus row, and per block the column of main position j
    // and of the first gap slot before j, plus the slot counts
    std::string cons;
    std::vector<std::vector<int64_t>> main_col, gap_col;
    std::vector<std::vector<int32_t>> slots;
    // device
    ReplayDev dev{};
    char* d_rows = nullptr;
    char* d_cons = nullptr;
    int32_t* d_parent = nullptr;
    int32_t* d_leaf = nullptr;
    uint32_t* d_presence = nullptr;
    int64_t* d_eoff = nullptr;
    uint32_t* d_ecol = nullptr;
    uint8_t* d_echr = nullptr;
    int64_t* d_blk_lo = nullptr;
    int64_t* d_blk_hi = nullptr;
    int32_t* d_tile_blk = nullptr;
    int2* d_tile2 = nullptr;
    int32_t *d_dfs_row = nullptr, *d_g_leaf_off = nullptr, *d_g_union_off = nullptr, *d_g_union = nullptr;
    uint16_t *d_dfs_len = nullptr, *d_dfs_lpfx = nullptr;
    int64_t* d_path_off = nullptr;
    int32_t* d_path = nullptr;
    int32_t* d_rebuilds = nullptr;   // [1] ReplayDev::dfs_rebuilds
    bool ran = false;
};

// Flatten a PanMAT for the GPU (canonical columns, per-node edits, per-leaf block state)
// and upload it; the rows are produced by launch_replay(c, r.dev).
// Leaves [leaf_begin, leaf_end) of the PanMAT's leaves in node-id order (-1, -1: all).
int replay_prepare(pm_ctx* c, const pm_panmat* p, ReplayState& r, int64_t leaf_begin = -1, int64_t leaf_end = -1);
// Host arrays of a flattened PanMAT that the replay kernels read (uploaded by replay_prepare).
struct ReplayHost {
    std::vector<char> cons_row;
    std::vector<uint32_t> presence;
    std::vector<int64_t> eoff;
    std::vector<uint32_t> ecol;
    std::vector<uint8_t> echr;
    std::vector<int64_t> blk_lo, blk_hi, tile_edit, path_off;   // (tile_edit: flattening scratch)
    std::vector<int2> tile2;   // [N][tiles + 1] {first plain edit, first overriding edit}
    std::vector<int32_t> tile_blk, path_all;
    int32_t max_depth = 0, words = 0, tiles = 0, tile_bytes = 0;
    // leaf groups for k_replay_dfs (dfs: every path fits kDfsUnionCap)
    bool dfs = false;
    std::vector<int32_t> dfs_row, g_leaf_off, g_union_off, g_union;
    std::vector<uint16_t> dfs_len, dfs_lpfx;
    int64_t stride = 0;
};
// Its host half (no device call): fills r and the arrays replay_prepare uploads.
int replay_flatten(const pm_panmat* p, ReplayState& r, ReplayHost& h, int64_t leaf_begin, int64_t leaf_end,
                   std::string& err_msg);

}  // namespace pm
