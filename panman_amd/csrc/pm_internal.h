// pm_internal.h -- context layout shared by the host side and the kernel launchers.
//
// HBM layout (one pm_ctx = one GPU = one shard of S sites, W = ceil(S/32) words):
//   leaf planes   [L][W] uint4     4 code bit-planes of 32 sites (16 B / 32 sites)
//   leaf present  [L][W] uint32    only for leaves with partially present columns
//   Fitch sets    [I][tile] records: 4 code planes per word; a word holding a multi-code or
//                 empty set adds its multi-code sites' 16-bit sets (compact complex lanes,
//                 pm_kernels.h store_fitch_set)
//   Sankoff sets  [I][W][32] u32   Z0 (optimal codes) + Z1 (one above optimal) planes
//   finals        the root's in root_final [W] uint4; every other internal node's in its
//                 record (complex lanes: quad 0 of the lane's slot; others: the record code)
//   consensus     [W] uint4        root's parent state; forced [W] uint4 (optional)
//   records       [shards][cap]    pm_mut, sharded write cursors (one atomic per wave)
// Internal nodes are addressed by a dense index (0..I-1), leaves by their rank among
// leaf node ids (0..L-1).  A child is encoded as its dense internal index (>= 0) or
// -(leaf rank + 1).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/panman_gpu.h"

namespace pm {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
#ifndef PM_SHARDS
#define PM_SHARDS 1024
#endif
constexpr int kShards = PM_SHARDS;
constexpr int kClasses = 6;   // post-order, pre-order levels, score, replay, whole graph, pre-order tail
constexpr int kDegreeClasses = 4;
// Compact complex lanes (Fitch records, pm_kernels.h cx_store): a complex word stores its code
// planes, its multi-code-site mask and up to kCxSets 16-bit sets (32 B) instead of 16 planes
// (64 B); 0 = the 16-plane format.  Record quads per word: simple area + complex areas.
#ifndef PM_CX_COMPACT
#define PM_CX_COMPACT 0
#endif
constexpr bool kCxCompact = PM_CX_COMPACT != 0;
constexpr int kFitchRecQuads = kCxCompact ? 6 : 5;
constexpr int kMaskWords = 8;     // record masks per (node, tile): complex, simple, dirty, parent's
                                  // complex, parent's simple, an S2 / S3 node's pushed dirty lanes,
                                  // Fitch: the first / second child's dirty lanes (one 64-B line)
// Grouped post-order launches (PM_OPT_UP_GROUP): heights of at most this many nodes group.
#ifndef PM_UP_GROUP_NODES
#define PM_UP_GROUP_NODES 2048
#endif
constexpr int32_t kUpGroupNodes = PM_UP_GROUP_NODES;

// ... and a node recomputes same-launch descendants at most this many levels down (a node
// recomputing a child that itself recomputes one: depth 2; such a chain holds one child per level).
#ifndef PM_UP_GROUP_DEPTH
#define PM_UP_GROUP_DEPTH 2
#endif
constexpr int kUpGroupDepth = PM_UP_GROUP_DEPTH;
inline int degree_class(int32_t deg) { return deg <= 3 ? 0 : deg <= 15 ? 1 : deg <= 255 ? 2 : 3; }

enum LeafFlag : uint8_t { kLeafAbsent = 0, kLeafPresent = 1, kLeafPartial = 2 };

// Level item of the Fitch / Sankoff passes: everything a wave needs to start its loads,
// in one 64-B scalar load (node, parent, child range, the first two children's encodings
// and, for virtual leaf-parent children, their leaves).
struct alignas(64) NodeDesc {
    int32_t node, parent, e0, e1;
    int32_t c0, c1, pad0, pad1;    // pad0: Sankoff up parts -- the first part; pre-order -- the grandparent, pad1 the great-grandparent (dense, -1)
    int32_t vl0[4], vl1[4];
};

// A leaf or virtual child beyond a node's first two (polytomies): its records need only
// the parent's final, so they are emitted by one flat launch after the pre-order levels
// instead of serially inside the parent's wave.
// Everything the tail wave needs is in the descriptor (one 64-B scalar load): no dependent
// id lookups (leaf_id[vl], internal_id[vinner]) between the descriptor and the records.
struct alignas(64) TailDesc {
    int32_t parent, enc, ix, iy;   // ix / iy: an S2 / S3 child's cherries (caller node ids), else -1
    int32_t vl[4];                 // a virtual child's leaves (ranks), -1 padded
    int32_t id[5];                 // caller node ids: the child itself, then its leaves vl[0..3]
    int32_t pad[3];
};

// Sankoff nodes of out-degree > 255: their children are cut into parts of kPartChildren,
// counted separately into 8-bit counters (16 codes x 8 planes + the finite plane).
constexpr int kPartChildren = 255;
constexpr int kPartPlanes = 16 * 8 + 1;
struct PartDesc {
    int32_t item;     // the node's position in its up-order descriptor array
    int32_t sub;      // children [e0 + sub * kPartChildren, ...)
    int32_t global;   // scratch slot
    int32_t pad;
};

struct DevTree {
    int32_t num_internal = 0;
    int32_t num_leaves = 0;
    int32_t root_dense = -1;          // dense index of the root (internal)
    int32_t* child_off = nullptr;     // [I+1] over dense internal index
    int32_t* child_enc = nullptr;     // [E]
    int32_t* parent_dense = nullptr;  // [I] parent dense index, -1 for the root
    int32_t* internal_id = nullptr;   // [I] caller node id
    int32_t* leaf_id = nullptr;       // [L] caller node id
    int32_t* up_order = nullptr;      // [I] dense indices grouped by height (post-order levels)
    int32_t* down_order = nullptr;    // [I] dense indices grouped by depth (pre-order levels)
    int32_t* leaf_parent = nullptr;   // [L] parent dense index (synthetic generator)
    int32_t* leaf_down = nullptr;     // [L] leaf ranks grouped by depth (synthetic generator)
    // Fitch with "virtual" leaf-parents: an internal node whose children are all leaves
    // (<= 4) is never materialised; its parent evaluates it from the leaves in both passes
    int32_t* child_enc_v = nullptr;   // [E] as child_enc, virtual children tagged kVirtualBit
    int32_t* up_order_v = nullptr;    // [I'] materialised internal nodes by height
    int32_t* down_order_v = nullptr;  // [I'] materialised internal nodes by depth
    // down-pass item descriptors {node, parent, first child, end child} (int4), in
    // down_order / down_order_v order, and each virtual node's leaves (int4, -1 padded)
    NodeDesc* down_desc = nullptr;
    NodeDesc* up_desc = nullptr;      // in up_order order
    NodeDesc* up_desc_v = nullptr;
    NodeDesc* down_desc_v = nullptr;
    int32_t* vleaf = nullptr;
    TailDesc* tail_desc = nullptr;     // tails over child_enc
    TailDesc* tail_desc_v = nullptr;   // tails over child_enc_v
    // Sankoff parts of the nodes of out-degree > 255 ([0] over child_enc, [1] over child_enc_v)
    PartDesc* part_desc = nullptr;
    PartDesc* part_desc_v = nullptr;
    PartDesc* part_desc_k = nullptr;   // subtree form (Sankoff)
    PartDesc* part_desc_gs = nullptr;  // grouped subtree form (Sankoff)
    // subtree form (Fitch, all leaves present): S2 / S3 nodes inline in their parent too
    int32_t* child_enc_k = nullptr;   // [E] shapes in bits 28-29
    NodeDesc* up_desc_k = nullptr;
    NodeDesc* up_desc_g = nullptr;     // grouped post-order launches of the subtree form
    NodeDesc* up_desc_gs = nullptr;    // ... Sankoff's (binary recomputed children; pad0 = first part above 255 children)
    NodeDesc* down_desc_k = nullptr;
    NodeDesc* down_desc_ks = nullptr;  // ... with their S2 / S3 children kept (PM_OPT_SUB_DOWN)
    int32_t* vinner = nullptr;        // [I][2] an S2 / S3 node's cherries (dense), -1 padded
    // up slots (UpArgs::upm): per up_desc_k / up_desc_g item, parent item * 2 + slot, or -1
    int32_t* pslot_k = nullptr;
    int32_t* pslot_g = nullptr;
    int32_t* pslot_gs = nullptr;      // ... of up_desc_gs (Sankoff's groups)
    TailDesc* tail_desc_k = nullptr;  // tails of the leaf-parent form + every S2 / S3 node
    // LDS-staged post-order sweeps (ClusterPlan on the device)
    NodeDesc* cl_items = nullptr;
    NodeDesc* cl_down_items = nullptr;
    int32_t* cl_wg_off = nullptr;
    int32_t* cl_slot_of = nullptr;
    // up slots with the sweeps (UpArgs::upm: the level items', then the sweep items' at
    // up_items_k + item): the level items' pslot, and each sweep item's (its parent in a later band)
    int32_t* pslot_kc = nullptr;
    int32_t* pslot_gc = nullptr;
    int32_t* cl_pslot = nullptr;
    // level tables on the device (the narrow-band launches walk several levels): the host
    // arrays up_class_off{,_v,_k}, down_level_off{,_v,_k}, down_dense_base_k back to back
    int32_t* lvl = nullptr;
};

// LDS-staged post-order sweeps (PM_OPT_CLUSTER, pm_cluster.cpp): LDS set slots per cluster wave
// (4 KiB each), most nodes per cluster, most heights per band
#ifndef PM_CL_SLOTS
#define PM_CL_SLOTS 4
#endif
constexpr int kClSlots = PM_CL_SLOTS;
#ifndef PM_CL_MAX_STEPS
#define PM_CL_MAX_STEPS 64
#endif
constexpr int32_t kClMaxSteps = PM_CL_MAX_STEPS;
#ifndef PM_CL_BAND
#define PM_CL_BAND 32
#endif
constexpr int32_t kClBandHeights = PM_CL_BAND;
// default PM_OPT_CLUSTER: the sweeps take the post-order from the first height whose level
// and every level above it hold at most this many materialised nodes (and above the last band
// whose clusters are bushy: more than kClChain nodes per level in its longest cluster)
#ifndef PM_CL_MAX_LEVEL
#define PM_CL_MAX_LEVEL (1 << 20)
#endif
#ifndef PM_CL_CHAIN
#define PM_CL_CHAIN 4
#endif
constexpr int32_t kClChain = PM_CL_CHAIN;
// ... or wide: more clusters than this (a level kernel's waves then fill the GPU as well, and
// its nodes run side by side where a cluster's run one after another).  C4 (T2) share
// 27.74 -> 26.88 ms (its bands below height 62 hold 25k-454k clusters), C3 unchanged (its
// widest band: 5.2k clusters); 4096 / 32768: 27.44 / 27.10 ms (r06mc, tools/gpu_r06mc.sh)
#ifndef PM_CL_MAX_CLUSTERS
#define PM_CL_MAX_CLUSTERS 16384
#endif
constexpr int32_t kClMaxClusters = PM_CL_MAX_CLUSTERS;
constexpr int32_t kClMaxLevel = PM_CL_MAX_LEVEL;
#ifndef PM_CL_FSLOTS
#define PM_CL_FSLOTS 8
#endif
constexpr int kClFSlots = PM_CL_FSLOTS;   // the pre-order sweeps' LDS final slots (1 KiB each)

struct ClusterPlan {
    int32_t h0 = 0;                  // first post-order level (subtree form) the sweeps take
    int32_t max_rounds = 0;          // steps of the longest cluster
    std::vector<NodeDesc> items;     // per cluster: its nodes in step order; parent = the node's
                                     // LDS slot, pad0 / pad1 its first two children's slots (-1:
                                     // not in the cluster)
    std::vector<int32_t> wg_off;     // [clusters + 1] item offsets
    std::vector<int32_t> band_wg;    // [bands + 1] cluster offsets
    std::vector<int32_t> band_level; // [bands + 1] first level of each band
    std::vector<int32_t> slot_of;    // [I] a node's slot (children beyond the first two), -1
    std::vector<int32_t> item_of;    // [I] a swept node's (first) item, -1
    int32_t n_items = 0;
    int32_t max_degree = 0;          // the items' largest out-degree (Sankoff sweeps: <= 255)
    int32_t upm_base = 0;            // the items' up slots follow both up orders' (UpArgs::upm)
    // the pre-order over the same clusters (plan_cluster_down; empty: the level kernels): per
    // cluster its nodes in depth-first pre-order; pad0 = the slot of the parent's final, pad1
    // = this node's (-1: none)
    std::vector<NodeDesc> down_items;
    bool down = false;
};

constexpr int32_t kVirtualBit = 1 << 30;
// Subtree form: a virtual child's shape in bits 28-29 of its encoding (0 = one or two leaves,
// 1 = S2 (cherry, leaf), 2 = S3 (cherry, cherry)); the dense index is the low 28 bits.
constexpr int kShapeShift = 28;
constexpr int32_t kDenseMask = (1 << kShapeShift) - 1;

struct HostTree {
    int32_t num_nodes = 0;
    int32_t root = -1;
    std::vector<int32_t> dense_of;        // [N] dense internal index or -(leaf rank + 1)
    std::vector<int32_t> internal_id;     // [I]
    std::vector<int32_t> leaf_id;         // [L]
    std::vector<int32_t> up_level_off;    // [H+1] offsets into up_order (level 0 = height 1)
    std::vector<int32_t> up_class_off;    // [4H+1] within a level, nodes by out-degree class
                                          // (<=3, <=15, <=255, more): Sankoff counter widths
    std::vector<int32_t> down_level_off;  // [D+1] offsets into down_order (level 0 = root)
    std::vector<int32_t> leaf_level_off;  // [D+1] offsets into leaf_down by depth
    std::vector<int32_t> child_off;       // dense CSR (host copy)
    std::vector<int32_t> child_enc;
    std::vector<int32_t> up_level_off_v;    // levels of up_order_v / down_order_v
    std::vector<int32_t> up_class_off_v;    // [4H+1] (level, degree class) buckets of up_order_v
    std::vector<uint8_t> up_leafy_v;        // [H] level's out-degree <= 3 nodes have leaf / virtual children only
    std::vector<int32_t> down_level_off_v;
    int64_t num_virtual = 0;
    bool down_dense_v = false;            // down_order_v[k] == k (dense order = pre-order levels)
    int32_t num_tail = 0, num_tail_v = 0;
    // Sankoff parts: prefix over the up-order descriptors ([I'+1]; nodes of out-degree <= 255
    // have none) of each form, and every descriptor's out-degree
    std::vector<int32_t> part_off, part_off_v, part_off_k, part_off_gs;
    std::vector<int32_t> up_degree[4];   // [0] plain, [1] leaf-parent form, [2] subtree form, [3] its Sankoff groups
    // subtree form: levels without the S2 / S3 nodes, each pre-order level's first dense index
    std::vector<int32_t> up_level_off_k, up_class_off_k, down_level_off_k, down_dense_base_k;
    std::vector<uint8_t> up_leafy_k;
    // subtree form, grouped post-order launches (PM_OPT_UP_GROUP): launch l's nodes by class
    std::vector<int32_t> up_level_off_g, up_class_off_g;
    std::vector<uint8_t> up_leafy_g, up_recomp_g;   // (recomp: some node of the launch recomputes a child)
    // ... and each launch's "plain" nodes at the front of its out-degree <= 3 class: binary, no
    // S2 / S3 child, no recomputed child -- the lean, higher-occupancy kernel (k_fitch_up<.., PLAIN>)
    std::vector<int32_t> up_plain_g, up_plain_gs;
    // ... and Sankoff's (a recomputed child must be binary)
    std::vector<int32_t> up_level_off_gs, up_class_off_gs;
    std::vector<uint8_t> up_leafy_gs, up_recomp_gs;
    bool down_dense_k = false;
    int32_t up_items_k = 0, up_items_g = 0, up_items_gs = 0;   // descriptor counts (up slot storage)
    int64_t num_sshape = 0;
    std::vector<uint8_t> sshape;          // [I] 1: S2, 2: S3 (subtree form), else 0
    int32_t num_tail_k = 0;
    int32_t num_tail_s = 0;               // subtree form: the first num_tail_s tail items are the S2 / S3 nodes
    int32_t sbase = -1;                   // ... dense indices sbase + item
    // offsets of the level tables in DevTree::lvl: [form] = plain, leaf-parent, subtree form,
    // (up only) its Fitch groups, its Sankoff groups
    int64_t lvl_up[5] = {0, 0, 0, 0, 0}, lvl_down[3] = {0, 0, 0}, lvl_base_k = 0;
    // LDS-staged post-order sweeps of the subtree form (items and slots on the device only)
    ClusterPlan cl;
};

// pm_cluster.cpp: the band / cluster / round / slot schedule above the first level of at most
// max_level nodes (0: none)
int plan_clusters(const HostTree& ht, const std::vector<int32_t>& up_order_k, const std::vector<int32_t>& child_enc_k,
                  const std::vector<int32_t>& parent_dense, const std::vector<int32_t>& vleaf, int32_t max_level,
                  bool chain_check, ClusterPlan& out);
bool plan_cluster_down(const HostTree& ht, const std::vector<int32_t>& down_order_k, const std::vector<NodeDesc>& down_desc_k,
                       const std::vector<int32_t>& child_enc_k, ClusterPlan& cl);

struct Timer {
    hipEvent_t a = nullptr, b = nullptr;
};

}  // namespace pm

namespace pm { struct ReplayState; }

struct pm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    // a second stream for independent launches of one level (side_fork / side_join)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    std::string err;

    pm::HostTree ht;
    pm::DevTree dt;
    size_t tree_bytes = 0;            // device bytes of the flattened tree (descriptors, level tables)
    bool has_tree = false;
    int32_t max_degree = 0;
    bool virtual_leaf_parents = true; // Fitch: leaf-parents evaluated inline (PM_OPT_VIRTUAL)
    bool subtree_form = true;         // Fitch, all leaves present: S2 / S3 inline too (PM_OPT_SUBTREE)
    int32_t narrow_max = 16;          // Fitch: runs of levels this narrow go to one band launch (PM_OPT_NARROW)
    int64_t group_waves = 32768;      // Fitch: pre-order levels grouped into one launch up to this many waves (PM_OPT_GROUP_WAVES)
    int32_t group_levels = 4;         // ... and up to this many levels (PM_OPT_GROUP_LEVELS)
    bool up_group = true;             // Fitch subtree form: grouped post-order launches (PM_OPT_UP_GROUP)
    bool sub_down = false;            // Fitch subtree form: S2 / S3 records in their parent's pre-order wave (PM_OPT_SUB_DOWN)
    bool plain_up = true;             // grouped subtree form: plain nodes in the lean post-order kernels (PM_OPT_PLAIN_UP)
    int64_t plain_min_waves = 0;      // ... from this many (node, tile) waves (0: kPlainMinWaves)
    bool cluster = true;              // Fitch subtree form: LDS-staged post-order sweeps above ht.cl.h0 (PM_OPT_CLUSTER)
    int32_t cluster_max_level = pm::kClMaxLevel;   // ... their plan's level threshold (at tree upload)
    bool cluster_chain = true;        // ... and only above the last bushy band (the default; an explicit threshold: off)

    // column shard
    int64_t num_sites = 0;
    int32_t words = 0;
    uint4* leaf_planes = nullptr;     // [L][W]
    uint32_t* leaf_present = nullptr; // [L][W] (allocated only when needed)
    uint8_t* leaf_flag = nullptr;     // [L]
    uint4* cons = nullptr;            // [W]
    uint4* forced = nullptr;          // [W]
    bool has_forced = false;
    bool has_leaves = false;
    bool leaves_all_present = false;   // every leaf row present at every site
    bool has_sites = false;

    // work buffers
    uint32_t* sets = nullptr;         // Fitch: [I][tile] 320 uint4 records; Sankoff: [I][W][32]
    size_t sets_bytes = 0;
    uint64_t* cmask = nullptr;        // Fitch: [I][tile] complex-lane masks
    size_t cmask_bytes = 0;
    uint64_t* upm = nullptr;          // Fitch subtree form: [up items][tile][4] up slots (UpArgs::upm)
    size_t upm_bytes = 0;
    uint4* finals = nullptr;          // [I][W] synthetic generator scratch (internal sequences)
    size_t finals_bytes = 0;
    uint32_t* sk_parts = nullptr;     // Sankoff part counters [parts][kPartPlanes][wpad]
    size_t sk_parts_bytes = 0;
    uint4* root_final = nullptr;      // [W] the root's final codes (other finals live in the records)
    pm_mut* recs = nullptr;           // [kShards][shard_cap]
    int64_t shard_cap = 0;
    int64_t record_cap = 0;           // PM_OPT_RECORD_CAP: first allocation per shard (0 = a guess)
    uint32_t* shard_cnt = nullptr;    // [kShards]
    // subtree form: each S2 / S3 node's three or four leaf words side by side per word
    // ([num_tail_s][wpad][4] uint4, built from leaf_planes by build_sub_planes), so a wave that
    // reads a subtree's leaves at scattered lanes draws one 64-B sector per lane, not four
    uint4* sub_planes = nullptr;
    size_t sub_planes_bytes = 0;
    bool sub_planes_ok = false;
    int32_t* score = nullptr;         // [S]
    uint8_t* root_code = nullptr;     // [S]
    bool ran = false;
    int last_mode = -1;

    // profiling
    bool profiling = false;
    std::vector<pm::Timer> timers[pm::kClasses];
    size_t timers_used[pm::kClasses] = {0, 0, 0, 0, 0, 0};

    // hipGraph of one pm_run (PM_OPT_GRAPH): captured on first use, replayed while the
    // launch sequence and every buffer it touches stay the same (graph_key)
    bool use_graph = false;
    int32_t nt_loads = -1;            // PM_OPT_NT_LOADS: -1 by level size (nt_policy), 0 off, 1 on
    hipGraphExec_t graph_exec = nullptr;
    uint64_t graph_key = 0;

    // replay (pm_replay.cpp)
    pm::ReplayState* replay = nullptr;

    // multi-GPU column shards (pm_rccl.hip): RCCL communicator + gather buffers
    void* comm = nullptr;             // ncclComm_t
    int comm_rank = 0, comm_size = 1;
    void* gather_buf = nullptr;       // [send chunk | ranks x chunk] packed site results
    size_t gather_bytes = 0;

    // grow-only buffers kept between calls (pm_hostio.cpp): pinned download slots, the FASTA
    // text and replay rows on the device
    void* stage = nullptr;
    hipEvent_t stage_ev[3] = {nullptr, nullptr, nullptr};
    void* text_buf = nullptr;
    size_t text_cap = 0;
    void* rows_buf = nullptr;
    size_t rows_cap = 0;
};

namespace pm {

int fail(pm_ctx* c, int code, const std::string& msg);
// Synchronise after a run; if a record shard overflowed, grow the buffer and run again (the
// per-site score only counts stored records).  pm_host.cpp.
int settle_run(pm_ctx* c);
int hip_fail(pm_ctx* c, hipError_t e, const char* what);

// Work queued on c->side between side_fork and side_join runs concurrently with the work
// queued on c->stream meanwhile (in a captured graph: parallel branches).
hipError_t side_fork(pm_ctx* c);
hipError_t side_join(pm_ctx* c);
void timer_begin(pm_ctx* c, int cls);
void timer_end(pm_ctx* c, int cls);

// kernel launchers (pm_fitch.hip / pm_sankoff.hip / pm_synth.hip)
hipError_t launch_fitch(pm_ctx* c, bool block);
hipError_t launch_sankoff(pm_ctx* c, bool block);
hipError_t launch_fitch_nt(pm_ctx* c, bool block);     // non-temporal set-record loads
hipError_t launch_sankoff_nt(pm_ctx* c, bool block);
// Records of the last run, sorted by (node, site) on the device, copied to host `out`.
// pm_warmup: one kernel of each code object looked up, so the object is loaded
hipError_t warm_fitch();
hipError_t warm_sankoff();
hipError_t warm_fitch_nt();
hipError_t warm_sankoff_nt();
hipError_t warm_replay();
hipError_t warm_synth();
hipError_t warm_sort();
hipError_t sort_records_to_host(pm_ctx* c, const std::vector<uint32_t>& counts, int64_t n, pm_mut* out);
// (Re)build the S2 / S3 leaf layout after the leaf columns or the tree changed (no-op when
// it is current or the tree has no S2 / S3 node).
int build_sub_planes(pm_ctx* c);
static_assert(sizeof(pm_mut) == 8, "pm_mut is {node, site_info}");
hipError_t launch_score(pm_ctx* c);
hipError_t launch_pack_codes(pm_ctx* c, const uint8_t* d_codes4, int64_t row_stride, const int32_t* d_row_of_leaf,
                             const uint8_t* d_present, int64_t present_stride);
hipError_t launch_pack_sites(pm_ctx* c, const uint8_t* d_codes4, uint4* dst);
hipError_t launch_synth(pm_ctx* c, int64_t site_begin, uint64_t seed);
hipError_t launch_unpack_leaf_codes(pm_ctx* c, int64_t s0, int64_t ns, uint8_t* d_out);
hipError_t launch_sub_planes(pm_ctx* c);
hipError_t launch_unpack_sites(pm_ctx* c, const uint4* src, int64_t s0, int64_t ns, uint8_t* d_out);
void free_replay(pm_ctx* c);
void comm_release(pm_ctx* c);   // pm_rccl.hip
int leaves_install(pm_ctx* c, int64_t S, const uint8_t* d_codes4, int64_t row_stride, const int32_t* node_row);

// host plumbing (pm_hostio.cpp)
// Phase log (pm_phase_report): drivers append (name, seconds) of their host / device phases.
void phase_add(const std::string& name, double seconds);
struct PhaseClock {
    std::chrono::steady_clock::time_point t;
    PhaseClock();
    double lap(const char* name);   // seconds since construction / the last lap, logged as `name`
};
int host_threads();   // host worker threads (PM_HOST_THREADS, else min(16, cores))
// hipMalloc that, on failure, releases the context's cached text / rows buffers and retries
hipError_t malloc_or_release(pm_ctx* c, void** p, size_t bytes);
void release_cached(pm_ctx* c);
void host_parallel_for(int tasks, const std::function<void(int)>& fn);
// malloc with transparent huge pages requested for large blocks (released with free / pm_free)
void* host_alloc_large(size_t n);
// dst (pageable host) <- src (device), n bytes, through pinned slots drained by host threads;
// synchronous on the ctx stream
hipError_t d2h_large(pm_ctx* c, void* dst, const void* src, size_t n);
// (device) src, n bytes, through the same slots, each landed chunk handed to `sink` in order
hipError_t d2h_stream(pm_ctx* c, const void* src, size_t n, const std::function<bool(const char*, size_t)>& sink,
                      bool& sink_ok);
bool write_all(int fd, const char* p, size_t n);   // write(2) until done; false on an error
// *buf grown (contents dropped) to hold `need` bytes
hipError_t grow_device(void** buf, size_t* cap, size_t need);
void free_hostio(pm_ctx* c);

// replay kernels (pm_replay.hip)
struct ReplayDev {
    int32_t leaves = 0;
    int64_t row_stride = 0;      // bytes per leaf row (multiple of 16)
    int64_t columns = 0;
    int32_t max_depth = 0;
    int32_t presence_words = 0;  // u32 words of block-presence bits per leaf
    char* rows = nullptr;        // [leaves][row_stride]
    const char* cons_row = nullptr;   // [row_stride]
    const int32_t* parent = nullptr;  // [N]
    const int32_t* leaf_node = nullptr;   // [leaves]
    const uint32_t* presence = nullptr;   // [leaves][presence_words]
    const int64_t* edit_off = nullptr;    // [N+1]
    const uint32_t* edit_col = nullptr;
    const uint8_t* edit_chr = nullptr;
    // blocks' column ranges [blk_lo, blk_hi) (id order = column order) and, per column tile,
    // the first block ending inside or after it: an absent block's columns are restored to
    // the consensus after the edits, so edits need no per-edit presence test
    int32_t blocks = 0;
    const int64_t* blk_lo = nullptr;
    const int64_t* blk_hi = nullptr;
    const int32_t* tile_blk = nullptr;   // [tiles + 1]
    // column tiles of kReplayTile bytes.  A node's edits are [plain | overriding] (an
    // overriding edit rewrites a column an ancestor edits), each part column-sorted; per
    // (node, tile) the first edit of each part in that tile
    int32_t tiles = 0;
    const int2* tile2 = nullptr;   // [N][tiles + 1] {plain, overriding}
    int32_t ring = 0;              // path nodes per leaf whose tile bounds a workgroup keeps in LDS
    int32_t tile_bytes = 0;        // column tile size of tile2 / tile_blk: kReplayTile or kDfsTile
    // k_replay_dfs: leaves in depth-first order (dfs_row = their rows), cut into groups
    // [g_leaf_off[g], g_leaf_off[g + 1]); a group's path nodes g_union[g_union_off[g] ..] in
    // order of first appearance; per leaf its path length and the prefix shared with the
    // previous leaf of its group (0 for a group's first)
    bool dfs = false;
    int32_t groups = 0;
    const int32_t* dfs_row = nullptr;
    const uint16_t* dfs_len = nullptr;
    const uint16_t* dfs_lpfx = nullptr;
    const int32_t* g_leaf_off = nullptr;
    const int32_t* g_union_off = nullptr;
    const int32_t* g_union = nullptr;
    const int64_t* path_off = nullptr;    // [leaves + 1] root-to-leaf node lists
    const int32_t* path = nullptr;
    // (leaf, tile) rows k_replay_dfs rebuilt from the consensus because an undo stack would
    // overflow, summed over the runs since replay_prepare (phase "replay.dfs_rebuilds")
    int32_t* dfs_rebuilds = nullptr;
};
#ifndef PM_REPLAY_TILE
#define PM_REPLAY_TILE 16384
#endif
constexpr int64_t kReplayTile = PM_REPLAY_TILE;   // leaf-row bytes assembled in LDS per workgroup
constexpr uint8_t kEditOverrides = 0x80;   // edit_chr flag: an ancestor edits the same column
constexpr int32_t kReplayRingMax = 512;     // ReplayDev::ring cap (deeper path nodes: bounds from HBM)
// k_replay_dfs: column tile per wave, leaves and path nodes per leaf group
#ifndef PM_DFS_TILE
#define PM_DFS_TILE 4096
#endif
constexpr int64_t kDfsTile = PM_DFS_TILE;
#ifndef PM_DFS_LEAVES
#define PM_DFS_LEAVES 16
#endif
constexpr int32_t kDfsLeaves = PM_DFS_LEAVES;
#ifndef PM_DFS_UNION
#define PM_DFS_UNION 128
#endif
constexpr int32_t kDfsUnionCap = PM_DFS_UNION;

// FASTA formatting on the device (printSequenceLinesNew, src/fasta.cpp:155-254): one
// segment per (leaf, print position) -- a block read forward or reverse-complemented from
// the leaf's row, or a run of dashes for an absent block (aligned output).
struct FmtSeg {
    int64_t src;     // first row column of the block, -1 for a dash run
    int64_t width;   // columns of the block, or the dash count
    int32_t rev;     // reverse strand: read backwards, complemented
    int32_t pad;
};
struct FmtArgs {
    const char* rows;
    int64_t row_stride;
    int32_t positions;        // print positions per leaf
    bool aligned;
    const FmtSeg* seg;        // [leaves][positions]
    int64_t* seg_len;         // [leaves][positions] chars each segment prints
    const int64_t* seg_off;   // [leaves][positions] offset in the leaf's line
    const int64_t* line_len;  // [leaves]
    const int64_t* start;     // [leaves] rotation of the line (circular offset)
    const int64_t* text_off;  // [leaves] byte offset of the leaf's record
    const int64_t* name_off;  // [leaves + 1] into names
    const char* names;
    char* text;
};
hipError_t launch_fmt_count(pm_ctx* c, const FmtArgs& f, int32_t leaves);
hipError_t launch_fmt_write(pm_ctx* c, const FmtArgs& f, int32_t leaves);
hipError_t launch_replay(pm_ctx* c, const ReplayDev& d);
// rows[leaf][c0 .. c0+n) chars -> packed codes out[leaf][(n+1)/2] ('-', 'x' -> 0)
hipError_t launch_rows_to_codes(pm_ctx* c, const char* rows, int64_t row_stride, int32_t leaves, int64_t c0,
                                int64_t n, uint8_t* out, int64_t out_stride);

}  // namespace pm
