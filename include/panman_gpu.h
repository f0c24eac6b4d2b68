/* panman_gpu.h -- C-ABI of the MI355X small-parsimony engine (libpanman_amd.so).
 *
 * Drop-in boundary for the reference's per-column parsimony path.  The reference
 * (faithokamoto/panman) has no FFI of its own: its kernels are C++ Tree members called
 * once per alignment column from the construction drivers.  Each entry point below names
 * the reference interface it replaces (paths relative to the reference root):
 *
 *   per-column Fitch      Tree::nucFitchForwardPass / BackwardPass / AssignMutations
 *                         src/panman.hpp:846-857, src/fitchSankoff.cpp:30-171
 *   per-column Sankoff    Tree::nucSankoff{Forward,Backward}Pass / AssignMutations
 *                         src/panman.hpp:860-875, src/fitchSankoff.cpp:359-703
 *   GPU batch entry       fitch_sankoff_on_gpu(Tree*, seqs, util*)   gpu/fitchSankoff.cuh:11
 *   column drivers        Tree(ifstream&, ifstream&, FILE_TYPE::MSA | MSA_OPTIMIZE, ref)
 *                         src/panman.cpp:1274-1649
 *
 * Conventions
 *   - Plain pointers and sizes only.  Host pointers unless a name says `_device`.
 *   - Every function returns PM_OK (0) or a negative PM_ERR_*; pm_last_error() gives the
 *     message.  Nothing here exits or aborts (the reference exit()s, src/panman.cpp:1297).
 *   - One pm_ctx per GPU; a ctx is not thread-safe, independent ctxs are.
 *   - Device work is queued on the ctx stream (pm_set_stream); functions that return
 *     host data synchronise that stream.
 *   - Codes are the reference's 4-bit NucCode (src/panman.hpp:27-44): A=1 C=2 G=4 T=8
 *     R=5 Y=10 S=6 W=9 K=12 M=3 B=14 D=13 H=11 V=7 N=15, gap/other=0.
 *     Packed code arrays hold two codes per byte, even site in the low nibble.
 */
#ifndef PANMAN_GPU_H
#define PANMAN_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_OK 0
#define PM_ERR_ARG (-1)
#define PM_ERR_OOM (-2)
#define PM_ERR_HIP (-3)
#define PM_ERR_UNSUPPORTED (-4)
#define PM_ERR_STATE (-5)

#define PM_MODE_FITCH 0   /* F1-F3: 16-bit one-hot state sets, M1 semantics            */
#define PM_MODE_SANKOFF 1 /* S1-S3: unit-cost Sankoff over 16 codes, M2 semantics      */
/* Block-level parsimony (columns = blocks; codes 0 block absent, 1 forward, 2 reverse):
 * B1 Tree::blockFitch*New   src/fitchSankoff.cpp:224-308 (leaf not in the column: state 0)
 * B2 Tree::blockSankoff*    src/fitchSankoff.cpp:707-818 (leaf not in the column: absent
 *    block, cost {0, INF, INF}).  Root parent state = consensus code (0 in the PanGraph
 *    driver, src/panman.cpp:906-909, :952-956); `forced` = defaultState of the backward
 *    pass.  Records: PM_MUT_NI -> BlockMut(BI, inversion = code == 2), PM_MUT_ND ->
 *    BlockMut(BD, false), PM_MUT_NS -> BlockMut(BD, inversion = true). */
#define PM_MODE_BLOCK_FITCH 2
#define PM_MODE_BLOCK_SANKOFF 3

#define PM_MUT_NS 0 /* NucMutationType::NS  src/panman.hpp:48 */
#define PM_MUT_ND 1 /* NucMutationType::ND  src/panman.hpp:50 */
#define PM_MUT_NI 2 /* NucMutationType::NI  src/panman.hpp:52 */

typedef struct pm_ctx pm_ctx;

/* Tree topology as CSR.  Replaces the Node* graph built by
 * Tree::createTreeFromNewickString (src/panman.cpp:310-450) and the flattening in
 * gpu/fitchSankoff.cu:40-83.  Children keep their Newick order.  A node with no
 * children is a leaf.  Node ids are the caller's; mutation records use them. */
typedef struct pm_tree {
    int32_t num_nodes;
    int32_t root;
    const int32_t* child_offsets; /* [num_nodes + 1] */
    const int32_t* child_index;   /* [child_offsets[num_nodes]] */
} pm_tree;

/* One mutation record: the (node, column, type, char) tuple the reference pushes into
 * nonGapMutationsMSA (src/panman.cpp:1426-1430, 1607-1610). */
typedef struct pm_mut {
    uint32_t node;      /* caller node id                                    */
    uint32_t site_info; /* (site << 8) | (type << 4) | code; type = PM_MUT_* */
} pm_mut;

/* Context / device (replaces the device setup of gpu/fitchSankoff.cu:370-440). */
int pm_create(int device, pm_ctx** out);
void pm_destroy(pm_ctx* ctx);
/* Initialise the HIP runtime on `device` and load the library's code objects (what the
 * first pm_create and first launches would otherwise pay), from any thread: a caller with
 * host work to do first (reading and decoding input) can overlap it.  Optional. */
int pm_warmup(int device);
const char* pm_last_error(const pm_ctx* ctx);
/* Queue all work on `hip_stream` (a hipStream_t; NULL = the ctx's own stream). */
int pm_set_stream(pm_ctx* ctx, void* hip_stream);
/* Options (results are identical either way):
 *   PM_OPT_VIRTUAL (default 1): the level kernels evaluate internal nodes whose children
 *                  are one or two leaves inline in their parent instead of materialising them.
 *   PM_OPT_GRAPH   (default 0): pm_run captures its launch sequence (per-level kernels,
 *                  memsets) into a hipGraph once and replays it while the tree, columns,
 *                  mode and buffers stay the same; kernel_times then reports the whole run
 *                  as class 4.
 *   PM_OPT_SUBTREE (default 1): Fitch with every leaf present also evaluates, inside its
 *                  binary parent, any node whose children are leaves or two-leaf cherries
 *                  (three- and four-leaf subtrees), so those are not materialised either.
 *   PM_OPT_NARROW  (default 16): Fitch -- a run of consecutive levels with at most this many
 *                  nodes each (a node of out-degree > 3 counts 4) is walked by one launch,
 *                  one 1024-thread workgroup per 2048-site tile with a barrier between levels,
 *                  instead of one launch per level (deep, ladder-like trees); 0 = off.
 *   PM_OPT_GROUP_WAVES (default 32768): Fitch -- up to PM_OPT_GROUP_LEVELS consecutive
 *                  pre-order levels of at most this many (node, tile) waves together go to one
 *                  launch, the lower levels' waves recomputing their ancestors' finals; 0 = off.
 *   PM_OPT_GROUP_LEVELS (default 4): 2 to 4 levels per such launch.
 *   PM_OPT_UP_GROUP (default 1): Fitch, subtree form -- a node of out-degree <= 3 whose
 *                  latest children have out-degree <= 3 runs in their post-order launch,
 *                  recomputing them, instead of one launch per height; 0 = by height.
 *   PM_OPT_SUB_DOWN (default 0): Fitch, subtree form -- a three- or four-leaf subtree's
 *                  finals and records come from its parent's pre-order wave instead of a
 *                  wave of their own after the levels.
 *   PM_OPT_PLAIN_UP (default 1): Fitch / Sankoff, grouped subtree form -- a post-order launch's binary
 *                  nodes with no three- / four-leaf subtree child and nothing recomputed run in
 *                  a lean kernel (fewer registers, more waves in flight) before the rest, when
 *                  they are at least 65536 (node, tile) waves; a value >= 2 sets that threshold;
 *                  0 = off.
 *   PM_OPT_RECORD_CAP: the record buffer's capacity per shard (1024 shards), replacing the
 *                  first guess (about 1.5 % of node*site pairs); a run that overflows it is
 *                  re-run with a larger buffer when its results are read (pm_mutation_count,
 *                  pm_site_results*, pm_run_gather), so results never depend on it.
 *   PM_OPT_NT_LOADS (default -1): set records read with non-temporal loads (1), ordinary
 *                  loads (0), or by the tree's widest level (-1: non-temporal from 64k
 *                  (node, tile) waves up, where the records have left the caches by the time
 *                  they are read).
 *   PM_OPT_CLUSTER (default 1): subtree form -- the Fitch post-order runs as LDS-staged
 *                  sweeps from the first height above which the tree's bands are chain-like and
 *                  hold at most 16384 clusters (deep ladder trees: every height; a random-join
 *                  tree: none): bands of heights, one wave per (connected cluster of the band,
 *                  2048-site tile) walking the cluster's nodes depth first with its inner sets
 *                  in LDS.  When every height is swept, the pre-order (Fitch and Sankoff) and
 *                  the Sankoff post-order (nodes of <= 255 children) run over the same clusters.
 *                  0 = the level kernels everywhere.  A value >= 2 instead takes every height
 *                  from the first whose level (and every level above it) holds at most that
 *                  many nodes.  Takes effect at the next pm_tree_upload; results identical.
 * (Option ids 1, 4, 5 and 11 -- subtree-region, heavy-path-chain and level-band schedules,
 * tail records overlapped with the pre-order levels -- were measured slower than, or no
 * faster than, the level kernels on MI355X and removed.) */
#define PM_OPT_VIRTUAL 2
#define PM_OPT_GRAPH 3
#define PM_OPT_SUBTREE 6
#define PM_OPT_NARROW 7
#define PM_OPT_GROUP_WAVES 8
#define PM_OPT_GROUP_LEVELS 9
#define PM_OPT_UP_GROUP 10
#define PM_OPT_RECORD_CAP 12
#define PM_OPT_SUB_DOWN 13
#define PM_OPT_PLAIN_UP 14
#define PM_OPT_NT_LOADS 16
#define PM_OPT_CLUSTER 17
int pm_set_option(pm_ctx* ctx, int option, int64_t value);
/* Accumulate per-kernel-class device time with HIP events (see pm_kernel_times). */
int pm_set_profiling(pm_ctx* ctx, int enable);

/* Upload the topology (host arrays).  Levels, dense indices and the device copy are built
 * here, once; replaces the recursion over Node* children in every per-column call. */
int pm_tree_upload(pm_ctx* ctx, const pm_tree* tree);

/* Upload the leaf columns.  Replaces the per-column `states` maps of the drivers
 * (src/panman.cpp:1409-1417 Fitch, :1574-1582 Sankoff).
 *   codes4[row * row_stride + s/2]: 4-bit code of site s for alignment row `row`.
 *   node_row[node]: the row of leaf `node`, or -1 if the leaf is absent from the
 *     alignment (reference: state 0 / all-INF, src/fitchSankoff.cpp:33-36, :362-368).
 *   present (nullable): per-row bitmask of present sites (bit s%8 of byte
 *     row * present_stride + s/8); a cleared bit makes that (leaf, site) absent, as the
 *     PanGraph driver does for leaves lacking a block (src/panman.cpp:1026-1028). */
int pm_leaves_upload(pm_ctx* ctx, int64_t num_sites, const uint8_t* codes4, int64_t row_stride,
                     const int32_t* node_row, const uint8_t* present, int64_t present_stride);

/* Per-site constants (packed codes, ceil(S/2) bytes each).
 *   consensus: the root's parent state, i.e. the block consensus character
 *     (src/panman.cpp:1424-1425, :1600-1606).
 *   forced (nullable): Fitch: refState forcing the root forward set (:1419);
 *     Sankoff: defaultState forcing the root (:1583-1596). */
int pm_sites_upload(pm_ctx* ctx, const uint8_t* consensus4, const uint8_t* forced4);

/* Run post-order, pre-order and mutation assignment for every uploaded site (async). */
int pm_run(pm_ctx* ctx, int mode);

/* Results (synchronise the stream). */
int pm_mutation_count(pm_ctx* ctx, int64_t* count);
/* Records sorted by (node, site); `cap` records fit in `out`. */
int pm_mutations_fetch(pm_ctx* ctx, pm_mut* out, int64_t cap, int64_t* count);
/* Per site: number of mutated edges below the root (parsimony score of the assignment)
 * and the root's final code (255 = unresolved).  Either pointer may be NULL. */
int pm_site_results(pm_ctx* ctx, int32_t* score, uint8_t* root_code);
/* Same, copied device-to-device into caller buffers on the ctx stream (async after the
 * record-buffer check, which synchronises), so that a collective can gather them without a
 * host copy. */
int pm_site_results_device(pm_ctx* ctx, void* score_device, void* root_code_device);
/* Accumulated device milliseconds and launch counts per kernel class since the last
 * call; classes: 0 post-order, 1 pre-order + assignment (levels, bands, sweeps), 2 score
 * histogram, 3 replay, 4 whole pm_run replayed from a hipGraph (PM_OPT_GRAPH), 5 the
 * pre-order's tail launch (children beyond the second, S2 / S3 subtrees). */
int pm_kernel_times(pm_ctx* ctx, double* ms, int64_t* launches, int classes);

/* ---- multi-GPU column shards ----------------------------------------- */
/* The reference runs one parsimony call per column (src/panman.cpp:1381 Fitch, :1568
 * Sankoff) -- columns are independent, so each GPU owns a contiguous site range with the
 * tree replicated.  The per-site results (parsimony score, root code) are reassembled with
 * ONE RCCL all-gather over xGMI; mutation records stay on their rank (site indices local
 * to the shard) and merge on the host by (node, site_begin + site).  RCCL is opened at run
 * time (librccl.so.1; inside a PyTorch process, torch's own copy).
 *   pm_comm_unique_id   rank 0 makes the id (ncclGetUniqueId); the caller broadcasts it.
 *   pm_comm_init_rank   one process per GPU: bind ctx to rank `rank` of `nranks`.
 *   pm_comm_init_all    one process, several GPUs: ncclCommInitAll over the ctxs' devices
 *                       (distinct devices; rank i = ctxs[i]).
 *   pm_run_gather       pm_run on this rank's shard [site_begin, site_begin + uploaded
 *                       sites) of `total_sites`, then the all-gather: score_device
 *                       [total_sites] int32 and root_device [total_sites] u8 (device
 *                       memory) receive every rank's sites.  Every rank must call it; it
 *                       returns when the gathered vectors are complete.  A rank whose shard
 *                       fails (bad range, run error) still joins the collective with a
 *                       failed chunk head, so every rank returns an error instead of one
 *                       rank leaving the others blocked.  Shards hold at most
 *                       ceil(total/ranks)+2 sites.
 *   pm_multi_run        the same for pm_comm_init_all contexts from one thread (RCCL group
 *                       call); site_begin[i] per ctx; results to host (nullable).
 *   pm_shard_range      the balanced rule [r*S/n, (r+1)*S/n) bench.py and shard.py use.
 * The gathered unit is one chunk per rank of `per` = ceil(S/ranks)+3 u64 entries: entry 0 =
 * site_begin << 32 | count (count 0xffffffff: that rank failed), then one entry per site =
 * score (int32) | root code << 32.  The same layout moves through any other collective:
 *   pm_pack_site_results    the ctx's last run into a chunk in device memory; syncs;
 *   pm_unpack_site_results  ranks x per gathered entries (device) into score / root device
 *                           vectors; checks the heads (failed rank, overlaps, gaps); syncs.
 *   pm_chunk_entries / pm_chunk_pack / pm_chunk_unpack  the same on host memory, no GPU. */
#define PM_COMM_ID_BYTES 128
int pm_comm_unique_id(uint8_t* id, int64_t len);
int pm_comm_init_rank(pm_ctx* ctx, const uint8_t* id, int nranks, int rank);
int pm_comm_init_all(pm_ctx* const* ctxs, int n);
int pm_run_gather(pm_ctx* ctx, int mode, int64_t total_sites, int64_t site_begin, void* score_device,
                  void* root_device);
int pm_multi_run(pm_ctx* const* ctxs, int n, int mode, const int64_t* site_begin, int64_t total_sites,
                 int32_t* score, uint8_t* root_code);
int pm_shard_range(int rank, int ranks, int64_t total_sites, int64_t* begin, int64_t* end);
int pm_pack_site_results(pm_ctx* ctx, int64_t site_begin, int64_t per, void* chunk_device);
int pm_unpack_site_results(pm_ctx* ctx, const void* all_device, int64_t per, int ranks, int64_t total_sites,
                           void* score_device, void* root_device);
int pm_chunk_entries(int64_t total_sites, int ranks, int64_t* per);
int pm_chunk_pack(int64_t site_begin, int64_t count, const int32_t* score, const uint8_t* root, int64_t per,
                  uint64_t* chunk);
int pm_chunk_unpack(const uint64_t* all, int64_t per, int ranks, int64_t total_sites, int32_t* score,
                    uint8_t* root);

/* ---- measurement (bench.py roofline; not part of the reference interface) ------------ */
/* Bytes this design must move in the last pm_run (nucleotide modes), counted from the run's
 * record masks at the kernels' 16-B-per-lane granularity: out[0] post-order (leaf words,
 * child records read, own record + masks written), out[1] pre-order + assignment (own
 * record, parent final, dirty-lane leaf words, compact finals, 8 B per mutation record),
 * out[2] score histogram, out[3] floor = 0.5 B per leaf-site + 8 B per record, out[4] the
 * record count; with n >= 14, out[5..13] split them: post-order leaf words, child records read,
 * own records + pushed masks written; pre-order own records, parent finals, dirty-lane leaf
 * words of the nodes' first two children (k_down), finals written, tail items and their
 * dirty-lane leaf words (k_tail).  With the LDS-staged sweeps (PM_OPT_CLUSTER) a child record
 * read from an LDS slot, and a parent final likewise, is not counted.  With n >= 20, out[14..19]:
 * the pre-order's reads at 128-B line granularity (every line a load touches, as the memory
 * fetches them: tools/calib_fetch.hip) -- level kernels: descriptors + masks + own records,
 * parent finals, dirty-lane leaf words; tail: descriptors + masks, dirty-lane leaf words,
 * parent finals.  `n` >= 5.
 * Synchronises the ctx stream. */
int pm_design_bytes(pm_ctx* ctx, double* out, int n);
/* FETCH_SIZE calibration for scattered reads: `lanes` threads each read 4 x 16 B, one 16-B
 * slot every `stride_bytes` (16 = a coalesced stream), and write 16 B coalesced; `reps`
 * launches, *ms_per_launch their average (profile it with rocprofv3 --pmc FETCH_SIZE). */
int pm_gather_probe(int device, int64_t lanes, int stride_bytes, int reps, double* ms_per_launch);
/* Device bytes the context holds now (n entries of): out[0] total, [1] leaf rows (code planes,
 * presence, flags), [2] the S2 / S3 side-by-side leaf copy, [3] state-set records, [4] record
 * masks, [5] Sankoff part counters, [6] mutation-record shards, [7] the flattened tree
 * (descriptors, level tables), [8] per-site columns (consensus, forced, finals of the root,
 * score, root code), [9] replay rows, FASTA text, gather and generator buffers.  No GPU call. */
int pm_memory_footprint(pm_ctx* ctx, int64_t* out, int n);
/* Hash of the library's sources (16 hex digits): profiled PMC traffic is tied to it. */
const char* pm_build_id(void);
/* Achievable HBM rate on `device`: a 16-B-per-lane streaming copy of `bytes` bytes, `reps`
 * times; *gbs = (read + write bytes) / s / 1e9. */
int pm_stream_copy_rate(int device, int64_t bytes, int reps, double* gbs);
/* The same for writes only (the replay rows' access pattern): 16 B per lane, 4 non-temporal
 * stores in flight; *gbs = written bytes / s / 1e9. */
int pm_stream_write_rate(int device, int64_t bytes, int reps, double* gbs);

/* Phase log: the drivers (pm_fasta, pm_msa_build / pm_msa_to_panman*, pm_panman_load /
 * pm_panman_write, pm_create) append the wall time of each host / device phase of every
 * call to one process-wide log.  pm_phase_report writes it as "name\tseconds\n" lines into
 * buf (truncated to len - 1 bytes, NUL-terminated) and returns the bytes the whole report
 * needs (with the NUL); pm_phase_reset empties it (it also stops growing at 4096 entries). */
void pm_phase_reset(void);
int64_t pm_phase_report(char* buf, int64_t len);

/* ---- column drivers ------------------------------------------------------------------ */
/* Drop-in for Tree(msa, newick, FILE_TYPE::MSA (mode PM_MODE_FITCH, "M1") or
 * FILE_TYPE::MSA_OPTIMIZE (PM_MODE_SANKOFF, "M2"), reference) -- src/panman.cpp:1274-1649:
 * Newick + aligned FASTA text -> consensus block, root block insertion and every node's
 * NucMut list (grouped as src/panman.cpp:1445-1466), computed on `device`.  Returns a
 * malloc'd text dump (release with pm_free):
 *   "#consensus\t<seq>\n" "#blockmut\t<root>\t0\t-1\t1\t0\n" then one line per NucMut,
 *   nodes in name order: "<node>\t<nucPosition>\t<nucGapPosition>\t<mutInfo>\t<nucs %06x>\n";
 * or "#error\t<message>\n" where the reference would exit or has undefined behaviour. */
char* pm_msa_build(const char* newick, const char* msa_text, const char* reference, int mode, int device);
void pm_free(void* p);
/* The same construction written as a PanMAN file (Tree(...) + writePanMAN,
 * src/panmanUtils.cpp:1409-1465, :271-299): one tree, one block. */
int pm_msa_to_panman(const char* newick, const char* msa_text, const char* reference, int mode, int device,
                     const char* out_path, char* err, int64_t err_len);
/* The same with the columns split into contiguous ranges over `devices` (one host thread
 * and context each; entries may repeat); records are merged by (node, site) on the host,
 * so the file is byte-identical to the single-device build. */
int pm_msa_to_panman_multi(const char* newick, const char* msa_text, const char* reference, int mode,
                           const int* devices, int num_devices, const char* out_path, char* err, int64_t err_len);

/* ---- root-to-leaf mutation replay (FASTA extraction) ---------------------------------- */
/* PanMAT fields used by printFASTAUltraFast (src/panman.hpp:520-543 Block / GapList,
 * :429-517 BlockMut, :75-313 NucMut, Tree::circularSequences / rotationIndexes /
 * sequenceInverted).  Per-node lists are CSR in list order; arrays are host memory. */
typedef struct pm_panmat {
    int32_t num_nodes;
    int32_t root;
    const int32_t* child_offsets;    /* [num_nodes + 1] */
    const int32_t* child_index;
    const char* names;               /* num_nodes NUL-terminated identifiers, back to back */
    int32_t num_blocks;
    const int32_t* block_primary;    /* [num_blocks] primaryBlockId */
    const int64_t* block_seq_offsets;/* [num_blocks + 1] into block_seq */
    const uint32_t* block_seq;       /* consensusSeq: 8 codes per word, MSB first, code 0 ends */
    int32_t num_gaps;
    const int32_t* gap_primary;      /* [num_gaps] */
    const int64_t* gap_offsets;      /* [num_gaps + 1] into gap_position / gap_length */
    const uint32_t* gap_position;
    const uint32_t* gap_length;
    const int64_t* block_mut_offsets;/* [num_nodes + 1] */
    const int32_t* block_mut_primary;
    const uint8_t* block_mut_info;   /* 1 = insertion (BI), 0 = deletion / inversion */
    const uint8_t* block_mut_inversion;
    const int64_t* nuc_mut_offsets;  /* [num_nodes + 1] */
    const int32_t* nuc_mut_primary;
    const int32_t* nuc_mut_secondary;
    const int32_t* nuc_mut_position;
    const int32_t* nuc_mut_gap_position; /* -1 = main position */
    const uint8_t* nuc_mut_info;     /* (length << 4) | type */
    const uint32_t* nuc_mut_nucs;    /* code i at bits 4 * (5 - i) */
    const int32_t* circular_offset;  /* nullable [num_nodes]; < 0 = not circular */
    const int32_t* rotation_index;   /* nullable [num_nodes] */
    const uint8_t* sequence_inverted;/* nullable [num_nodes] */
    const float* branch_length;      /* nullable [num_nodes]; Newick branch lengths (root 0) */
} pm_panmat;

/* Drop-in for Tree::printFASTAUltraFast(fout, aligned) (src/fasta.cpp:1981-2099): one
 * record per leaf, ">name\n" + 70-column lines + "\n", leaves in node-id order (the
 * reference's order is TBB-scheduled).  `*text` is malloc'd (release with pm_free).
 * Replay runs on the GPU (consensus expansion + path mutations per leaf); block order,
 * strands, rotation, circular offset and line wrapping are applied by the host formatter.
 * A nucleotide mutation's secondary block id is ignored (applied to its primary block), as
 * printFASTAUltraFastHelper does (src/fasta.cpp:1838-1842).
 * Memory: the replayed rows (leaves x columns bytes) and the text stay on the device in
 * grow-only per-context buffers until pm_destroy, so the next pm_fasta on the context does not
 * allocate again; a later large allocation on the context that fails releases them and
 * retries once. */
int pm_fasta(pm_ctx* ctx, const pm_panmat* panmat, int aligned, char** text, int64_t* length);
/* pm_fasta over several devices: leaves split into contiguous ranges, one host thread and
 * context per entry of `devices` (entries may repeat), texts concatenated in leaf order --
 * byte-identical to pm_fasta.  On failure `err` receives the first shard's reason. */
int pm_fasta_multi(const pm_panmat* panmat, int aligned, const int* devices, int num_devices, char** text,
                   int64_t* length, char* err, int64_t err_len);
/* The same in stages: prepare (host flattening + upload), run (GPU replay, async on the
 * ctx stream; profiling class 3), format (download + text). */
int pm_replay_prepare(pm_ctx* ctx, const pm_panmat* panmat);
/* Prepare only leaves [leaf_begin, leaf_end) of the PanMAT (leaves in node-id order): one
 * GPU's shard when FASTA extraction is split by leaves. */
int pm_replay_prepare_range(pm_ctx* ctx, const pm_panmat* panmat, int64_t leaf_begin, int64_t leaf_end);
int pm_replay_run(pm_ctx* ctx);
int pm_replay_format(pm_ctx* ctx, int aligned, char** text, int64_t* length);
/* The same FASTA text written to the file descriptor `fd` (a pipe, stdout, a file) instead of
 * returned: the device text streams through pinned slots to `fd` while later chunks are still
 * in flight, with no host copy of the whole text.  `length` (nullable): the bytes written.
 * pm_fasta_fd = pm_fasta to a descriptor; pm_fasta_multi_fd = pm_fasta_multi to a descriptor
 * (the shards' texts in leaf order).  A failed write returns PM_ERR_ARG (errno kept). */
int pm_replay_format_fd(pm_ctx* ctx, int aligned, int fd, int64_t* length);
int pm_fasta_fd(pm_ctx* ctx, const pm_panmat* panmat, int aligned, int fd, int64_t* length);
int pm_fasta_multi_fd(const pm_panmat* panmat, int aligned, const int* devices, int num_devices, int fd, int64_t* length,
                      char* err, int64_t err_len);
/* Canonical aligned columns per leaf of the prepared PanMAT (gap slots before each main
 * position, block sentinels included) and the number of leaves. */
int pm_replay_shape(pm_ctx* ctx, int64_t* leaves, int64_t* columns, int64_t* edits);

/* ---- PanMAN files (xz + Cap'n Proto, schema panman.capnp) ----------------------------- */
typedef struct pm_panman pm_panman;
/* Load a .panman: TreeGroup(istream) + Tree::protoMATToTree (src/panman.cpp:6847-6877,
 * :1661-1751, mutations assigned in pre-order :576-618).  Host only, no device needed.
 * On failure `err` (nullable, err_len bytes) receives the reason. */
int pm_panman_load(const char* path, pm_panman** out, char* err, int64_t err_len);
/* The older Google Protobuf PanMAN (`panmanOld.treeGroup`, panman.proto; xz-compressed or
 * raw), as TreeGroup(istream, isOld = true) reads it (src/panman.cpp:6865-6876 with
 * Tree::protoMATToTree(panmanOld::tree), :1803-1866) -- into the same handle as
 * pm_panman_load, so pm_panman_write converts it (the reference's --protobuf2capnp,
 * src/panmanUtils.cpp:939-952). */
int pm_panman_load_old(const char* path, pm_panman** out, char* err, int64_t err_len);
int pm_panman_tree_count(const pm_panman* file);
/* View of tree `index` as a pm_panmat (pointers into `file`, valid until pm_panman_free);
 * node ids are pre-order positions of the stored Newick, names follow the reference's
 * Newick naming. */
int pm_panman_tree(const pm_panman* file, int index, pm_panmat* view);
const char* pm_panman_newick(const pm_panman* file, int index);
void pm_panman_free(pm_panman* file);
/* Write trees as TreeGroup::writeToFile + writePanMAN do (src/panman.cpp:6885-7015,
 * src/panmanUtils.cpp:271-299): capnp message, xz level 9 when `compress`. */
int pm_panman_write(const char* path, const pm_panmat* const* trees, int count, int compress);

/* Drop-in for Tree::reroot(leaf) (src/reroot.cpp:4-262; CLI --reroot,
 * src/panmanUtils.cpp:855-892): every leaf's sequence is replayed on the GPU
 * (getSequenceFromReference, src/panman.cpp:4676-5000), the root moves next to `leaf`
 * (transform, :5831-5906) and every block and nucleotide mutation is re-derived by Fitch
 * with the root forced to the leaf's states.  The result is a new one-tree pm_panman (in
 * the pre-order of the new topology; release with pm_panman_free).  Replaces the ctx's
 * tree, columns and replay state.  Within a node, block mutations are ordered by block
 * id (the reference's order is TBB-scheduled).  A PanMAT with secondary blocks (a nucleotide
 * mutation with secondaryBlockId != -1) returns PM_ERR_UNSUPPORTED ("secondary blocks"):
 * the reference rebuilds the secondary blocks' own sequences and block states
 * (src/reroot.cpp:55-89, src/panman.cpp:4722-4890), a second block level this layout does
 * not hold -- although pm_fasta, like printFASTAUltraFastHelper, replays such a PanMAT (the
 * mutation lands on the primary block). */
int pm_reroot(pm_ctx* ctx, const pm_panmat* tree, const char* leaf, pm_panman** out);

/* Drop-in for Tree(pangraph.json, newick, FILE_TYPE::PANGRAPH, reference) (src/panman.cpp:
 * 820-1273; CLI -P/-N, src/panmanUtils.cpp:1364-1407): the PanGraph model
 * (src/panman.cpp:6200-6476), block order by chained alignment of the paths
 * (src/chaining.cpp) and rotation of circular paths (src/rotation.cpp) on the host; block
 * and nucleotide parsimony for every column on the GPU (Fitch, or Sankoff when the tree
 * has a polytomy).  `json` and `newick` are file contents; `reference` may be NULL / "".
 * Without a reference the main-column root forcing follows oneTBB's iteration order of
 * the per-block sequences.  Result: a one-tree pm_panman. */
int pm_pangraph_build(pm_ctx* ctx, const char* json, const char* newick, const char* reference, pm_panman** out);

/* ---- summary ------------------------------------------------------------------------- */
/* Drop-in for Tree::printSummary (src/summary.cpp:257-273; CLI --summary, src/panmanUtils.cpp:
 * 356-384): mutation counts reduced on the GPU from the PanMAT's flat mutation arrays
 * (getTotalParsimonyParallel, :3-59; getBlockMutationsParallelHelper, :61-109), leaf depths
 * as the Newick parser computes them (float sum in leaf order, src/panman.cpp:386-394),
 * block duplications / translocations by the reference's presence walk (:111-193). */
typedef struct pm_summary {
    int64_t nodes, samples;                                 /* Total Nodes / Samples in Tree */
    int64_t substitutions, insertions, deletions, inversions;
    int64_t max_depth;
    float mean_depth;
    int64_t block_insertions, block_deletions, block_inversions;
    int64_t block_duplications, block_translocations;
} pm_summary;
int pm_summary_compute(pm_ctx* ctx, const pm_panmat* tree, pm_summary* out);

/* ---- synthetic inputs (bench / tests; seeded, counter-based) ------------------------ */
/* Random-join binary tree on `leaves` leaves (SURVEY.md §8d family T1): writes
 * 2*leaves-1 nodes as CSR; leaves are ids [0, leaves), internal nodes follow. */
int pm_synth_tree_random_join(int64_t leaves, uint64_t seed, int32_t* child_offsets,
                              int32_t* child_index, int32_t* root);
/* "SARS-like" tree (SURVEY.md §8d family T2): ladderised sequential insertion (leaf i
 * splits the pendant edge of leaf i-1 with p = 0.9, else of a uniform earlier leaf), then
 * 10 % of the internal nodes contracted into polytomies of 3-64 children.  Buffers must
 * hold 2*leaves-1 nodes (child_offsets 2*leaves entries, child_index 2*leaves-2); the
 * node count written is returned in *num_nodes; leaves are ids [0, leaves). */
int pm_synth_tree_sars_like(int64_t leaves, uint64_t seed, int32_t* child_offsets, int32_t* child_index,
                            int32_t* root, int64_t* num_nodes);
/* Evolve columns [site_begin, site_begin + num_sites) of a seeded alignment down the
 * uploaded tree on the device and install them as the leaf columns plus the consensus
 * (the root sequence).  Identical global sites give identical columns on every rank. */
int pm_synth_columns(pm_ctx* ctx, int64_t site_begin, int64_t num_sites, uint64_t seed);
/* Copy leaf codes of sites [s0, s0+ns) to host, one byte per site:
 * out[leaf * ns + (s - s0)] for every leaf in increasing node-id order (absent = 0). */
int pm_leaf_codes_fetch(pm_ctx* ctx, int64_t s0, int64_t ns, uint8_t* out);
int pm_consensus_fetch(pm_ctx* ctx, int64_t s0, int64_t ns, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif /* PANMAN_GPU_H */
