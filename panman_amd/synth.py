"""Seeded synthetic PanMATs for the replay bench (SURVEY.md §8d config C5, E. coli-like):
a random-join tree, blocks of random ACGT with gap slots, block insertions / deletions /
inversions at 1e-2 per block-edge, and nucleotide mutations (SNPs, MNPs, deletions,
insertions into gap slots) at `mu` per site-edge.  Vectorised numpy; identical for a seed."""
from __future__ import annotations

import numpy as np

from .engine import random_join_tree
from .panmat import PanMAT


def _pack_words(codes: np.ndarray) -> np.ndarray:
    n = codes.shape[0]
    pad = (-n) % 8
    c = np.concatenate([codes.astype(np.uint32), np.zeros(pad, np.uint32)]).reshape(-1, 8)
    shifts = (4 * (7 - np.arange(8))).astype(np.uint32)
    return np.bitwise_xor.reduce(c << shifts, axis=1).astype(np.uint32)


def c5_panmat(leaves: int = 1000, blocks: int = 500, mean_len: int = 10_000, mu: float = 1e-3,
              block_rate: float = 1e-2, gaps_per_block: int = 20, seed: int = 3, tree=None) -> PanMAT:
    """`tree` = (child_offsets, child_index, root) replaces the random-join tree (e.g. a deep
    sars_like_tree or a caterpillar); `leaves` is then ignored."""
    rng = np.random.default_rng(seed)
    if tree is None:
        off, idx, root = random_join_tree(leaves, seed=1)
    else:
        off, idx, root = (np.asarray(tree[0], np.int32), np.asarray(tree[1], np.int32), int(tree[2]))
    n = off.shape[0] - 1
    names = [f"s{i}" if off[i] == off[i + 1] else f"node_{i}" for i in range(n)]
    pm = PanMAT(names, off, idx, root)
    lens = rng.integers(mean_len // 2, mean_len * 3 // 2 + 1, size=blocks)
    seq_off = np.zeros(blocks + 1, np.int64)
    words = []
    for b in range(blocks):
        w = _pack_words(rng.choice(np.array([1, 2, 4, 8], np.uint8), size=int(lens[b])))
        words.append(w)
        seq_off[b + 1] = seq_off[b] + w.size
    # gap slots
    g_off = np.zeros(blocks + 1, np.int64)
    g_pos, g_len = [], []
    for b in range(blocks):
        pos = np.unique(rng.integers(0, lens[b] + 1, size=gaps_per_block))
        g_pos.append(pos)
        g_len.append(rng.integers(1, 11, size=pos.size))
        g_off[b + 1] = g_off[b] + pos.size
    g_pos_all = np.concatenate(g_pos).astype(np.uint32)
    g_len_all = np.concatenate(g_len).astype(np.uint32)
    g_blk_all = np.repeat(np.arange(blocks), np.diff(g_off))
    # block mutations: root inserts every block; 1e-2 per block-edge elsewhere
    bm_node = [np.full(blocks, root)]
    bm_blk = [np.arange(blocks)]
    bm_info = [np.ones(blocks, np.uint8)]
    bm_inv = [np.zeros(blocks, np.uint8)]
    hits = rng.random((n, blocks)) < block_rate
    hits[root] = False
    hn, hb = np.nonzero(hits)
    kind = rng.choice(3, size=hn.size, p=[0.5, 0.25, 0.25])   # BD, inversion, BI
    bm_node.append(hn)
    bm_blk.append(hb)
    bm_info.append((kind == 2).astype(np.uint8))
    bm_inv.append((kind == 1).astype(np.uint8))
    bm_node = np.concatenate(bm_node)
    order = np.argsort(bm_node, kind="stable")
    bm_node = bm_node[order]
    bm_blk = np.concatenate(bm_blk)[order]
    bm_info = np.concatenate(bm_info)[order]
    bm_inv = np.concatenate(bm_inv)[order]
    bm_off = np.zeros(n + 1, np.int64)
    np.add.at(bm_off, bm_node + 1, 1)
    bm_off = np.cumsum(bm_off)
    # nucleotide mutations per non-root node
    total = int(lens.sum())
    counts = rng.poisson(mu * total, size=n)
    counts[root] = 0
    m = int(counts.sum())
    node = np.repeat(np.arange(n), counts)
    in_gap = rng.random(m) < 0.1
    blk = rng.integers(0, blocks, size=m)
    pos = (rng.random(m) * lens[blk]).astype(np.int64)
    gap = np.full(m, -1, np.int64)
    gsel = rng.integers(0, g_pos_all.size, size=m)
    blk = np.where(in_gap, g_blk_all[gsel], blk)
    pos = np.where(in_gap, g_pos_all[gsel].astype(np.int64), pos)
    gap = np.where(in_gap, (rng.random(m) * g_len_all[gsel]).astype(np.int64), gap)
    room = np.where(in_gap, g_len_all[gsel].astype(np.int64) - gap, lens[blk] - pos)
    typ = rng.choice(np.array([3, 0, 1, 2, 5]), size=m, p=[0.6, 0.15, 0.1, 0.1, 0.05])
    ln = np.where(typ >= 3, 1, np.minimum(rng.integers(1, 7, size=m), room))
    typ = np.where(in_gap & (typ == 0), 2, typ)      # substitutions inside slots are insertions
    codes = rng.choice(np.array([1, 2, 4, 8, 15], np.uint32), size=(m, 6))
    codes[np.isin(typ, (1, 5))] = 0
    k = np.arange(6)
    codes = np.where(k[None, :] < ln[:, None], codes, 0)
    nucs = np.bitwise_or.reduce(codes << (4 * (5 - k)).astype(np.uint32), axis=1).astype(np.uint32)
    info = ((ln << 4) + typ).astype(np.uint8)
    n_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    pm.set_arrays(
        block_primary=np.arange(blocks, dtype=np.int32), block_seq_offsets=seq_off,
        block_seq=np.concatenate(words), gap_primary=np.arange(blocks, dtype=np.int32), gap_offsets=g_off,
        gap_position=g_pos_all, gap_length=g_len_all, block_mut_offsets=bm_off, block_mut_primary=bm_blk,
        block_mut_info=bm_info, block_mut_inversion=bm_inv, nuc_mut_offsets=n_off, nuc_mut_primary=blk,
        nuc_mut_secondary=np.full(m, -1), nuc_mut_position=pos, nuc_mut_gap_position=gap, nuc_mut_info=info,
        nuc_mut_nucs=nucs)
    return pm
