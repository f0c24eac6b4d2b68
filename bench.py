#!/usr/bin/env python3
"""Fitch small-parsimony throughput on MI355X (site*node updates/s), driver contract.

Workload (BASELINE.json north star / SURVEY.md §8d): synthetic random-join tree (T1,
seed 1) with `--leaves` leaves per GPU and `--sites` alignment columns in total
(default 1M x 30k = N*, 1 GPU).  At N GPUs the job is weak-scaled exactly as config C4:
the tree has N x leaves leaves and the columns are sharded across ranks (S/N each), so
per-GPU work is constant; 8 GPUs = 8M leaves x 30k sites.  One step = post-order +
pre-order + mutation assignment + per-site score over the rank's shard, then one RCCL
all-gather of (score, root code) per site.  Inputs are generated on the
device before timing (resident in HBM).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import panman_amd  # noqa: E402  (after torch: one HIP runtime per process)
from panman_amd.shard import gather_site_results_device, shard_range  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md chip-level table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--leaves", type=int, default=1_000_000, help="leaves per GPU")
    p.add_argument("--sites", type=int, default=30_000, help="alignment columns in total")
    p.add_argument("--cpu-sites", type=int, default=0,
                   help="columns timed on the all-core CPU baseline (0: 2 per host thread, at least 512)")
    p.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: every core this process may use)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--e2e", action="store_true",
                   help="also time the end-to-end path (H2D of the packed leaf matrix, the run, D2H of "
                        "every mutation record) on the same workload (SURVEY.md §8d), N=1 only")
    p.add_argument("--cpu-sites-1t", type=int, default=4, help="columns timed on the 1-thread CPU baseline")
    p.add_argument("--eager", action="store_true",
                   help="launch each step's kernels one by one instead of replaying the step's launch "
                        "sequence from a hipGraph (PM_OPT_GRAPH, the default; per-kernel times then come "
                        "from an extra untimed eager pass)")
    p.add_argument("--graph", action="store_true", help="(default) hipGraph replay")
    p.add_argument("--no-subtree", action="store_true",
                   help="Fitch: leaf-parent form only (PM_OPT_SUBTREE off; A/B of the subtree form)")
    p.add_argument("--narrow", type=int, default=-1,
                   help="Fitch: PM_OPT_NARROW, most nodes per level walked in a band launch (-1: library "
                        "default 16; 0: one launch per level)")
    p.add_argument("--group", type=int, default=-1,
                   help="Fitch: PM_OPT_GROUP_WAVES, most waves of grouped pre-order levels in one launch "
                        "(-1: library default, 0: off)")
    p.add_argument("--group-levels", type=int, default=4, help="PM_OPT_GROUP_LEVELS (2 to 4)")
    p.add_argument("--no-up-group", action="store_true",
                   help="Fitch: post-order launches by height (PM_OPT_UP_GROUP off)")
    p.add_argument("--sub-down", type=int, default=-1,
                   help="Fitch: PM_OPT_SUB_DOWN, S2 / S3 records from the parent's pre-order wave (1) or "
                        "the tail (0); -1: library default")
    p.add_argument("--nt-loads", type=int, default=-1, choices=(-1, 0, 1),
                   help="set records read non-temporal (1), ordinary (0), or by level size (-1, default)")
    p.add_argument("--plain-up", type=int, default=-1,
                   help="Fitch: PM_OPT_PLAIN_UP, the grouped post-order's plain nodes in the lean kernel (1) or "
                        "not (0); >= 2: on for launches of at least that many waves; -1: library default")
    p.add_argument("--cluster", type=int, default=-1,
                   help="Fitch: PM_OPT_CLUSTER, the post-order's LDS-staged sweeps: 0 off, 1 on, >= 2 on with that "
                        "level-size threshold; -1: library default")
    p.add_argument("--mode", choices=["fitch", "sankoff", "replay"], default="fitch")
    p.add_argument("--tree", choices=["random-join", "sars-like"], default="random-join",
                   help="SURVEY.md §8d tree family: T1 random-join (N*, C4) or T2 sars-like (C3)")
    p.add_argument("--replay-leaves", type=int, default=1000)
    p.add_argument("--replay-tree", choices=["random-join", "sars-like"], default="random-join",
                   help="C5 replay tree: T1 random-join (paths <= ~30 nodes) or T2 sars-like (deep paths, "
                        "several 64-node edit chunks per tile)")
    p.add_argument("--replay-blocks", type=int, default=500)
    p.add_argument("--replay-block-len", type=int, default=10_000)
    p.add_argument("--cpu-leaves", type=int, default=128, help="leaves replayed on the CPU baseline (~10 s)")
    p.add_argument("--with", dest="with_", default="sankoff,replay,e2e,commands",
                   help="secondary blocks in the default run's line: comma list of sankoff (N* Sankoff "
                        "line), replay (C5 FASTA replay line), e2e (PCIe-inclusive rate), commands "
                        "(panmanUtils -M / --low-mem-mode / -I --fasta-aligned wall times beside the "
                        "oracle's restated drivers), or none")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_fitch.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    a = p.parse_args()
    a.graph = not a.eager
    return a


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.mode == "replay":
        return replay_main(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    extra = set() if args.with_ == "none" else set(args.with_.split(","))

    L = args.leaves * world
    S = args.sites
    lo, hi = shard_range(rank, world, S)
    s_local = hi - lo
    t0 = time.time()
    if args.tree == "random-join":
        off, idx, root = panman_amd.random_join_tree(L, seed=1)
    else:
        off, idx, root = panman_amd.sars_like_tree(L, seed=1)
    n_nodes = off.shape[0] - 1
    log(rank, f"[bench] tree: {L} leaves, {n_nodes} nodes ({time.time() - t0:.1f}s)")

    eng = panman_amd.Engine(local)
    stream = torch.cuda.current_stream()
    eng.set_stream(stream.cuda_stream)
    if args.cluster >= 0:   # (the plan is built at tree upload)
        eng.set_cluster(args.cluster)
    panman_amd.phase_reset()
    eng.tree_upload(off, idx, root)
    eng.synth_columns(lo, s_local, seed=2)
    upload_phases = {}
    for name, secs in panman_amd.phase_report():
        upload_phases[name] = round(upload_phases.get(name, 0.0) + secs, 4)
    if args.no_subtree:
        eng.set_subtree(False)
    if args.narrow >= 0:
        eng.set_narrow(args.narrow)
    if args.no_up_group:
        eng.set_up_group(False)
    if args.sub_down >= 0:
        eng.set_sub_down(bool(args.sub_down))
    if args.nt_loads != -1:   # set-record load policy (default: the library's, by level size)
        eng.set_nt_loads(args.nt_loads)
    if args.plain_up >= 0:   # 0 off, 1 on (library threshold), >= 2: on from that many waves
        eng.set_plain_up(bool(args.plain_up), args.plain_up if args.plain_up >= 2 else 0)
    if args.group >= 0 or args.group_levels != 4:
        eng.set_group(args.group if args.group >= 0 else 32768, args.group_levels)

    torch.cuda.synchronize()
    log(rank, f"[bench] columns {lo}..{hi} generated ({time.time() - t0:.1f}s)")
    gather = "none (1 GPU)"
    if world > 1:   # the product's own RCCL communicator (pm_rccl.hip); torch only ships the id
        box = [panman_amd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        try:
            eng.comm_init_rank(box[0], world, rank)
            ok = 1
        except panman_amd.PanmanError as exc:
            print(f"[bench] rank {rank}: pm_comm_init_rank failed ({exc})", file=sys.stderr, flush=True)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather = "pm_run_gather (library RCCL communicator)" if flag.item() else \
            "torch.distributed all_gather (library communicator failed to initialise)"
    ctx = dict(world=world, rank=rank, L=L, S=S, lo=lo, s_local=s_local, n_nodes=n_nodes,
               lib_gather=gather.startswith("pm_run_gather"))

    mode = panman_amd.MODE_FITCH if args.mode == "fitch" else panman_amd.MODE_SANKOFF
    main_block = parsimony_block(args, eng, mode, ctx)
    footprint = {"fitch" if mode == panman_amd.MODE_FITCH else "sankoff": eng.memory_footprint()}
    secondary = {}
    if mode == panman_amd.MODE_FITCH and "sankoff" in extra:
        log(rank, f"[bench] secondary: Sankoff on the same workload ({time.time() - t0:.1f}s)")
        secondary["sankoff"] = parsimony_block(args, eng, panman_amd.MODE_SANKOFF, ctx)
        footprint["fitch+sankoff"] = eng.memory_footprint()   # (grow-only buffers: both modes' records)
        eng.run(mode)   # leave the context as the main line ran it (cpu-baseline parity sample)
        torch.cuda.synchronize()

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log(rank, f"[bench] CPU baseline ({time.time() - t0:.1f}s)")
        cpu, parity = cpu_baseline(args, eng, off, idx, root, L, n_nodes, mode)
    e2e = None
    if rank == 0 and world == 1 and (args.e2e or "e2e" in extra):
        log(rank, f"[bench] end to end ({time.time() - t0:.1f}s)")
        e2e = end_to_end(eng, L, S, n_nodes, mode)
    eng.close()
    del eng
    torch.cuda.empty_cache()
    if world == 1 and "replay" in extra:
        log(rank, f"[bench] secondary: C5 replay ({time.time() - t0:.1f}s)")
        secondary["replay"] = replay_block(args, world, rank, local)

    commands = None
    if world == 1 and "commands" in extra and rank == 0:
        log(rank, f"[bench] command-level block ({time.time() - t0:.1f}s)")
        commands = commands_block(args)

    if rank == 0:
        out = {
            "metric": f"Fitch-Sankoff site*node updates/sec ({args.mode} mode)",
            "value": main_block["value"],
            "unit": "site*node updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_block["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 bit-planes (16-bit one-hot state sets)" if mode == panman_amd.MODE_FITCH
            else "u32 bit-planes (Z0/Z1 optimal-code sets, exact unit-cost Sankoff)",
            "data": f"synthetic (seeded on-device tree-evolved columns, {args.tree} tree)",
            "build_id": panman_amd.build_id(),
            "config": {
                "workload": workload_label(args.mode, args.tree, L, S, world),
                "tree": args.tree,
                "leaves": L, "nodes": n_nodes, "sites": S, "sites_per_gpu": s_local,
                "parallelism": f"column shards x{world}, one all-gather of per-site score/root",
                "gather": gather,
                "mutations_total": main_block["mutations_total"],
                "launch": ("hipGraph replay" if args.graph else "eager") + ", per-level kernels",
            },
            "roofline": main_block["roofline"],
            "upload": {"phases_s": upload_phases,
                       "scope": "tree flattening + descriptor upload (tree.*), on-device column generation, "
                                "and the S2 / S3 side-by-side leaf copy (upload.sub_planes, k_sub_planes)"},
            "footprint": {"device_bytes": footprint,
                          "hbm_bytes_per_gpu": 288 * 2**30,
                          "note": "pm_memory_footprint: device buffers the context holds after the run"},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "end_to_end": e2e,
            "commands": commands,
            "secondary": {k: {kk: v[kk] for kk in ("value", "unit", "ms_per_step", "metric", "roofline",
                                                   "config", "cpu_baseline", "parity_sample", "host_format_s",
                                                   "format_phases_s", "end_to_end_leaf_col_per_s",
                                                   "upload", "footprint")
                              if kk in v}
                          for k, v in secondary.items()} or None,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def workload_label(mode: str, tree: str, L: int, S: int, world: int) -> str:
    """Which BASELINE.json config a run measures (SURVEY.md §8d names): N* (1M x 30k, one
    GPU), C4 (N x 1M leaves x 30k sites over N GPUs) and its one-rank share (8M x 3750), C3
    (T2 100k x 30k), C2 (RSV-like ~4k x 15k); anything else is labelled by its shape only."""
    shape = f"{L} leaves x {S} sites {tree} tree"
    if tree == "random-join":
        if world == 1 and (L, S) == (1_000_000, 30_000):
            return f"N* {mode}: {shape} (one MI355X, north-star size)"
        if world > 1 and L == world * 1_000_000 and S == 30_000:
            return f"C4 {mode} weak scaling: {shape}, columns over {world} GPUs"
        if world == 1 and (L, S) == (8_000_000, 3_750):
            return f"C4 rank share {mode}: {shape} (one rank of --gpus 8)"
        if world == 1 and L <= 5_000 and S == 15_000:
            return f"C2 {mode}: {shape} (RSV-like size)"
    elif world == 1 and (L, S) == (100_000, 30_000):
        return f"C3 {mode}: {shape} (T2, SARS-like)"
    elif world == 1 and (L, S) == (8_000_000, 3_750):
        return f"C4 rank share (T2) {mode}: {shape} (one rank of --gpus 8 on the SARS-like tree)"
    elif world > 1 and L == world * 1_000_000 and S == 30_000:
        return f"C4 (T2) {mode} weak scaling: {shape}, columns over {world} GPUs"
    return f"{mode}: {shape} (not a BASELINE config size)"


def parsimony_block(args, eng, mode, ctx):
    """Warm up, time exactly `steps` steps of `mode` (barrier + synchronize on both sides,
    max over ranks), then the per-kernel roofline of the dominant kernel."""
    world, rank, L, S, s_local, n_nodes = (ctx[k] for k in ("world", "rank", "L", "S", "s_local", "n_nodes"))
    # per-site (score, root code) of every site of the job, on every rank
    score_all = torch.zeros(S, dtype=torch.int32, device="cuda")
    root_all = torch.zeros(S, dtype=torch.uint8, device="cuda")

    def step():
        if world > 1 and ctx["lib_gather"]:   # shard run + ONE RCCL all-gather inside the library
            eng.run_gather(mode, S, ctx["lo"], score_all.data_ptr(), root_all.data_ptr())
        elif world > 1:   # the same chunks through a torch.distributed all-gather
            eng.run(mode)
            gather_site_results_device(eng, ctx["lo"], S, score_all, root_all)
        else:   # (score, root code) of every site stay in the context's device buffers
            eng.run(mode)

    eng.set_graph(False)
    for _ in range(max(1, args.warmup)):
        step()
    muts = eng.mutation_count()   # sizes the record buffers (re-runs once if a shard overflowed)
    torch.cuda.synchronize()

    if args.graph:
        eng.set_graph(True)
        step()   # capture outside the timed region
    eng.set_profiling(not args.graph)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world == 1:   # untimed: the last step's (score, root code), record buffers checked
        eng.site_results_device(score_all.data_ptr(), root_all.data_ptr())
    if args.graph:   # per-kernel durations for the roofline: same steps, eager, untimed
        eng.set_graph(False)
        eng.set_profiling(True)
        for _ in range(args.steps):
            eng.run(mode)
        torch.cuda.synchronize()
    ms, launches = eng.kernel_times(6)
    # the pre-order pass = its levels / sweeps (class 1) + its tail launch (class 5)
    tail_ms, tail_launches = ms[5], launches[5]
    ms[1] += tail_ms
    launches[1] += tail_launches
    eng.set_profiling(False)
    design = eng.design_bytes()   # counted from the last run's record masks (untimed)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        m = torch.tensor([float(muts)], dtype=torch.float64, device="cuda")
        dist.all_reduce(m, op=dist.ReduceOp.SUM)
        muts_total = int(m.item())
    else:
        muts_total = muts

    updates = float(S) * n_nodes * args.steps
    value = updates / elapsed
    ms_step = elapsed * 1e3 / args.steps
    roofline = roofline_of(args, mode, ms, launches, design, ctx, muts, ms_step, rank, tail_ms, tail_launches)
    name = "fitch" if mode == panman_amd.MODE_FITCH else "sankoff"
    return {"metric": f"Fitch-Sankoff site*node updates/sec ({name} mode)", "value": value,
            "unit": "site*node updates/s", "ms_per_step": ms_step, "mutations_total": muts_total,
            "roofline": roofline,
            "config": {"workload": workload_label(name, args.tree, L, S, world), "sites_per_gpu": s_local}}


def traffic_key(mode: str, tree: str, leaves: int, sites: int) -> str:
    """profiles/traffic_fitch.json's workload key (tools/profile_fitch.sh writes the same):
    mode:leaves x sites-per-GPU, with the tree family unless it is the random-join default."""
    return f"{mode}:{leaves}x{sites}" + ("" if tree == "random-join" else f":{tree}")


def roofline_of(args, mode, ms, launches, design, ctx, muts, ms_step, rank, tail_ms=0.0, tail_launches=0):
    """Roofline of the dominant kernel.  `achieved` = the bytes THIS design must move per
    launch (pm_design_bytes: leaf words, compressed records written and read, compact
    finals, dirty-lane leaf words, 8 B per record -- counted from the run's record masks)
    / the kernel's average launch time (HIP events on the launch stream).  `traffic` = HBM
    bytes per launch from the rocprofv3 PMC passes committed under profiles/.  The SURVEY
    §8d state-through-memory contract (2-B sets per node) is kept as
    `contract_effective_GBs` only: this layout beats that model, so it is not a roofline."""
    L, s_local, n_nodes = ctx["L"], ctx["s_local"], ctx["n_nodes"]
    n_int = n_nodes - L
    steps = max(1, args.steps)
    fitch = mode == panman_amd.MODE_FITCH
    names = ("k_fitch_up", "k_down<Fitch>") if fitch else ("k_sankoff_up", "k_down<Sankoff>")
    # each timed class is a pass: every launch of these kernels (levels, narrow bands, wide
    # nodes, Sankoff parts, the tail of leaf-ish children) -- PMC bytes are summed per run
    up_k = ("k_fitch_up", "k_fitch_up_wide", "k_fitch_up_band", "k_fitch_up_mixed", "k_fitch_up_cluster") if fitch else \
        ("k_sankoff_up", "k_sankoff_up_wide", "k_sankoff_part", "k_sankoff_merge", "k_sankoff_up_band", "k_sankoff_up_mixed", "k_sankoff_up_cluster")
    down_k = ("k_down", "k_down_band", "k_down_cluster")
    prof_names = {names[0]: up_k, names[1]: down_k + ("k_tail",)}
    key = "fitch" if fitch else "sankoff"
    classes = {
        names[0]: (ms[0] / steps, launches[0] / steps, design["up"]),
        names[1]: (ms[1] / steps, launches[1] / steps, design["down"]),
    }
    dom = max(classes, key=lambda k: classes[k][0])
    dms, dl, dbytes = classes[dom]
    achieved = dbytes / (dms * 1e-3) / 1e9 if dms > 0 else 0.0
    traffic_all, score_traffic = {}, None   # HBM bytes per run of each pass (PMC)
    build = panman_amd.build_id()
    traffic_note = f"no PMC traffic for this workload in {os.path.relpath(args.traffic, ROOT)}"
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            wk = traffic_key(key, args.tree, L, s_local)
            # PMC bytes count only for the library build they were measured on
            stamps = {tj[n].get(wk + ":build") for kk in prof_names.values() for n in kk if wk in tj.get(n, {})}
            if stamps and stamps != {build}:
                traffic_note = (f"PMC traffic in {os.path.relpath(args.traffic, ROOT)} was measured on build(s) "
                                f"{sorted(str(x) for x in stamps)}, the loaded library is {build}: re-profile")
            elif stamps:
                traffic_note = f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes on this build ({build})"
                for k, kernels in prof_names.items():
                    got = [tj[n][wk + ":step"] for n in kernels if wk + ":step" in tj.get(n, {})]
                    traffic_all[k] = sum(got) if got else None
                score_traffic = tj.get("k_site_score", {}).get(wk + ":step")
        except (OSError, ValueError, KeyError):
            traffic_all = {}
    traffic = traffic_all[dom] / dl if traffic_all.get(dom) and dl else None   # per launch of the pass
    # the pre-order pass by kernel: its levels / bands / sweeps (k_down*) and its tail launch,
    # each kernel's design bytes (pm_design_bytes parts; the 8-B mutation records are written by
    # both and counted apart) beside its PMC bytes, per step
    parts = design.get("parts", {})
    tail_design = parts.get("down_tail_items", 0.0) + parts.get("down_tail_leaf_words", 0.0)
    levels_design = sum(parts.get(k, 0.0) for k in ("down_own_records", "down_parent_finals", "down_dirty_leaf_words",
                                                       "down_finals_written"))
    pmc_by_kernel, fetch_by_kernel = {}, {}
    if traffic_all:
        try:
            tj = json.load(open(args.traffic))
            wk = traffic_key(key, args.tree, L, s_local)
            for kk in down_k + ("k_tail",):
                v = tj.get(kk, {}).get(wk + ":step")
                if v is not None and tj[kk].get(wk + ":build") == build:
                    pmc_by_kernel[kk] = v
                    fetch_by_kernel[kk] = tj[kk].get(wk + ":fetch_step")
        except (OSError, ValueError):
            pmc_by_kernel = {}
    lv_pmc = sum(pmc_by_kernel.get(k, 0.0) for k in down_k) if any(k in pmc_by_kernel for k in down_k) else None
    tl_pmc = pmc_by_kernel.get("k_tail")
    lv_fetch = sum(fetch_by_kernel.get(k) or 0.0 for k in down_k) if any(fetch_by_kernel.get(k) for k in down_k) else None
    tl_fetch = fetch_by_kernel.get("k_tail")
    lines = design.get("line_reads", {})
    pre_split = {
        "records_bytes_per_step": 8.0 * muts,
        "records_note": "8-B mutation records: written by both kernels, not split",
        "levels": {"kernels": " + ".join(down_k), "ms_per_step": round((ms[1] - tail_ms) / steps, 3),
                   "launches_per_step": (launches[1] - tail_launches) / steps,
                   "design_bytes_per_step": levels_design, "pmc_bytes_per_step": lv_pmc,
                   "pmc_over_design": round(lv_pmc / levels_design, 3) if lv_pmc and levels_design else None,
                   "line_read_bytes_per_step": lines.get("levels"), "pmc_fetch_bytes_per_step": lv_fetch,
                   "pmc_fetch_over_line_reads": round(lv_fetch / lines["levels"], 3) if lv_fetch and lines.get("levels") else None},
        "tail": {"kernels": "k_tail", "ms_per_step": round(tail_ms / steps, 3), "launches_per_step": tail_launches / steps,
                 "design_bytes_per_step": tail_design, "pmc_bytes_per_step": tl_pmc,
                 "pmc_over_design": round(tl_pmc / tail_design, 3) if tl_pmc and tail_design else None,
                 "line_read_bytes_per_step": lines.get("tail"), "pmc_fetch_bytes_per_step": tl_fetch,
                 "pmc_fetch_over_line_reads": round(tl_fetch / lines["tail"], 3) if tl_fetch and lines.get("tail") else None},
        "line_read_parts_per_step": lines.get("parts"),
        "line_note": "line reads: the pass's loads at 128-B line granularity (pm_design_bytes out[14..19]; a scattered "
                     "16-B read draws a whole line, tools/calib_fetch.hip, profiles/r06_calib_fetch.txt)",
    }
    if fitch:   # SURVEY.md §8d contract: 2-B sets through memory
        contract = s_local * (0.5 * L + 2.0 * n_int + 2.0 * (n_int - 1)) + \
            s_local * (2.0 * n_int + 0.5 * n_int + 0.5 * (n_nodes - 1) + 0.5 * L) + 8.0 * muts
    else:       # 16 x u16 cost vectors
        contract = s_local * (1.5 * L + 97.0 * n_int)
    step_design = design["up"] + design["down"] + design["score"]
    kernel_launch_s = dms / dl * 1e-3 if dl else 0.0
    out = {
        "bound": "hbm",
        "kernel": dom,
        "kernel_note": "the pass's launches: " + " + ".join(prof_names[dom]),
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_note": traffic_note,
        "build_id": build,
        "bytes_model": "pm_design_bytes: bytes this record layout must move (16-B lane granularity)",
        "design_bytes_per_launch": dbytes / dl if dl else None,
        "traffic_over_design": round(traffic / (dbytes / dl), 3) if traffic and dl and dbytes else None,
        "traffic_GBs": round(traffic / kernel_launch_s / 1e9, 1) if traffic and kernel_launch_s else None,
        "traffic_frac": round(traffic / kernel_launch_s / 1e9 / HBM_PEAK_GBS, 4) if traffic and kernel_launch_s else None,
        "avg_launch_ms": round(dms / dl, 4) if dl else None,
        "launches_per_step": dl,
        "kernel_ms_per_step": round(dms, 3),
        "other_kernels_ms_per_step": {k: round(v[0], 3) for k, v in classes.items() if k != dom},
        "score_kernel_ms_per_step": round(ms[2] / steps, 3),
        "pre_order_by_kernel": pre_split,
        "step_design_bytes": step_design,
        "step_design_parts": {k: round(v / 1e9, 3) for k, v in design.get("parts", {}).items()},
        "step_design_parts_unit": "GB",
        "step_design_GBs": round(step_design / (ms_step * 1e-3) / 1e9, 1),
        "floor_bytes": design["floor"],
        "floor_note": "0.5 B per leaf-site (leaf codes read once) + 8 B per mutation record",
        "design_over_floor": round(step_design / design["floor"], 3),
        "floor_GBs": round(design["floor"] / (ms_step * 1e-3) / 1e9, 1),
        "contract_bytes": contract,
        "contract_effective_GBs": round(contract / (ms_step * 1e-3) / 1e9, 1),
    }
    if all(traffic_all.get(k) for k in names):
        step_traffic = sum(traffic_all[k] for k in names) + (score_traffic or 0.0)
        out["step_traffic_bytes"] = step_traffic
        out["step_traffic_GBs"] = round(step_traffic / (ms_step * 1e-3) / 1e9, 1)
        out["traffic_over_floor"] = round(step_traffic / design["floor"], 3)
    copy_gbs = round(panman_amd.stream_copy_rate(torch.cuda.current_device()), 1) if rank == 0 else None
    out["measured_copy_GBs"] = copy_gbs
    out["measured_copy_kernel"] = "k_stream_copy (pm_measure.hip): 16 B per lane, 4 loads in flight, 4 GiB"
    out["frac_of_measured_copy"] = round(achieved / copy_gbs, 4) if copy_gbs else None
    return out


def end_to_end(eng, L, S, n_nodes, mode):
    """End-to-end rate: the packed leaf matrix (0.5 B per leaf-site) goes
    host -> device through pm_leaves_upload, the full run, then every mutation record
    device -> host, sorted by (node, site).  The host matrix is built untimed from the
    device-generated columns."""
    import ctypes as C
    stride = (S + 1) // 2
    packed = np.empty((L, stride), np.uint8)
    chunk = 2048
    for s0 in range(0, S, chunk):
        ns = min(chunk, S - s0)
        codes = eng.leaf_codes(s0, ns, L)
        packed[:, s0 // 2:(s0 + ns + 1) // 2] = panman_amd.pack_codes(codes)
        del codes
    cons = eng.consensus(0, S)
    node_row = np.full(n_nodes, -1, np.int32)
    node_row[:L] = np.arange(L, dtype=np.int32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng._check(eng.lib.pm_leaves_upload(eng.ctx, S, packed.ctypes.data, stride, node_row.ctypes.data, None, 0),
               "pm_leaves_upload")
    eng.sites_upload(cons)
    t1 = time.perf_counter()
    eng.run(mode)
    n = eng.mutation_count()
    t2 = time.perf_counter()
    buf = np.empty(2 * max(n, 1), np.uint32)
    got = C.c_int64(0)
    eng._check(eng.lib.pm_mutations_fetch(eng.ctx, buf.ctypes.data, n, C.byref(got)), "pm_mutations_fetch")
    t3 = time.perf_counter()
    total = t3 - t0
    return {"seconds": round(total, 3), "value": S * n_nodes / total, "unit": "site*node updates/s",
            "h2d_s": round(t1 - t0, 3), "run_s": round(t2 - t1, 3), "d2h_s": round(t3 - t2, 3),
            "h2d_bytes": int(packed.nbytes), "d2h_bytes": int(8 * got.value), "records": int(got.value),
            "note": "pageable host buffers; records sorted by (node, site) inside pm_mutations_fetch"}


def cgroup_cpus():
    """CPUs the cgroup quota grants this process (cpu.max), or None when unlimited / unknown."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def host_threads(args):
    """Every CPU this process may run on: the affinity set, capped by the cgroup's CPU quota
    (the GPU box exposes 256 CPUs but grants a 16-CPU quota; more threads than that only
    time-slice the same 16 CPUs).  Returns (threads, usable, quota, effective)."""
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    effective = max(1, min(usable, int(quota))) if quota else usable
    return args.cpu_threads or effective, usable, quota, effective


def cpu_baseline(args, eng, off, idx, root, L, n_nodes, mode):
    """Reference-faithful CPU path (oracle: per-column unordered_map<string,int> +
    recursion, src/fitchSankoff.cpp:30-171) on a bounded column sample, plus a bit-exact
    check of the GPU kernels on the same sample at full tree size."""
    sys.path.insert(0, ROOT)
    import oracle as orc
    threads, usable, quota, effective = host_threads(args)
    ns = args.cpu_sites or 3 * threads   # ~15 s of CPU work at 1M leaves
    codes = eng.leaf_codes(0, ns, L)
    cons = eng.consensus(0, ns)
    names = [f"s{i}" if i < L else f"node_{i}" for i in range(n_nodes)]
    node_row = np.full(n_nodes, -1, np.int32)
    node_row[:L] = np.arange(L, dtype=np.int32)
    o = orc.load()
    print(f"[bench] CPU baseline: {ns} columns on {threads} threads", file=sys.stderr, flush=True)
    secs, want = o.csr_columns(off, idx, root, names, codes, node_row, cons, None, algo=mode, threads=threads)
    n1 = max(1, min(args.cpu_sites_1t, ns))
    print(f"[bench] CPU baseline: {secs:.1f}s; 1-thread sample of {n1} columns", file=sys.stderr, flush=True)
    secs1, _ = o.csr_columns(off, idx, root, names, codes[:, :n1], node_row, cons[:n1], None, algo=mode, threads=1)
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cpu = {"value": ns * n_nodes / secs, "unit": "site*node updates/s", "cores": threads,
           "kind": "port (reference unbuildable here: oracle/pm_oracle.cpp restates src/fitchSankoff.cpp)",
           "sample": f"first {ns} of the same columns, {L} leaves x {ns} sites, {threads} threads "
                     f"({secs:.1f}s), oracle/pm_oracle.cpp faithful per-column loop "
                     f"(unordered_map<string,int> per column + recursion, the reference's tbb::parallel_for body)",
           "single_thread_value": n1 * n_nodes / secs1,
           "single_thread_sample": f"first {n1} columns, 1 thread ({secs1:.1f}s): the reference M1 driver's "
                                   f"sequential loop (src/panman.cpp:1380-1381)",
           "host": {"nproc": os.cpu_count(), "usable_cpus": usable, "cgroup_cpu_quota": quota,
                    "effective_cpus": effective, "cpu_model": model, "threads_used": threads,
                    "note": "threads = every CPU the cgroup quota grants this process (all of them busy)"}}
    # GPU on the identical sample columns (same kernels, separate context)
    e2 = panman_amd.Engine(0)
    e2.tree_upload(off, idx, root)
    e2.leaves_upload(codes, node_row)
    e2.sites_upload(cons)
    e2.run(mode)
    got = e2.mutations()
    e2.close()
    parity = {"sites": ns, "records": int(want.shape[0]),
              "bit_exact": bool(got.shape == want.shape and (got == want).all())}
    return cpu, parity


def evolved_msa(leaves: int, sites: int, seed: int, mu: float = 1e-3, gap: float = 1e-4):
    """Random-join tree (T1) and a tree-evolved alignment: uniform ACGT root, per edge and
    site a substitution (mu) or a one-site gap (gap); no all-gap column.
    Returns (newick with leaves s<i>, MSA FASTA text)."""
    off, idx, root = panman_amd.random_join_tree(leaves, seed=seed)
    n = off.shape[0] - 1
    rng = np.random.default_rng(seed + 1)
    alphabet = np.frombuffer(b"-ACGT", np.uint8)
    seq = np.zeros((n, sites), np.uint8)   # 1..4 = ACGT, 0 = gap
    seq[root] = rng.integers(1, 5, size=sites)
    order = [root]
    for v in order:
        kids = idx[off[v]:off[v + 1]]
        order.extend(int(c) for c in kids)
        for c in kids:
            s = seq[v].copy()
            r = rng.random(sites)
            sub = r < mu
            s[sub] = (s[sub] + rng.integers(0, 3, size=int(sub.sum()))) % 4 + 1   # another base (gap -> a base)
            s[(r >= mu) & (r < mu + gap)] = 0
            seq[c] = s
    leaf = [v for v in range(n) if off[v] == off[v + 1]]
    all_gap = (seq[leaf] == 0).all(axis=0)
    seq[leaf[0], all_gap] = 1
    names = {v: f"s{v}" for v in leaf}

    def nwk(v):
        kids = idx[off[v]:off[v + 1]]
        return names[v] if len(kids) == 0 else "(" + ",".join(nwk(int(c)) for c in kids) + ")"
    sys.setrecursionlimit(max(10000, 4 * n))
    text = "".join(f">{names[v]}\n{alphabet[seq[v]].tobytes().decode()}\n" for v in leaf)
    return nwk(root) + ";\n", text


def commands_block(args):
    """Command-level wall times of the drop-in CLI (bin/panmanUtils over the C-ABI: input
    parsing, grouping, the GPU kernels, the PanMAN writer / FASTA text) beside the oracle's
    restatement of the reference's drivers on the same host and inputs:
      -M (M1, src/panman.cpp:1274-1466, a sequential per-column loop: 1 thread),
      --low-mem-mode (M2, :1467-1649, tbb::parallel_for over columns: every quota thread),
      -I <C5 .panman> --fasta-aligned (R1, src/fasta.cpp:1981-2099, parallel_for_each over
      leaves: every quota thread).
    The survey's compiled-reference probe of M1 on 2 000 x 2 000 took 2.63 s."""
    import subprocess
    import tempfile
    sys.path.insert(0, ROOT)
    import oracle as orc
    cli = os.path.join(ROOT, "bin", "panmanUtils")
    if not os.path.exists(cli):
        return {"error": "bin/panmanUtils not built"}
    threads = host_threads(args)[0]
    o = orc.load()
    out = {"threads": threads, "cli": "bin/panmanUtils (C++ over libpanman_amd.so, 1 GPU)",
           "oracle": "oracle/pm_oracle.cpp restated drivers (reference unbuildable here)",
           "survey_reference_probe": {"M1 2000x2000": "2.63 s", "M1 20000x300": "6.78 s",
                                      "M2 2000x2000 (serial TBB stand-in)": "9.52 s",
                                      "M2 20000x300 (serial TBB stand-in)": "19.47 s"},
           "runs": []}

    def phases_of(pairs):
        """(name, seconds) list -> {name: seconds}, repeated names summed."""
        out = {}
        for name, secs in pairs:
            out[name] = round(out.get(name, 0.0) + secs, 4)
        return out

    def run_cli(argv, cwd, stdout=None):
        """Wall seconds of one CLI run, and its phase log (PANMAN_PHASES=1 on stderr)."""
        env = dict(os.environ, PANMAN_PHASES="1")
        t = time.perf_counter()
        r = subprocess.run([cli] + argv, cwd=cwd, stdout=stdout or subprocess.PIPE, stderr=subprocess.PIPE,
                           timeout=600, env=env)
        dt = time.perf_counter() - t
        if r.returncode != 0:
            raise RuntimeError(f"panmanUtils {' '.join(argv)}: {r.stderr.decode(errors='replace')[-400:]}")
        pairs = []
        for line in r.stderr.decode(errors="replace").splitlines():
            name, tab, secs = line.rpartition("\t")
            if tab and name and not name.startswith("#"):
                try:
                    pairs.append((name, float(secs)))
                except ValueError:
                    pass
        return dt, phases_of(pairs)

    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        for leaves, sites in ((2000, 2000), (20000, 300)):
            nwk, msa = evolved_msa(leaves, sites, seed=11)
            with open(os.path.join(tmp, "t.nwk"), "w") as f:
                f.write(nwk)
            with open(os.path.join(tmp, "a.fa"), "w") as f:
                f.write(msa)
            for low_mem in (False, True):
                flag = ["--low-mem-mode"] if low_mem else []
                try:
                    gpu_s, cli_phases = run_cli(["-M", "a.fa", "-N", "t.nwk", "-o", "cmd"] + flag, tmp)
                except (RuntimeError, subprocess.TimeoutExpired) as exc:
                    out["runs"].append({"command": f"-M {'--low-mem-mode ' if low_mem else ''}{leaves}x{sites}",
                                        "error": str(exc)})
                    continue
                nt = threads if low_mem else 1
                mode = panman_amd.MODE_SANKOFF if low_mem else panman_amd.MODE_FITCH
                panman_amd.msa_build(nwk, msa, "", mode)   # warm (the first call pays the kernels' load)
                panman_amd.phase_reset()
                t = time.perf_counter()
                gdump = panman_amd.msa_build(nwk, msa, "", mode)
                gpu_drv_s = time.perf_counter() - t
                drv_phases = phases_of(panman_amd.phase_report())
                t = time.perf_counter()
                dump = o.msa_build(nwk, msa, "", mode=1 if low_mem else 0, threads=nt)
                cpu_s = time.perf_counter() - t
                recs = sum(1 for line in dump.splitlines() if line and not line.startswith("#"))
                out["runs"].append({
                    "command": f"panmanUtils -M a.fa -N t.nwk -o cmd{' --low-mem-mode' if low_mem else ''}",
                    "workload": f"{leaves} leaves x {sites} columns (random-join tree, tree-evolved MSA)",
                    "gpu_cli_wall_s": round(gpu_s, 3),
                    "gpu_driver_s": round(gpu_drv_s, 3),
                    "gpu_driver_scope": "pm_msa_build in this process (MSA parse, columns, GPU run, grouping): "
                                        "the oracle's scope",
                    "oracle_driver_s": round(cpu_s, 3), "oracle_threads": nt,
                    "oracle_scope": "construction only (the CLI also starts a process, initialises HIP and writes "
                                    "the .panman: Cap'n Proto + xz level 9)",
                    "speedup_driver": round(cpu_s / gpu_drv_s, 2), "speedup_cli": round(cpu_s / gpu_s, 2),
                    "gpu_cli_phases_s": cli_phases, "gpu_driver_phases_s": drv_phases,
                    "dumps_identical": gdump == dump, "oracle_nucmut_records": recs})
        # C5: -I <file> --fasta-aligned, text to stdout (discarded)
        from panman_amd.synth import c5_panmat
        pm = c5_panmat(leaves=args.replay_leaves, blocks=args.replay_blocks, mean_len=args.replay_block_len)
        path = os.path.join(tmp, "c5.panman")
        try:
            panman_amd.write_panman(path, [pm])
            with open(os.devnull, "wb") as devnull:
                gpu_s, cli_phases = run_cli(["-I", path, "-m"], tmp, stdout=devnull)
            eng = panman_amd.Engine(0)
            try:
                import ctypes as C
                st, keep = pm.as_struct()
                walls = []
                for rep in range(3):   # warm-up, then the better of two timed calls
                    ptr, n = C.c_void_p(), C.c_int64(0)
                    panman_amd.phase_reset()
                    t = time.perf_counter()
                    eng._check(eng.lib.pm_fasta(eng.ctx, C.byref(st), 1, C.byref(ptr), C.byref(n)), "pm_fasta")
                    walls.append(time.perf_counter() - t)
                    phases = phases_of(panman_amd.phase_report())
                    if rep < 2:
                        eng.lib.pm_free(ptr)
                gtext = eng._take_text(ptr, n)   # (the Python str copy: outside the timed call)
                del keep
                gpu_drv_s = min(walls[1:])
            finally:
                eng.close()
            text, cpu_s = o.fasta(pm, True, timed=True, threads=threads)
            out["runs"].append({
                "command": "panmanUtils -I c5.panman --fasta-aligned (stdout)",
                "workload": f"C5: {args.replay_leaves} leaves, {args.replay_blocks} blocks, aligned text "
                            f"{len(text) / 1e9:.2f} GB",
                "gpu_cli_wall_s": round(gpu_s, 3),
                "gpu_driver_s": round(gpu_drv_s, 3),
                "gpu_driver_scope": "the pm_fasta C call in this process: flatten + upload, replay, text on the "
                                    "device, download into one host buffer (the Python str copy excluded)",
                "gpu_cli_phases_s": cli_phases, "gpu_driver_phases_s": phases,
                "oracle_driver_s": round(cpu_s, 3), "oracle_threads": threads,
                "oracle_scope": "replay + text in memory (the CLI also starts a process, loads and xz-decodes "
                                "the file and writes the text)",
                "speedup_driver": round(cpu_s / gpu_drv_s, 2), "speedup_cli": round(cpu_s / gpu_s, 2),
                "records_identical": sorted(gtext.split(">")) == sorted(text.split(">"))})
            del text, gtext
        except (RuntimeError, subprocess.TimeoutExpired, OSError) as exc:
            out["runs"].append({"command": "-I c5.panman --fasta-aligned", "error": str(exc)})
    return out


def replay_main(args):
    """`--mode replay`: the C5 replay block as the line's main metric."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    out = replay_block(args, world, rank, local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def replay_block(args, world, rank, local):
    """FASTA replay (R1-R3) on config C5 (E. coli-like PanMAT, synthetic): leaf*column/s of
    the GPU replay (consensus expansion + path mutations), inputs resident in HBM; host
    formatting and the end-to-end rate are reported beside it."""
    import ctypes as C

    from panman_amd.synth import c5_panmat
    t0 = time.time()
    # weak scaling over leaves: N x replay-leaves leaves, rank r replays
    # its contiguous share; tree and mutations are replicated, no collective
    total_leaves = args.replay_leaves * world
    tree = None
    if args.replay_tree == "sars-like":
        from panman_amd.engine import sars_like_tree
        tree = sars_like_tree(total_leaves, seed=1)
    pm = c5_panmat(leaves=total_leaves, blocks=args.replay_blocks, mean_len=args.replay_block_len, tree=tree)
    off = pm.child_offsets
    leaf_nodes = [i for i in range(pm.num_nodes) if off[i] == off[i + 1]]
    lo, hi = shard_range(rank, world, len(leaf_nodes))
    eng = panman_amd.Engine(local)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    panman_amd.phase_reset()
    eng.replay_prepare(pm, (lo, hi) if world > 1 else None)
    leaves, cols, edits = eng.replay_shape()
    prep = dict(panman_amd.phase_report())
    # the kernel launch_replay picks: depth-first leaf groups when every path fits, else k_replay
    kernel = "k_replay_dfs" if prep.get("replay.dfs_groups", 0) > 0 else "k_replay"
    dfs_groups = int(prep.get("replay.dfs_groups", 0))
    log(rank, f"[bench] replay PanMAT {leaves} of {total_leaves} leaves x {cols} columns, {edits} edits "
              f"({time.time() - t0:.1f}s)")
    for _ in range(max(1, args.warmup)):
        eng.replay_run()
    torch.cuda.synchronize()
    eng.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.replay_run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    ms, launches = eng.kernel_times(4)
    eng.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    units = float(leaves) * cols
    value = float(total_leaves) * cols * args.steps / elapsed
    # path mutation records per leaf (8 B each in the SURVEY.md §8d replay model)
    a = pm._arrays
    per_node = np.diff(a["nuc_mut_offsets"])
    parent = np.full(pm.num_nodes, -1, np.int64)
    for v in range(pm.num_nodes):
        parent[pm.child_index[off[v]:off[v + 1]]] = v
    acc = per_node.astype(np.int64).copy()
    order = []   # BFS so parents come first
    q = [pm.root]
    while q:
        v = q.pop()
        order.append(v)
        q.extend(pm.child_index[off[v]:off[v + 1]].tolist())
    for v in order:
        if parent[v] >= 0:
            acc[v] += acc[parent[v]]
    path_recs = float(acc[leaf_nodes[lo:hi]].sum())
    # bytes the replay must move: every row byte written once, the consensus row read once
    # (it stays cache-resident across leaves), 5 B (column u32 + char) per edit read: the
    # depth-first kernel reads each edit of a leaf group's path-node union once per group
    # (`replay.group_edits`, counted by replay_prepare), not once per leaf below it; k_replay
    # reads every edit on each leaf's path (round 4's model, `path_model_bytes` below)
    edits_read = float(prep.get("replay.group_edits", 0.0)) if dfs_groups else 0.0
    alg_bytes = units + float(cols) + 5.0 * (edits_read if dfs_groups else 0.0)
    path_model_bytes = units + float(cols) + 5.0 * path_recs
    if not dfs_groups:
        alg_bytes = path_model_bytes
    kms = ms[3] / args.steps
    achieved = alg_bytes / (kms * 1e-3) / 1e9
    # host formatting (aligned FASTA of every leaf)
    ptr, n = C.c_void_p(), C.c_int64(0)
    eng._check(eng.lib.pm_replay_format(eng.ctx, 1, C.byref(ptr), C.byref(n)), "pm_replay_format")
    eng.lib.pm_free(ptr)   # (warm: the context's text buffer and pinned download slots)
    panman_amd.phase_reset()
    tf = time.perf_counter()
    ptr, n = C.c_void_p(), C.c_int64(0)
    eng._check(eng.lib.pm_replay_format(eng.ctx, 1, C.byref(ptr), C.byref(n)), "pm_replay_format")
    fmt_s = time.perf_counter() - tf
    fmt_phases = {}
    for name, secs in panman_amd.phase_report():
        fmt_phases[name] = round(fmt_phases.get(name, 0.0) + secs, 4)
    text = panman_amd.engine.bytes_at(ptr, n.value)   # (ctypes.string_at truncates past 2 GiB)
    eng.lib.pm_free(ptr)
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle as orc
        threads = host_threads(args)[0]
        k = max(args.cpu_leaves, 32 * threads)   # every thread replays many leaves (~2-3 s wall)
        want, secs = orc.load().fasta(pm, True, leaf_limit=k, timed=True, threads=threads)
        names = sorted(nm for nm, i in zip(pm.names, range(pm.num_nodes)) if off[i] == off[i + 1])[:k]
        got = []
        for nm in names:
            at = text.find(b">" + nm.encode() + b"\n")
            end = text.find(b">", at + 1)
            got.append(text[at: end if end >= 0 else len(text)].decode())
        parity = {"leaves": k, "bit_exact": "".join(got) == want}
        cpu = {"value": k * cols / secs, "unit": "leaf*column/s", "cores": threads, "kind": "port",
               "sample": f"first {k} leaves by name, aligned FASTA, oracle printFASTAUltraFast restatement "
                         f"({secs:.1f}s on {threads} threads, leaves in parallel as the reference's "
                         f"tbb::parallel_for_each over leaves, src/fasta.cpp:1993)"}
    # PMC-measured HBM bytes per replay launch (tools/pmc_traffic.py, key replay:LxC)
    traffic, traffic_note = None, "no PMC traffic for this workload"
    if os.path.exists(args.traffic):
        try:
            entry = json.load(open(args.traffic)).get(kernel, {})
            key = f"replay:{leaves}x{cols}"
            if key in entry and entry.get(key + ":build") == panman_amd.build_id():
                traffic = entry[key]
                traffic_note = f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes on this build ({panman_amd.build_id()})"
            elif key in entry:
                traffic_note = (f"PMC traffic measured on build {entry.get(key + ':build')}, the loaded library is "
                                f"{panman_amd.build_id()}: re-profile")
        except (OSError, ValueError):
            traffic = None
    # the replay's bytes are ~98 % row writes: the achievable write-only rate beside the spec
    write_gbs = round(panman_amd.stream_write_rate(torch.cuda.current_device()), 1) if rank == 0 else None
    out = {
        "metric": "FASTA replay leaf*column/s (aligned, GPU replay kernels)", "build_id": panman_amd.build_id(),
        "value": value, "unit": "leaf*column/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8 (ASCII IUPAC)",
        "data": f"synthetic C5-like PanMAT (seeded: {args.replay_tree} tree, blocks, gap slots, block and nuc mutations)",
        "config": {"workload": f"C5 replay: {total_leaves} leaves x {cols} aligned columns, "
                               f"{args.replay_blocks} blocks, {edits} edits, {args.replay_tree} tree",
                   "leaves": total_leaves, "leaves_per_gpu": leaves, "columns": cols,
                   "path_mutation_records_rank0": path_recs,
                   "parallelism": f"leaf shards x{world}, tree + mutations replicated, no collective"},
        "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_note": traffic_note, "design_bytes_per_launch": alg_bytes,
                     "bytes_model": "row bytes written once + consensus row once + 5 B per edit read (k_replay_dfs: "
                                    "each edit of a leaf group's path-node union once per group; k_replay: every "
                                    "edit on each leaf's path)",
                     "edits_read": edits_read if dfs_groups else path_recs, "distinct_edits": edits,
                     "path_model_frac": round(path_model_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "leaf_groups": dfs_groups,
                     "traffic_GBs": round(traffic / (kms * 1e-3) / 1e9, 1) if traffic else None,
                     "avg_launch_ms": round(kms, 4), "launches_per_step": launches[3] / args.steps,
                     "measured_write_GBs": write_gbs,
                     "measured_write_kernel": "k_stream_write (pm_measure.hip): 16 B per lane, 4 non-temporal stores in flight, "
                                              "4 GiB",
                     "frac_of_measured_write": round(achieved / write_gbs, 4) if write_gbs else None},
        "host_format_s": round(fmt_s, 3),
        "format_phases_s": fmt_phases,
        "format_scope": "pm_replay_format: segment table (host), text kernels, download of the text into one "
                        "host buffer (pinned slots drained by host threads)",
        "end_to_end_leaf_col_per_s": units / (kms * 1e-3 + fmt_s),
        "cpu_baseline": cpu, "parity_sample": parity,
    }
    eng.close()
    return out


if __name__ == "__main__":
    main()
