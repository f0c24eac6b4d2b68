#!/usr/bin/env python3
"""Static check of a gfx950 assembly file for VGPRs consumed while the vector-memory load
that writes them may still be in flight (a missing or too-weak `s_waitcnt vmcnt`) -- the
hazard class a spilled value reloaded from scratch would hit if its wait were missing.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -x hip --cuda-device-only -S SRC -o out.s
    tools/isa_waitcnt_check.py out.s [kernel-substring]

Model (gfx9 counters, as the compiler's waitcnt pass assumes for gfx950): every VMEM load
(global_/buffer_/flat_/scratch_load*, not the LDS-DMA forms) puts its destination VGPRs in
flight; vector-memory operations (loads, stores, atomics, LDS-DMA) retire in issue order, so
`s_waitcnt vmcnt(N)` retires exactly the in-flight loads with at least N younger VMEM
operations behind them.  A VGPR read or written by any later
instruction while it is still in flight is reported.  Control flow: basic blocks split at
labels and branches; the in-flight sets meet at joins (union, fewest younger loads), iterated
to a fixpoint.  The same for LDS reads (lgkmcnt, in order) and scalar loads (lgkmcnt, out of order: only
lgkmcnt(0) retires them).  Prints one line per kernel: loads, scratch reloads, and hazards
(expected 0).
"""
import re
import subprocess
import sys

VMEM_LOAD = re.compile(r"^(global_load|buffer_load|flat_load|scratch_load)\w*")
VMEM_ANY = re.compile(r"^(global|buffer|flat|scratch)_(load|store|atomic)\w*")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
LDS_LOAD = re.compile(r"^ds_(read|load)\w*")
SMEM_LOAD = re.compile(r"^s_(buffer_)?load\w*")


def sgprs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def vgprs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def parse_kernels(lines):
    kernels, cur, body = {}, None, []
    for line in lines:
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end") or line.startswith("\t.end_amdhsa_kernel"):
            kernels[cur] = body
            cur = None
            continue
        body.append(line)
    return kernels


def blocks_of(body):
    """[(label, [instructions], [successor labels])] in order."""
    blocks, label, insts = [], "entry", []
    for raw in body:
        s = raw.split(";")[0].strip()
        if not s or s.startswith("."):
            m = re.match(r"^(\.LBB\S+):", raw.strip())
            if m:
                blocks.append([label, insts])
                label, insts = m.group(1), []
            continue
        if s.endswith(":"):
            blocks.append([label, insts])
            label, insts = s[:-1], []
            continue
        insts.append(s)
    blocks.append([label, insts])
    out = []
    for i, (lab, ins) in enumerate(blocks):
        succ = []
        fall = True
        if ins:
            op = ins[-1].split()[0]
            if op == "s_branch":
                succ.append(ins[-1].split()[1])
                fall = False
            elif op.startswith("s_cbranch"):
                succ.append(ins[-1].split()[1])
            elif op in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and i + 1 < len(blocks):
            succ.append(blocks[i + 1][0])
        out.append((lab, ins, succ))
    return out


def step(state, inst, report):
    """state: {(kind, reg): younger ops}: kind 'v' = a VGPR a VMEM load writes (vmcnt, in
    order), 'l' = a VGPR an LDS read writes (lgkmcnt, in order), 's' = an SGPR a scalar load
    writes (lgkmcnt, out of order: only lgkmcnt(0) retires it).  Returns the new state."""
    op = inst.split()[0]
    operands = inst[len(op):]
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", operands)
        if m:
            n = int(m.group(1))
            state = {r: y for r, y in state.items() if r[0] != "v" or y < n}
        m = re.search(r"lgkmcnt\((\d+)\)", operands)
        if m:
            n = int(m.group(1))
            state = {r: y for r, y in state.items() if r[0] == "v" or (r[0] == "l" and y < n) or (r[0] == "s" and n > 0)}
        return state
    is_lds = bool(LDS_LOAD.match(op))
    is_smem = bool(SMEM_LOAD.match(op))
    is_lgkm = op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load") or op.startswith("s_store")
    if is_lds or is_smem or is_lgkm:
        parts = [p.strip() for p in operands.split(",")]
        src_text = ",".join(parts[1:]) if (is_lds or is_smem) else operands
        used = {("v", r) for r in vgprs(src_text)} | {("l", r) for r in vgprs(src_text)} | {("s", r) for r in sgprs(src_text)}
        hit = used & set(state)
        if hit:
            report.append((inst, sorted(hit)))
            state = {r: y for r, y in state.items() if r not in hit}
        state = {r: (y + 1 if r[0] != "v" else y) for r, y in state.items()}
        if is_lds:
            for r in vgprs(parts[0]):
                state[("l", r)] = 0
        if is_smem:
            for r in sgprs(parts[0]):
                state[("s", r)] = 0
        return state
    is_load = bool(VMEM_LOAD.match(op)) and "_lds" not in op and not operands.rstrip().endswith(" lds")
    is_vmem = bool(VMEM_ANY.match(op))
    text = operands
    if is_load:   # a load may re-target registers still in flight (returns are in order): only its sources count
        parts = [p.strip() for p in operands.split(",")]
        text = ",".join(parts[1:])
    used = ({("v", r) for r in vgprs(text)} | {("l", r) for r in vgprs(operands)} | {("s", r) for r in sgprs(operands)})
    hit = used & set(state)
    if hit:
        report.append((inst, sorted(hit)))
        state = {r: y for r, y in state.items() if r not in hit}
    if is_vmem:
        state = {r: (y + 1 if r[0] == "v" else y) for r, y in state.items()}
    if is_load:
        parts = [p.strip() for p in operands.split(",")]
        for r in vgprs(parts[0]) if parts else set():
            state[("v", r)] = 0
    return state


def check(body):
    blocks = blocks_of(body)
    index = {lab: i for i, (lab, _, _) in enumerate(blocks)}
    ins_state = [None] * len(blocks)
    ins_state[0] = {}
    work = [0]
    reports = {}
    while work:
        i = work.pop()
        lab, insts, succ = blocks[i]
        st = dict(ins_state[i])
        rep = []
        for inst in insts:
            st = step(st, inst, rep)
        reports[i] = rep
        for s in succ:
            j = index.get(s)
            if j is None:
                continue
            if ins_state[j] is None:
                ins_state[j] = dict(st)
                work.append(j)
                continue
            merged = dict(ins_state[j])
            for r, y in st.items():
                merged[r] = min(y, merged.get(r, y))
            if merged != ins_state[j]:
                ins_state[j] = merged
                work.append(j)
    loads = sum(1 for _, ins, _ in blocks for x in ins if VMEM_LOAD.match(x.split()[0]))
    reloads = sum(1 for _, ins, _ in blocks for x in ins if x.split()[0].startswith("scratch_load"))
    hazards = [h for r in reports.values() for h in r]
    return loads, reloads, hazards


def main():
    lines = open(sys.argv[1]).read().splitlines()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    kernels = parse_kernels(lines)
    names = list(kernels)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    total = 0
    for name, pretty in zip(names, dem):
        if want not in pretty:
            continue
        loads, reloads, hazards = check(kernels[name])
        total += len(hazards)
        print(f"{len(hazards):3d} hazards  {loads:4d} vmem loads  {reloads:3d} scratch reloads  {pretty[:110]}")
        for inst, regs in hazards[:5]:
            print(f"      {inst}   <- in flight: {' '.join(k + str(r) for k, r in regs)}")
    print(f"total hazards: {total}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
