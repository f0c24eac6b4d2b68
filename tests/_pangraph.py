"""PanGraph helpers for the M3 tests: flatten a PanGraph JSON for the oracle (one record
per line), and dump a built PanMAN in the oracle's M3 dump format."""
from __future__ import annotations


def flatten(d: dict) -> str:
    """P name circular offset n id:strand...; B id SEQUENCE; G id pos len (keys in string
    order, as jsoncpp's getMemberNames); S/I/D id seq number fields (mutation strings
    uppercased, src/panman.cpp:6221-6247)."""
    out = []
    for p in d.get("paths", []):
        blocks = [f"{b['id']}:{1 if b.get('strand') else 0}" for b in p.get("blocks", [])]
        off = p.get("offset") or 0
        out.append("\t".join(["P", p["name"], "1" if p.get("circular") else "0", str(int(off)), str(len(blocks))] + blocks))
    for b in d.get("blocks", []):
        bid = b["id"]
        out.append(f"B\t{bid}\t{b['sequence'].upper()}")
        for k in sorted((b.get("gaps") or {}).keys()):
            out.append(f"G\t{bid}\t{int(k)}\t{int(b['gaps'][k])}")
        for who, muts in b.get("mutate") or []:
            for pos, s in muts:
                out.append(f"S\t{bid}\t{who['name']}\t{int(who['number'])}\t{int(pos)}\t{s.upper()}")
        for who, muts in b.get("insert") or []:
            for (pos, off2), s in muts:
                out.append(f"I\t{bid}\t{who['name']}\t{int(who['number'])}\t{int(pos)}\t{int(off2)}\t{s.upper()}")
        for who, muts in b.get("delete") or []:
            for pos, ln in muts:
                out.append(f"D\t{bid}\t{who['name']}\t{int(who['number'])}\t{int(pos)}\t{int(ln)}")
    return "\n".join(out) + "\n"


def decode_block(words) -> str:
    tab = "-ACMGRSVTWYHKDBN"
    out = []
    for w in words:
        for k in range(8):
            c = (int(w) >> (4 * (7 - k))) & 15
            if c == 0:
                return "".join(out)
            out.append(tab[c])
    return "".join(out)


def m3_dump(f, i: int = 0) -> str:
    """Blocks (consensus, gap slots) then, per node in name order, block mutations and NucMut
    records -- the oracle_pangraph format."""
    pm = f.to_panmat(i)
    a = pm._arrays
    out = []
    for b in range(len(a["block_primary"])):
        seq = decode_block(a["block_seq"][a["block_seq_offsets"][b]:a["block_seq_offsets"][b + 1]])
        gl = []
        g = list(a["gap_primary"]).index(a["block_primary"][b])
        for k in range(a["gap_offsets"][g], a["gap_offsets"][g + 1]):
            gl.append(f"{a['gap_position'][k]}:{a['gap_length'][k]}")
        out.append("\t".join([f"block\t{a['block_primary'][b]}\t{seq}"] + gl))
    for name in sorted(pm.names):
        v = pm.index(name)
        for k in range(a["block_mut_offsets"][v], a["block_mut_offsets"][v + 1]):
            out.append(f"{name}\tB\t{a['block_mut_primary'][k]}\t{a['block_mut_info'][k]}\t{a['block_mut_inversion'][k]}")
        for k in range(a["nuc_mut_offsets"][v], a["nuc_mut_offsets"][v + 1]):
            out.append(f"{name}\tN\t{a['nuc_mut_primary'][k]}\t{a['nuc_mut_position'][k]}\t"
                       f"{a['nuc_mut_gap_position'][k]}\t{a['nuc_mut_info'][k]}\t{int(a['nuc_mut_nucs'][k]):06x}")
    return "\n".join(out) + "\n"


def random_pangraph(rng, seqs=12, blocks=8, circular=False, dup_rate=0.15, flip_rate=0.1, drop_rate=0.15):
    """A random, well-formed PanGraph JSON: blocks with gap slots, paths that drop, duplicate
    and reverse blocks, and per-occurrence substitutions / insertions / deletions."""
    import json as _json
    bases = "ACGT"
    ids = [f"B{k:03d}X" for k in range(blocks)]
    seq = {b: "".join(rng.choice(list(bases), size=int(rng.integers(12, 60)))) for b in ids}
    gaps = {}
    for b in ids:
        g = {}
        for p in sorted(set(rng.integers(0, len(seq[b]) + 1, size=int(rng.integers(0, 4))).tolist())):
            g[str(p)] = int(rng.integers(1, 6))
        gaps[b] = g
    names = [f"seq{k}|x/{k}" for k in range(seqs)]
    paths = []
    occ = {b: [] for b in ids}
    for nm in names:
        order = [b for b in ids if rng.random() > drop_rate] or [ids[0]]
        if rng.random() < dup_rate:
            order.insert(int(rng.integers(0, len(order) + 1)), order[int(rng.integers(0, len(order)))])
        if circular:
            r = int(rng.integers(0, len(order)))
            order = order[r:] + order[:r]
        pb, count = [], {}
        for b in order:
            count[b] = count.get(b, 0) + 1
            strand = bool(rng.random() > flip_rate)
            pb.append({"id": b, "name": nm, "number": count[b], "strand": strand})
            occ[b].append((nm, count[b]))
        paths.append({"name": nm, "offset": int(rng.integers(0, 9)) if circular else None, "circular": circular,
                      "blocks": pb})
    out_blocks = []
    for b in ids:
        L = len(seq[b])
        mut, ins, dele = [], [], []
        for nm, num in occ[b]:
            who = {"name": nm, "number": num, "strand": True}
            subs = [[int(p), str(rng.choice(list("ACGTN")))] for p in rng.integers(1, L + 1, size=int(rng.integers(0, 4)))]
            mut.append([who, subs])
            ii = []
            for p, gl in gaps[b].items():
                if rng.random() < 0.5:
                    off = int(rng.integers(0, gl))
                    n = int(rng.integers(1, gl - off + 1))
                    ii.append([[int(p), off], "".join(rng.choice(list(bases), size=n)).lower()])
            ins.append([who, ii])
            dd = []
            if rng.random() < 0.4:
                p = int(rng.integers(1, L + 1))
                dd.append([p, int(rng.integers(1, min(6, L + 2 - p) + 1))])
            dele.append([who, dd])
        out_blocks.append({"id": b, "sequence": seq[b].lower() if rng.random() < 0.3 else seq[b], "gaps": gaps[b],
                           "mutate": mut, "insert": ins, "delete": dele})
    return _json.dumps({"paths": paths, "blocks": out_blocks}), names
