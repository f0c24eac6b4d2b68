#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS / instruction counts of a gfx950 assembly file.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -x hip --cuda-device-only -S SRC -o out.s
    tools/isa_stats.py out.s [substring]
"""
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().splitlines()
    kernels = {}
    cur = None
    for line in text:
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            kernels.setdefault(cur, {"insts": 0, "valu": 0, "salu": 0, "vmem": 0, "smem": 0, "lds": 0, "scratch_ops": 0})
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        k = kernels[cur]
        k["insts"] += 1
        if op.startswith("v_"):
            k["valu"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer"):
            k["smem"] += 1
        elif op.startswith("s_"):
            k["salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            k["vmem"] += 1
        elif op.startswith("ds_"):
            k["lds"] += 1
        elif op.startswith("scratch_"):
            k["scratch_ops"] += 1
    meta = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", "\n".join(text), re.S):
        body = m.group(2)
        get = lambda key: int(re.search(key + r"\s+(\d+)", body).group(1)) if re.search(key + r"\s+(\d+)", body) else -1
        meta[m.group(1)] = (get(r"\.amdhsa_next_free_vgpr"), get(r"\.amdhsa_accum_offset"),
                            get(r"\.amdhsa_private_segment_fixed_size"), get(r"\.amdhsa_group_segment_fixed_size"))
    names = list(kernels)
    pretty = demangle(names)
    for n, p in zip(names, pretty):
        if want and want not in p:
            continue
        k = kernels[n]
        v = meta.get(n, (-1, -1, -1, -1))
        print(f"{p[:110]}\n    vgpr {v[0]} scratch {v[2]} lds {v[3]} | insts {k['insts']} valu {k['valu']} salu {k['salu']} "
              f"smem {k['smem']} vmem {k['vmem']} lds {k['lds']} scratch {k['scratch_ops']}")


if __name__ == "__main__":
    main()
