"""Every shipped gfx950 kernel consumes a register only after the wait that covers the load
writing it (VMEM vmcnt incl. scratch reloads of spilled values, LDS and scalar lgkmcnt):
tools/isa_waitcnt_check.py over the device assembly of each .hip source, compiled with the
library's flags.  CPU only (hipcc cross-compiles); guards the spilling kernels."""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
         "-x", "hip", "--cuda-device-only", "-S"]

sys.path.insert(0, os.path.join(ROOT, "tools"))


def _asm(src, out_dir):
    out = os.path.join(out_dir, os.path.basename(src) + ".s")
    subprocess.run([HIPCC] + FLAGS + [src, "-o", out], check=True, capture_output=True)
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_register_consumed_before_its_wait(tmp_path):
    import isa_waitcnt_check as chk
    sources = sorted(glob.glob(os.path.join(ROOT, "panman_amd", "csrc", "*.hip")))
    assert sources
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        outs = list(ex.map(lambda s: _asm(s, str(tmp_path)), sources))
    checked, bad = 0, []
    for path in outs:
        kernels = chk.parse_kernels(open(path).read().splitlines())
        for name, body in kernels.items():
            loads, reloads, hazards = chk.check(body)
            checked += 1
            if hazards:
                bad.append((os.path.basename(path), name, hazards[:3]))
    assert checked > 50
    assert not bad, bad


def test_checker_sees_a_missing_wait():
    import isa_waitcnt_check as chk
    body = [
        "\tglobal_load_dwordx4 v[4:7], v[0:1], off",
        "\ts_waitcnt vmcnt(0)",
        "\tv_add_u32_e32 v8, v4, v5",
        "\tglobal_load_dwordx4 v[10:13], v[0:1], off",
        "\tv_add_u32_e32 v9, v10, v5",      # v10 still in flight
        "\ts_load_dwordx2 s[4:5], s[0:1], 0x0",
        "\ts_add_u32 s6, s4, 1",            # s4 still in flight
        "\ts_endpgm",
    ]
    _, _, hazards = chk.check(body)
    assert len(hazards) == 2
