"""Debug: histogram of records per flush (Fitch pre-order waves), read with pm_dbg_hist()."""
import sys
p = sys.argv[1] + "/pm_kernels.h"
s = open(p).read()
old = "    if (lane == 0) base = atomicAdd(&a.shard_cnt[em.shard], total);\n"
assert old in s
s = s.replace(old, old + "    if (lane == 0 && a.dbg) atomicAdd(&a.dbg[total < 4095u ? total : 4095u], 1u);\n")
old = "    const uint4* sleaf;"
if old not in s:
    old = "    int32_t sbase;         // ... of dense index sbase + item\n"
assert old in s
s = s.replace(old, old + "    uint32_t* dbg = nullptr;\n")
open(p, "w").write(s)
p = sys.argv[1] + "/pm_fitch.hip"
s = open(p).read()
old = "    dn.vinner = dt.vinner;\n"
assert old in s
s = s.replace(old, old + "    dn.dbg = pm_dbg_buf();\n")
head = "hipError_t launch_fitch("
i = s.index(head)
j = s.rfind("\n", 0, s.rfind("namespace", 0, i))  # insert before the enclosing line is fragile; use a plain global
s = s[:i] + """static uint32_t* g_dbg_hist = nullptr;
static uint32_t* pm_dbg_buf() {
    if (!g_dbg_hist && hipMalloc(reinterpret_cast<void**>(&g_dbg_hist), 4096 * 4) == hipSuccess)
        (void)hipMemset(g_dbg_hist, 0, 4096 * 4);
    return g_dbg_hist;
}
""" + s[i:]
s += """
extern "C" int pm_dbg_hist(uint32_t* out, int clear) {
    uint32_t* b = pm::pm_dbg_buf();
    if (!b) return -3;
    if (hipDeviceSynchronize() != hipSuccess) return -4;
    if (hipMemcpy(out, b, 4096 * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (clear && hipMemset(b, 0, 4096 * 4) != hipSuccess) return -2;
    return 0;
}
"""
open(p, "w").write(s)
