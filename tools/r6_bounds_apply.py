"""Round 6 diagnostic (scratch trees only): every workspace pointer the fused
kernel takes from its residency table (Ctx::a) is checked against the
problem's LDS plan and HBM workspace.  A bad one is recorded (first event:
array, pointer bits, thread, workgroup, count) in a device global read by
thip_debug_bad(), and replaced by the array's HBM home so the run can go on.

    python tools/r6_bounds_apply.py <tree>
"""
import sys

root = sys.argv[1] + "/trajopt-1_amd/csrc/"
p = root + "sqp_kernel.hip"
s = open(p).read()
old = ("  __device__ __forceinline__ double* a(int k) const { return ptab ? ptab[k] : w + L.doff[k]; }\n")
new = ("  __device__ double* a(int k) const\n  {\n    double* p = ptab ? ptab[k] : w + L.doff[k];\n"
       "    const bool in_lds = big && p >= big && p < big + L.lds_budget;\n"
       "    const bool in_ws = p >= w && p < w + L.dstride;\n"
       "    if (!in_lds && !in_ws && k != A_CHM)\n    {\n"
       "      if (atomicAdd(&g_bad[0], 1ULL) == 0)\n      {\n"
       "        g_bad[1] = k;\n        g_bad[2] = reinterpret_cast<unsigned long long>(p);\n"
       "        g_bad[3] = threadIdx.x;\n        g_bad[4] = blockIdx.x;\n"
       "        g_bad[5] = reinterpret_cast<unsigned long long>(big);\n"
       "        g_bad[6] = reinterpret_cast<unsigned long long>(w);\n      }\n"
       "      p = w + L.doff[k];\n    }\n    return p;\n  }\n")
assert s.count(old) == 1
s = s.replace(old, new)
old = "struct Ctx\n{\n"
new = "__device__ unsigned long long g_bad[8];\nstruct Ctx\n{\n"
assert s.count(old) == 1
s = s.replace(old, new)
s += ('\n#if THIP_GENERIC_ONLY\nextern "C" int thip_debug_bad(unsigned long long* out)\n#else\n'
      'extern "C" int thip_debug_bad_main(unsigned long long* out)\n#endif\n{\n'
      '  return hipMemcpyFromSymbol(out, HIP_SYMBOL(thip::g_bad), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -1;\n'
      '}\n')
open(p, "w").write(s)
print("bounds patch applied to", sys.argv[1])
