"""Round 6 diagnostic (scratch trees only): every workspace pointer the fused
kernel takes from its residency table (Ctx::a / Ctx::ia) checked against the
problem's LDS plan and HBM workspace; the first bad ones are printed.

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
       "    if (!in_lds && !in_ws && k != A_CHM)\n"
       "      printf(\"BOUNDS a(%d) tid %d block %d: p %p big %p w %p budget %d dstride %lld\\n\", k, (int)threadIdx.x,\n"
       "             (int)blockIdx.x, (void*)p, (void*)big, (void*)w, L.lds_budget, (long long)L.dstride);\n"
       "    return p;\n  }\n")
assert s.count(old) == 1
s = s.replace(old, new)
old = "  __device__ __forceinline__ int* ia(int k) const { return iw + L.ioff[k]; }\n"
new = ("  __device__ int* ia(int k) const\n  {\n"
       "    if (k < 0 || k >= I_COUNT || L.ioff[k] < 0 || L.ioff[k] >= L.istride)\n"
       "      printf(\"BOUNDS ia(%d) tid %d block %d\\n\", k, (int)threadIdx.x, (int)blockIdx.x);\n"
       "    return iw + L.ioff[k];\n  }\n")
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
print("bounds patch applied to", sys.argv[1])
