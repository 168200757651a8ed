"""Round 6 diagnostic (scratch trees only): NaN-poison everything the fused
kernel could read before writing -- the HBM workspace at thip_create (all bits
set: a quiet NaN in every double) and the problem's dynamic LDS at the start of
every problem -- so a read of unwritten memory shows as a NaN result instead of
depending on what an earlier allocation or launch left there.

    python tools/r6_poison_apply.py <tree>
"""
import sys

root = sys.argv[1] + "/trajopt-1_amd/csrc/"


def edit(f, old, new):
    p = root + f
    s = open(p).read()
    assert s.count(old) == 1, (f, old[:60], s.count(old))
    open(p, "w").write(s.replace(old, new))


edit("thip_api.hip", "    return fail(std::string(\"hipMalloc(workspace): \") + hipGetErrorString(e));\n",
     "    return fail(std::string(\"hipMalloc(workspace): \") + hipGetErrorString(e));\n"
     "  if ((e = hipMemset(ctx->d_ws, 0xFF, B * static_cast<size_t>(L.dstride) * sizeof(double))) != hipSuccess)\n"
     "    return fail(\"poison\");\n")
edit("sqp_kernel.hip", "  double* wsb = args.ws + (long long)b * L.dstride;\n",
     "  double* wsb = args.ws + (long long)b * L.dstride;\n"
     "  __syncthreads();\n"
     "  for (int k = threadIdx.x; k < L.lds_budget; k += kBlock)\n"
     "    dyn[k] = __longlong_as_double(-1LL);\n"
     "  __syncthreads();\n")
print("poison patch applied to", sys.argv[1])
