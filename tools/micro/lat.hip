// Latency microbenchmark (diagnostic): dependent FP64 add/fma chains and the
// octet / cross-octet DPP reductions used by block_chain, one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double octet_sum(double v)
{
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  return v;
}
__device__ __forceinline__ double cross_octet_sum(double v)
{
  v += dpp_f64<0x128>(v);
  {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  return v;
}
__global__ void k(double* out, long long* cyc, double a, double b, int n)
{
  double v = threadIdx.x * 1e-3;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) v = v * a + b;  // dependent fma
  long long t1 = clock64();
  for (int i = 0; i < n; ++i) v = v + b;      // dependent add
  long long t2 = clock64();
  for (int i = 0; i < n; ++i) v = b - octet_sum(v * a);
  long long t3 = clock64();
  for (int i = 0; i < n; ++i) v = b - cross_octet_sum(v * a);
  long long t4 = clock64();
  for (int i = 0; i < n; ++i) { float f = (float)v; f = f * (float)a + (float)b; v = f; }
  long long t5 = clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4; }
}
int main()
{
  double* o; long long* c;
  hipMalloc(&o, 64 * 8); hipMalloc(&c, 8 * 8);
  const int n = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, 0.999, 1e-3, n);
    hipDeviceSynchronize();
  }
  long long h[5]; hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  printf("cycles per iteration: fma %.1f  add %.1f  octet_step %.1f  cross_octet_step %.1f  f32-cvt-roundtrip %.1f\n",
         h[0] / (double)n, h[1] / (double)n, h[2] / (double)n, h[3] / (double)n, h[4] / (double)n);
  return 0;
}
