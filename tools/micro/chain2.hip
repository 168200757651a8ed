// Chain-step latency variants (diagnostic microbenchmark, one wave).
// v_t = c_t - G_t v_{t-1} with D = 7, N steps, G and c in registers-from-LDS.
//   V1 octet layout (the round-1 block_chain step: fma + DPP/permlane reduction)
//   V2 row lanes + readlane broadcast into SGPRs + in-lane tree
//   V3 row lanes + 64-bit DPP row_newbcast + fma chain
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
__device__ __forceinline__ double rdl(double v, int k)
{
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}
template <int K>
__device__ __forceinline__ double bcast(double v)
{
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xF, 0xF, false);
}

constexpr int kN = 16;

__global__ void k(double* out, long long* cyc, int reps)
{
  const int lane = threadIdx.x;
  double g[kN], cc[kN];
  for (int u = 0; u < kN; ++u)
  {
    g[u] = 0.01 * ((lane * 7 + u) % 13) - 0.05;
    cc[u] = 0.1 * ((lane + u) % 5);
  }
  double gr[8][8];
  for (int a = 0; a < 8; ++a)
    for (int b = 0; b < 8; ++b)
      gr[a][b] = 0.01 * ((lane * 3 + a * 8 + b) % 11) - 0.05;
  double v = lane * 1e-3;
  long long t0 = clock64();
  for (int r = 0; r < reps; ++r)
  {
#pragma unroll
    for (int u = 0; u < kN; ++u)
    {
      const double p = fma(g[u], v, cc[u]);
      v = (u & 1) ? cross_octet_sum(p) : octet_sum(p);
    }
  }
  long long t1 = clock64();
  // V2: lane i < 7 holds v[i]; readlane broadcast, in-lane tree over G row
  for (int r = 0; r < reps; ++r)
  {
#pragma unroll
    for (int u = 0; u < kN; ++u)
    {
      double s[7];
#pragma unroll
      for (int kk = 0; kk < 7; ++kk)
        s[kk] = rdl(v, kk);
      const double* G = gr[u & 7];
      const double a0 = fma(-G[0], s[0], cc[u]);
      const double a1 = -G[1] * s[1];
      const double a2 = -G[2] * s[2];
      const double a3 = -G[3] * s[3];
      const double b0 = fma(-G[4], s[4], a0);
      const double b1 = fma(-G[5], s[5], a1);
      const double b2 = fma(-G[6], s[6], a2);
      v = (b0 + b1) + (b2 + a3);
    }
  }
  long long t2 = clock64();
  // V3: DPP row_newbcast fma chain (two accumulators)
  for (int r = 0; r < reps; ++r)
  {
#pragma unroll
    for (int u = 0; u < kN; ++u)
    {
      const double* G = gr[u & 7];
      double a0 = cc[u], a1 = 0.0;
      a0 = fma(-G[0], bcast<0>(v), a0);
      a1 = fma(-G[1], bcast<1>(v), a1);
      a0 = fma(-G[2], bcast<2>(v), a0);
      a1 = fma(-G[3], bcast<3>(v), a1);
      a0 = fma(-G[4], bcast<4>(v), a0);
      a1 = fma(-G[5], bcast<5>(v), a1);
      a0 = fma(-G[6], bcast<6>(v), a0);
      v = a0 + a1;
    }
  }
  long long t3 = clock64();
  // dependent fp64 fma / add / mul latency
  double w = v;
  for (int r = 0; r < reps * kN; ++r)
    w = fma(w, 0.999, 1e-3);
  long long t4 = clock64();
  for (int r = 0; r < reps * kN; ++r)
    w = w + 1e-3;
  long long t5 = clock64();
  // V2b: readlane broadcast alone (7 doubles) + one dependent add
  for (int r = 0; r < reps * kN; ++r)
  {
    double s = rdl(w, (r & 3));
    w = w + s * 1e-9;
  }
  long long t6 = clock64();
  out[lane] = v + w;
  if (lane == 0)
  {
    const double n = (double)reps * kN;
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
    cyc[3] = t4 - t3;
    cyc[4] = t5 - t4;
    cyc[5] = t6 - t5;
    (void)n;
  }
}
int main()
{
  double* o;
  long long* c;
  hipMalloc(&o, 64 * 8);
  hipMalloc(&c, 8 * 8);
  const int reps = 256;
  for (int rep = 0; rep < 2; ++rep)
  {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, reps);
    hipDeviceSynchronize();
  }
  long long h[6];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  const double n = (double)reps * kN;
  printf("cycles per chain step: V1 octet %.1f  V2 readlane+tree %.1f  V3 dpp-bcast fma %.1f\n", h[0] / n, h[1] / n,
         h[2] / n);
  printf("dependent fp64: fma %.1f  add %.1f  readlane+mul+add %.1f\n", h[3] / n, h[4] / n, h[5] / n);
  return 0;
}
