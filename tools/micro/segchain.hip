// Diagnostic microbenchmark (gfx950): the ADMM segment's block chain as
// sqp_kernel.hip's seg_chain_solve runs it -- one workgroup of 256 threads,
// waves 0 and 1 each run a 16-step half (octet layout, fma + DPP / permlane
// reductions), blocks and right-hand side in LDS -- timed per wave without the
// barriers.  Variants:
//   lds   blocks loaded from LDS one group of 4 steps ahead (the kernel's code)
//   regs  blocks held in registers across iterations (the loads' cost removed)
//   bare  the dependent step alone (fma + reduction, no LDS traffic at all)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) double lds_f64;

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
__device__ __forceinline__ double lds_at(unsigned a) { return *(const lds_f64*)(unsigned long)a; }

constexpr int H = 16, G = 4, D = 7, DD = 49;

template <int V>
__global__ __launch_bounds__(256) void k(double* out, long long* cyc, int reps)
{
  __shared__ double LI[2 * H * DD], MF[2 * H * DD], NB[2 * H * DD], BV[2 * H * D + 8], ZERO[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 2 * H * DD; e += 256)
  {
    LI[e] = 0.01 * ((e * 7) % 13) + 0.3;
    MF[e] = 0.001 * ((e * 5) % 11) - 0.005;
    NB[e] = 0.001 * ((e * 3) % 7) - 0.003;
  }
  for (int e = tid; e < 2 * H * D + 8; e += 256)
    BV[e] = 0.1 * (e % 5);
  if (tid == 0)
    ZERO[0] = 0.0;
  __syncthreads();
  const int i = lane >> 3, kk = lane & 7;
  const bool act = i < D && kk < D;
  const unsigned z = (unsigned)(unsigned long)(lds_f64*)ZERO;
  const unsigned base = wave * H * DD * 8;
  const unsigned offN = (i * D + kk) * 8, offT = (kk * D + i) * 8;
  const unsigned li_n = act ? (unsigned)(unsigned long)(lds_f64*)LI + base + offN : z;
  const unsigned li_t = act ? (unsigned)(unsigned long)(lds_f64*)LI + base + offT : z;
  const unsigned mf_n = act ? (unsigned)(unsigned long)(lds_f64*)MF + base + offN : z;
  const unsigned mf_t = act ? (unsigned)(unsigned long)(lds_f64*)MF + base + offT : z;
  const unsigned nb_n = act ? (unsigned)(unsigned long)(lds_f64*)NB + base + offN : z;
  const unsigned nb_t = act ? (unsigned)(unsigned long)(lds_f64*)NB + base + offT : z;
  const int stride = act ? DD * 8 : 0;
  const unsigned b0 = (unsigned)(unsigned long)(lds_f64*)BV + wave * H * D * 8;
  const unsigned b_e = b0 + ((i < D) ? i : D - 1) * 8, b_o = b0 + ((kk < D) ? kk : D - 1) * 8;
  const int R = 15;
  double acc = 0;
  long long own_f = 0, own_b = 0;
  double rli[H], rmf[H], rnb[H];
  if (V == 1)
    for (int r = 0; r < H; ++r)
    {
      rli[r] = lds_at(r < R ? ((r & 1) ? li_n : li_t) + r * stride : z);
      rmf[r] = lds_at(r < R ? ((r & 1) ? mf_n : mf_t) + r * stride : z);
      rnb[r] = lds_at(r < R ? ((r & 1) ? nb_t : nb_n) + r * stride : z);
    }
  for (int rep = 0; rep < reps; ++rep)
  {
    __syncthreads();
    long long t0 = clock64();
    double q[H];
    double y = 0.0;
    if (wave < 2)
    {
      double li[H], mf[H], lb[H];
      auto load = [&](int r) {
        const bool on = r < R;
        const bool odd = r & 1;
        if (V == 0)
        {
          li[r] = lds_at(on ? (odd ? li_n : li_t) + r * stride : z);
          mf[r] = lds_at(on ? (odd ? mf_n : mf_t) + r * stride : z);
        }
        else
        {
          li[r] = rli[r];
          mf[r] = rmf[r];
        }
        lb[r] = (V == 2) ? 0.5 : lds_at(on ? (odd ? b_o : b_e) + r * 8 * D : z);
      };
#pragma unroll
      for (int u = 0; u < G; ++u)
        load(H - 1 - u);
#pragma unroll
      for (int g = 0; g < H / G; ++g)
      {
        if (g + 1 < H / G)
        {
#pragma unroll
          for (int u = 0; u < G; ++u)
            load(H - 1 - G * (g + 1) - u);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < G; ++u)
        {
          const int r = H - 1 - G * g - u;
          const double p = fma(-mf[r], y, li[r] * lb[r]);
          y = (r & 1) ? octet_sum(p) : cross_octet_sum(p);
          q[r] = li[r] * y;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    long long t1 = clock64();
    own_f += t1 - t0;
    __syncthreads();
    t0 = clock64();
    if (wave < 2)
    {
      double nb[H];
#pragma unroll
      for (int r = 0; r < H; ++r)
        nb[r] = (V == 0) ? lds_at(r < R ? ((r & 1) ? nb_t : nb_n) + r * stride : z) : rnb[r];
      __builtin_amdgcn_sched_barrier(0);
      double x = y;
#pragma unroll
      for (int r = 0; r < H; ++r)
      {
        const double p2 = fma(-nb[r], x, q[r]);
        x = (r & 1) ? cross_octet_sum(p2) : octet_sum(p2);
        acc += x;
      }
    }
    t1 = clock64();
    own_b += t1 - t0;
  }
  out[blockIdx.x * 256 + tid] = acc;
  if (blockIdx.x == 0 && lane == 0 && wave < 2)
  {
    cyc[wave * 2] = own_f;
    cyc[wave * 2 + 1] = own_b;
  }
}

int main(int argc, char** argv)
{
  const int grid = argc > 1 ? atoi(argv[1]) : 1;  // workgroups (1: one CU; 256+: every CU busy)
  double* o;
  long long* c;
  hipMalloc(&o, 256 * 8 * (size_t)grid);
  hipMalloc(&c, 8 * 8);
  const int reps = 512;
  const char* names[3] = { "lds", "regs", "bare" };
  for (int v = 0; v < 3; ++v)
  {
    long long h[4];
    for (int rep = 0; rep < 2; ++rep)
    {
      if (v == 0)
        hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, o, c, reps);
      else if (v == 1)
        hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, o, c, reps);
      else
        hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, o, c, reps);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    printf("grid %d %-5s forward %.1f  backward %.1f cycles per step (wave 0), forward %.1f  backward %.1f (wave 1)\n",
           grid, names[v], h[0] / (reps * 16.0), h[1] / (reps * 16.0), h[2] / (reps * 16.0), h[3] / (reps * 16.0));
  }
  return 0;
}
