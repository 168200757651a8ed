// Standalone benchmark of block_chain (diagnostic, extracted from sqp_kernel.hip)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ lds_f64* lds(double* p) { return (lds_f64*)p; }
__device__ __forceinline__ const lds_f64* lds(const double* p) { return (const lds_f64*)p; }

// ---- wave-level chain of the block solve ---------------------------------
// 64-bit DPP move (two 32-bit halves)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// sum over the 8 lanes of a lane octet (lane & 7): xor 1, xor 2 (quad_perm),
// then the mirrored octet half (row_half_mirror)
__device__ __forceinline__ double octet_sum(double v)
{
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  return v;
}
// sum over the 8 octets (lane >> 3) at fixed lane & 7: xor 8 (row_ror:8),
// xor 16 (v_permlane16_swap), xor 32 (v_permlane32_swap) -- gfx950
__device__ __forceinline__ double cross_octet_sum(double v)
{
  v += dpp_f64<0x128>(v);  // row_ror:8 within each 16-lane row
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

// Block-bidiagonal recurrence v_t = c_t - G_t v_{t-1} (FWD, t = 1..N-1) or
// v_t = c_t - G_t v_{t+1} (backward, t = N-2..0), run by one wave.  Lane
// (i, k) = (lane >> 3, lane & 7) multiplies one element of the D x D block.
// The vector alternates between "column" layout (value indexed by k) and
// "row" layout (indexed by i): odd steps reduce over k inside an octet, even
// steps use the transposed block and reduce over i across octets, so no
// lane permutation (ds_bpermute) sits on the serial path.  Blocks and c
// values are loaded kChainChunk steps at a time into registers (one LDS wait
// per chunk); inside a chunk the steps are unrolled with static parity.
constexpr int kChainChunk = 8;

template <bool FWD>
__device__ __forceinline__ void block_chain(const double* Gp, const double* cvp, double* outp, int N, int D,
                                            int lane)
{
  const lds_f64* G = lds(Gp);
  const lds_f64* cv = lds(cvp);
  lds_f64* out = lds(outp);
  const int i = lane >> 3, k = lane & 7;
  const bool act = (i < D) && (k < D);
  const int DD = D * D;
  const int t0 = FWD ? 0 : N - 1;
  double v = (k < D) ? cv[t0 * D + k] : 0.0;  // column layout
  if (i == 0 && k < D)
    out[t0 * D + k] = v;
  // offsets of this lane's element in the normal / transposed block
  const int off_n = i * D + k, off_t = k * D + i;
  for (int s0 = 1; s0 < N; s0 += kChainChunk)
  {
    double g[kChainChunk], cc[kChainChunk];
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const int s = s0 + u;
      const int t = FWD ? s : N - 1 - s;
      const bool ok = s < N;
      // s0 is odd, so even u are odd steps (normal block, c by row i)
      if ((u & 1) == 0)
      {
        g[u] = (ok && act) ? G[t * DD + off_n] : 0.0;
        cc[u] = (ok && i < D) ? cv[t * D + i] : 0.0;
      }
      else
      {
        g[u] = (ok && act) ? G[t * DD + off_t] : 0.0;
        cc[u] = (ok && k < D) ? cv[t * D + k] : 0.0;
      }
    }
    // serial part: no loads, stores or branches (steps past N compute zeros)
    double vs[kChainChunk];
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const double p = g[u] * v;
      if ((u & 1) == 0)
        v = cc[u] - octet_sum(p);  // row layout: v = v_t[i]
      else
        v = cc[u] - cross_octet_sum(p);  // column layout: v = v_t[k]
      vs[u] = v;
    }
#pragma unroll
    for (int u = 0; u < kChainChunk; ++u)
    {
      const int s = s0 + u;
      const int t = FWD ? s : N - 1 - s;
      if ((u & 1) == 0)
      {
        if (s < N && k == 0 && i < D)
          out[t * D + i] = vs[u];
      }
      else if (s < N && i == 0 && k < D)
        out[t * D + k] = vs[u];
    }
  }
}


__global__ void bench(long long* cyc, double* outg, int N, int D, int reps)
{
  __shared__ double G[64 * 64];
  __shared__ double cv[64 * 8];
  __shared__ double out[64 * 8];
  for (int e = threadIdx.x; e < N * D * D; e += blockDim.x) G[e] = 0.01 * ((e * 7) % 13) - 0.05;
  for (int e = threadIdx.x; e < N * D; e += blockDim.x) cv[e] = 0.1 * (e % 5);
  __syncthreads();
  long long t0 = clock64();
  for (int r = 0; r < reps; ++r)
  {
    if (threadIdx.x < 64) block_chain<true>(G, cv, out, N, D, threadIdx.x);
    __syncthreads();
  }
  long long t1 = clock64();
  for (int r = 0; r < reps; ++r)
  {
    if (threadIdx.x < 64) block_chain<false>(G, cv, out, N, D, threadIdx.x);
    __syncthreads();
  }
  long long t2 = clock64();
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
  for (int e = threadIdx.x; e < N * D; e += blockDim.x) outg[e] = out[e];
}
int main()
{
  long long* c; double* o;
  hipMalloc(&c, 16 * 8); hipMalloc(&o, 64 * 8 * 8);
  const int reps = 200;
  for (int bs : {64, 256})
  {
    for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(bench, dim3(1), dim3(bs), 0, 0, c, o, 30, 7, reps);
    hipDeviceSynchronize();
    long long h[2]; hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    printf("block %d: fwd chain %.0f cycles, bwd chain %.0f cycles (N=30, D=7)\n", bs, h[0] / (double)reps, h[1] / (double)reps);
  }
  return 0;
}
