// Barrier and LDS hand-off latency (diagnostic microbenchmark): one 256-thread
// workgroup (4 waves, one per SIMD, as sqp_kernel runs), timed with s_memtime.
//   barrier      __syncthreads() back to back
//   handoff      one lane of wave w writes a double to LDS, barrier, wave w+1 reads it
//                and adds (the dependent LDS + barrier + fp64 round trip of a phase edge)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void bench(long long* out, double* sink, int n)
{
  __shared__ double buf[256];
  const int tid = threadIdx.x;
  buf[tid] = tid;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i)
    __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  double v = tid * 1e-3;
  for (int i = 0; i < n; ++i)
  {
    buf[tid] = v;
    __syncthreads();
    v = buf[(tid + 64) & 255] + 1.0;
    __syncthreads();
  }
  long long t2 = __builtin_amdgcn_s_memtime();
  if (tid == 0)
  {
    out[0] = t1 - t0;
    out[1] = t2 - t1;
  }
  sink[tid] = v;
}

int main()
{
  long long* d;
  double* s;
  hipMalloc(&d, 2 * sizeof(long long));
  hipMalloc(&s, 256 * sizeof(double));
  const int n = 4096;
  hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, d, s, n);
  hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, d, s, n);
  long long h[2];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("cycles: barrier %.1f  lds_handoff %.1f\n", (double)h[0] / n, (double)h[1] / n);
  hipFree(d);
  hipFree(s);
  return 0;
}
