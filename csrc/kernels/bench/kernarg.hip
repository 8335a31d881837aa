// kernarg.hip — largest by-value kernel argument HIP accepts on gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N> struct Big { long v[N]; };
template <int N> __global__ void k(Big<N> b, long* out) { if (threadIdx.x == 0) out[0] = b.v[0] + b.v[N - 1]; }
template <int N> void run(long* d) {
  Big<N> b; for (int i = 0; i < N; ++i) b.v[i] = i;
  hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, 0, b, d);
  hipError_t e = hipDeviceSynchronize(); long h = -1; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("kernarg %6d B: %s result %ld (want %d)\n", (int)sizeof(b), hipGetErrorString(e), h, N - 1);
}
int main() { long* d; hipMalloc(&d, 8); run<256>(d); run<512>(d); run<1024>(d); run<2048>(d); return 0; }
