// dispatch_probe.hip — where the dispatcher puts the workgroups of a grid that fits the chip at
// once (every workgroup resident in the first fill), and in what order.
//
// Question it answers (docs/FINDINGS.md §36): the causal attention forward launches B·H·T/128
// workgroups that all fit in the first fill (GPT-2: 768 = 256 CUs x 3), so its time is the most
// loaded CU's sum, and which workgroups share a CU decides that sum.  Each workgroup records its
// XCD (HW_REG_XCC_ID), its SE / CU (HW_REG_HW_ID) and its start / end clock, then holds its slot
// for a fixed time so the whole grid is resident together.  LDS per workgroup is sized so that
// `per_cu` workgroups fit a CU (as the attention forward's VGPRs allow 3).
//
//   hipcc --offload-arch=gfx950 -O2 -o dispatch_probe benchmarks/dispatch_probe.hip
//   ./dispatch_probe [grid=768] [per_cu=3] [spin_us=30] > placement.csv
//
// Output: one CSV row per workgroup: block, xcc, se, cu, start_ns, end_ns (relative).  Reads of
// hardware registers and vector stores only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

// s_getreg immediates: id | offset << 6 | (size - 1) << 11
constexpr int kHwId = 4 | (0 << 6) | (31 << 11);   // HW_REG_HW_ID, all 32 bits
constexpr int kXccId = 20 | (0 << 6) | (15 << 11); // HW_REG_XCC_ID, low 16 bits

__global__ __launch_bounds__(256) void probe(unsigned* __restrict__ out, long long spin_ticks) {
  extern __shared__ unsigned char lds[];
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(kHwId);
    const unsigned xcc = __builtin_amdgcn_s_getreg(kXccId);
    lds[0] = 1;  // touch the allocation
    unsigned* o = out + (size_t)blockIdx.x * 6;
    o[0] = blockIdx.x;
    o[1] = xcc & 0xf;
    o[2] = (hw >> 13) & 0x7;  // se_id
    o[3] = (hw >> 8) & 0xf;   // cu_id
    o[4] = (unsigned)(t0 & 0xffffffffu);
  }
  long long t = t0;
  while (t - t0 < spin_ticks) {
    __builtin_amdgcn_s_sleep(2);
    t = wall_clock64();
  }
  __syncthreads();
  if (threadIdx.x == 0) out[(size_t)blockIdx.x * 6 + 5] = (unsigned)(wall_clock64() & 0xffffffffu);
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? std::atoi(argv[1]) : 768;
  const int per_cu = argc > 2 ? std::atoi(argv[2]) : 3;
  const double spin_us = argc > 3 ? std::atof(argv[3]) : 30.0;
  if (grid <= 0 || grid > (1 << 20) || per_cu < 1 || per_cu > 8) {
    std::fprintf(stderr, "bad arguments\n");
    return 2;
  }
  int dev = 0, wall_khz = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev));
  const long long ticks = (long long)(spin_us * 1e-3 * wall_khz);
  const size_t lds = (160 * 1024) / per_cu - 1024;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds));
  unsigned* d = nullptr;
  CHECK(hipMalloc(&d, (size_t)grid * 6 * sizeof(unsigned)));
  for (int rep = 0; rep < 3; ++rep) {  // the last launch is reported (the first pays the code load)
    CHECK(hipMemset(d, 0, (size_t)grid * 6 * sizeof(unsigned)));
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), lds, 0, d, ticks);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  std::vector<unsigned> h((size_t)grid * 6);
  CHECK(hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
  unsigned tmin = 0xffffffffu;
  for (int i = 0; i < grid; ++i) tmin = h[i * 6 + 4] < tmin ? h[i * 6 + 4] : tmin;
  const double ns = 1e6 / wall_khz;
  std::printf("block,xcc,se,cu,start_ns,end_ns\n");
  for (int i = 0; i < grid; ++i)
    std::printf("%u,%u,%u,%u,%.0f,%.0f\n", h[i * 6], h[i * 6 + 1], h[i * 6 + 2], h[i * 6 + 3],
                (double)(h[i * 6 + 4] - tmin) * ns, (double)(h[i * 6 + 5] - tmin) * ns);
  CHECK(hipFree(d));
  return 0;
}
