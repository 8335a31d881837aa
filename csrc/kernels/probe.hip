// probe.hip — host-side cost of the pieces of a kernel launch on this stack
// (torch.ops.nbd.launch_probe; benchmarks/launch_probe.py).  An eager SmolLM2 notebook step is
// host-bound (≈570 launches per step, docs/FINDINGS.md §15): this measures what one launch costs
// the issuing thread — hipLaunchKernelGGL with a small and a GEMM-sized argument block, the
// launch through a pre-resolved hipFunction_t (hipModuleLaunchKernel with a packed argument
// buffer), and the wrappers every op adds around it (stream getter, device guard, error check,
// a caching-allocator at::empty).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/hip/HIPException.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <chrono>
#include <vector>

namespace nbd {
namespace probe {

struct Small {
  float* p;
  int n;
};
struct Big {  // the size class of gemm.hip's Args (pointers, strides, flags)
  const void* ptr[8];
  int64_t v[20];
  int i[8];
};

__global__ void small_kernel(Small a) {
  if (a.n < 0 && threadIdx.x == 0) a.p[blockIdx.x] = 0.f;  // never taken (n >= 0)
}
__global__ void big_kernel(Big a) {
  if (a.i[0] < 0 && threadIdx.x == 0) reinterpret_cast<float*>(const_cast<void*>(a.ptr[0]))[0] = 0.f;
}

// mode: 0 small-arg hipLaunchKernelGGL, 1 GEMM-sized args, 2 hipModuleLaunchKernel (small, packed
// buffer, function resolved once), 3 = 0 + stream getter + guard + hipGetLastError per launch,
// 4 = 3 + one at::empty per launch, 5 = 0 with 8 workgroups of 256 (a real grid shape).
// Returns host microseconds per launch (the kernels run; the device is synchronised before and
// after, outside the timed loop).
double launch_probe(const at::Tensor& dev_tensor, int64_t n, int64_t mode) {
  TORCH_CHECK(dev_tensor.is_cuda() && n > 0, "launch_probe: a GPU tensor and n > 0");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard0(dev_tensor.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  Small s{static_cast<float*>(dev_tensor.data_ptr()), 1};
  Big b{};
  b.ptr[0] = dev_tensor.data_ptr();
  b.i[0] = 1;
  hipFunction_t fn = nullptr;
  if (mode == 2) C10_HIP_CHECK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&small_kernel)));
  C10_HIP_CHECK(hipStreamSynchronize(st));
  auto t0 = std::chrono::steady_clock::now();
  for (int64_t it = 0; it < n; ++it) {
    switch (mode) {
      case 0: hipLaunchKernelGGL(small_kernel, dim3(1), dim3(64), 0, st, s); break;
      case 1: hipLaunchKernelGGL(big_kernel, dim3(1), dim3(64), 0, st, b); break;
      case 2: {
        size_t sz = sizeof(Small);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &s, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        C10_HIP_CHECK(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg));
        break;
      }
      case 3:
      case 4: {
        const c10::hip::HIPGuardMasqueradingAsCUDA guard(dev_tensor.device());
        hipStream_t s2 = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
        if (mode == 4) {
          at::Tensor t = at::empty({1024}, dev_tensor.options());
          s.p = static_cast<float*>(t.data_ptr());
        }
        hipLaunchKernelGGL(small_kernel, dim3(1), dim3(64), 0, s2, s);
        C10_HIP_KERNEL_LAUNCH_CHECK();
        break;
      }
      default: hipLaunchKernelGGL(small_kernel, dim3(8), dim3(256), 0, st, s); break;
    }
  }
  auto t1 = std::chrono::steady_clock::now();
  C10_HIP_CHECK(hipStreamSynchronize(st));
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / (double)n;
}

}  // namespace probe
}  // namespace nbd

TORCH_LIBRARY_FRAGMENT(nbd, m) { m.def("launch_probe(Tensor dev, int n, int mode) -> float"); }
TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("launch_probe", &nbd::probe::launch_probe); }
