// copy_bw.hip — standalone HBM streaming microbenchmark for the bucket-kernel design space.
// hipcc --offload-arch=gfx950 -O3 -o copy_bw copy_bw.hip && ./copy_bw
// Variants: grid-stride float4 copy (roof), chunked (bucket-kernel shape) with unroll 1/2/4,
// non-temporal stores, persistent grid over chunks, and the fp32->bf16 casting copy.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_gridstride(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  for (; i < n4; i += st) d[i] = s[i];
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunked(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4, int64_t chunk4) {
  int64_t b = (int64_t)blockIdx.x * chunk4, e = min(b + chunk4, n4);
  int64_t i = b + threadIdx.x;
  for (; i + (U - 1) * 256 < e; i += U * 256) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], &d[i + u * 256]);
      else d[i + u * 256] = v[u];
    }
  }
  for (; i < e; i += 256) d[i] = s[i];
}

template <int U>
__global__ __launch_bounds__(256) void copy_persistent(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4, int64_t chunk4, int64_t nchunks) {
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    int64_t b = c * chunk4, e = min(b + chunk4, n4);
    int64_t i = b + threadIdx.x;
    for (; i + (U - 1) * 256 < e; i += U * 256) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = s[i + u * 256];
#pragma unroll
      for (int u = 0; u < U; ++u) d[i + u * 256] = v[u];
    }
    for (; i < e; i += 256) d[i] = s[i];
  }
}

// fp32 -> bf16 cast copy, 8 elements per lane-iteration (32 B in, 16 B out)
template <int U, bool NT>
__global__ __launch_bounds__(256) void cast_chunked(const float* __restrict__ s, uint16_t* __restrict__ d, int64_t n, int64_t chunk, float scale) {
  int64_t b = (int64_t)blockIdx.x * chunk, e = min(b + chunk, n);
  int64_t i = b + threadIdx.x * 8;
  const int64_t st = 256 * 8;
  for (; i + (U - 1) * st + 8 <= e; i += U * st) {
    f4 a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { a[u] = *(const f4*)(s + i + u * st); c[u] = *(const f4*)(s + i + u * st + 4); }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u4 w;
      for (int j = 0; j < 2; ++j) {
        __bf16 x0 = (__bf16)(a[u][2 * j] * scale), x1 = (__bf16)(a[u][2 * j + 1] * scale);
        w[j] = (uint32_t)__builtin_bit_cast(uint16_t, x0) | ((uint32_t)__builtin_bit_cast(uint16_t, x1) << 16);
        __bf16 y0 = (__bf16)(c[u][2 * j] * scale), y1 = (__bf16)(c[u][2 * j + 1] * scale);
        w[2 + j] = (uint32_t)__builtin_bit_cast(uint16_t, y0) | ((uint32_t)__builtin_bit_cast(uint16_t, y1) << 16);
      }
      if (NT) __builtin_nontemporal_store(w, (u4*)(d + i + u * st));
      else *(u4*)(d + i + u * st) = w;
    }
  }
}

template <typename F>
float timeit(F f, int iters = 20) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  std::vector<float> ts;
  for (int i = 0; i < iters; ++i) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int64_t bytes = 512ll << 20;  // 512 MiB each way (2x the Infinity Cache)
  const int64_t n4 = bytes / 16;
  f4 *s, *d;
  CHECK(hipMalloc(&s, bytes)); CHECK(hipMalloc(&d, bytes));
  CHECK(hipMemset(s, 1, bytes)); CHECK(hipMemset(d, 0, bytes));
  auto bw = [&](float ms, double moved) { return moved / (ms * 1e-3) / 1e12; };
  for (int g : {1024, 2048, 4096}) {
    float ms = timeit([&] { copy_gridstride<<<g, 256>>>(s, d, n4); });
    printf("gridstride grid=%-5d %.3f ms  %.2f TB/s\n", g, ms, bw(ms, 2.0 * bytes));
  }
  for (int64_t c4 : {1024ll, 2048ll, 4096ll, 8192ll}) {
    int64_t nb = (n4 + c4 - 1) / c4;
    float m1 = timeit([&] { copy_chunked<1, false><<<nb, 256>>>(s, d, n4, c4); });
    float m2 = timeit([&] { copy_chunked<2, false><<<nb, 256>>>(s, d, n4, c4); });
    float m4 = timeit([&] { copy_chunked<4, false><<<nb, 256>>>(s, d, n4, c4); });
    float n2 = timeit([&] { copy_chunked<2, true><<<nb, 256>>>(s, d, n4, c4); });
    float n4t = timeit([&] { copy_chunked<4, true><<<nb, 256>>>(s, d, n4, c4); });
    printf("chunked chunk=%5lld KiB blocks=%-7lld U1 %.2f  U2 %.2f  U4 %.2f  U2nt %.2f  U4nt %.2f TB/s\n",
           (long long)(c4 * 16 / 1024), (long long)nb, bw(m1, 2.0 * bytes), bw(m2, 2.0 * bytes), bw(m4, 2.0 * bytes),
           bw(n2, 2.0 * bytes), bw(n4t, 2.0 * bytes));
  }
  for (int g : {1024, 2048, 4096}) {
    int64_t c4 = 4096, nc = (n4 + c4 - 1) / c4;
    float ms = timeit([&] { copy_persistent<2><<<g, 256>>>(s, d, n4, c4, nc); });
    printf("persistent grid=%-5d chunk=64KiB U2 %.2f TB/s\n", g, bw(ms, 2.0 * bytes));
  }
  const int64_t n = bytes / 4;
  uint16_t* db = (uint16_t*)d;
  for (int64_t chunk : {8192ll, 16384ll, 32768ll, 65536ll}) {
    int64_t nb = (n + chunk - 1) / chunk;
    float m1 = timeit([&] { cast_chunked<1, false><<<nb, 256>>>((float*)s, db, n, chunk, 0.5f); });
    float m2 = timeit([&] { cast_chunked<2, false><<<nb, 256>>>((float*)s, db, n, chunk, 0.5f); });
    float m4 = timeit([&] { cast_chunked<4, false><<<nb, 256>>>((float*)s, db, n, chunk, 0.5f); });
    float n2 = timeit([&] { cast_chunked<2, true><<<nb, 256>>>((float*)s, db, n, chunk, 0.5f); });
    printf("cast f32->bf16 chunk=%6lld elems blocks=%-6lld U1 %.2f  U2 %.2f  U4 %.2f  U2nt %.2f TB/s\n",
           (long long)chunk, (long long)nb, bw(m1, 1.5 * bytes), bw(m2, 1.5 * bytes), bw(m4, 1.5 * bytes),
           bw(n2, 1.5 * bytes));
  }
  hipFree(s); hipFree(d);
  return 0;
}
