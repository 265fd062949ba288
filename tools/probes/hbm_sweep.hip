// HBM streaming micro-benchmark sweep for the diag kernels (gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/hbm_sweep.hip -o bin/hbm_sweep
// Prints one JSON object per variant: {"kernel","nt","unroll","bpc","gbps"}.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t b = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; b < n; b += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = b + u * stride;
      if (i < n) v[u] = NT ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = b + u * stride;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], &d[i]);
        else d[i] = v[u];
      }
    }
  }
}

// contiguous-chunk variant: each block owns a contiguous slab (better DRAM page locality)
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk_k(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t per_block = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t beg = static_cast<uint64_t>(blockIdx.x) * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t b = beg + threadIdx.x; b < end; b += 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = b + u * 256;
      if (i < end) v[u] = NT ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = b + u * 256;
      if (i < end) {
        if (NT) __builtin_nontemporal_store(v[u], &d[i]);
        else d[i] = v[u];
      }
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ s, uint64_t n, uint32_t* out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  uint32_t acc = 0;
  for (uint64_t b = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; b < n; b += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = b + u * stride;
      if (i < n) v[u] = NT ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
double time_ms(F f, int iters) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int i = 0; i < iters; ++i) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  uint64_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096ULL) << 20;
  uint64_t n = bytes / 16;
  u32x4 *s, *d;
  uint32_t* out;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(s, 1, bytes));
  int cus = 256;
  auto report = [&](const char* k, bool nt, int u, int bpc, double ms, double moved) {
    std::printf("{\"kernel\":\"%s\",\"nt\":%d,\"unroll\":%d,\"bpc\":%d,\"ms\":%.4f,\"gbps\":%.1f}\n", k, nt ? 1 : 0, u, bpc,
                ms, moved / (ms * 1e-3) / 1e9);
  };
#define COPY(U, NT, BPC)                                                                                       \
  report("copy", NT, U, BPC,                                                                                  \
         time_ms([&] { hipLaunchKernelGGL((copy_k<U, NT>), dim3(cus * BPC), dim3(256), 0, 0, s, d, n); }, 5), \
         2.0 * bytes)
#define CHUNK(U, NT, BPC)                                                                                           \
  report("copy_chunk", NT, U, BPC,                                                                                 \
         time_ms([&] { hipLaunchKernelGGL((copy_chunk_k<U, NT>), dim3(cus * BPC), dim3(256), 0, 0, s, d, n); }, 5), \
         2.0 * bytes)
#define READ(U, NT, BPC)                                                                                        \
  report("read", NT, U, BPC,                                                                                   \
         time_ms([&] { hipLaunchKernelGGL((read_k<U, NT>), dim3(cus * BPC), dim3(256), 0, 0, s, n, out); }, 5), \
         1.0 * bytes)
  COPY(4, true, 8); COPY(4, false, 8); COPY(8, false, 8); COPY(2, false, 8); COPY(4, false, 4);
  COPY(4, false, 16); COPY(1, false, 16); COPY(8, true, 8); COPY(2, true, 16); COPY(4, false, 2);
  CHUNK(4, false, 8); CHUNK(4, true, 8); CHUNK(8, false, 4); CHUNK(2, false, 16); CHUNK(4, false, 2);
  READ(4, true, 8); READ(4, false, 8); READ(8, false, 8); READ(8, true, 8); READ(4, false, 16); READ(16, false, 4);
  return 0;
}
